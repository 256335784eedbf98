# Round 4, call N: the drain's cooperative trace with each lane's leaf tests bounded by te = succ(its best
# so far) (base) against te = inf (librtw_note.so: RTW_COOP_TE=0): parity, suzanne's 8-way rank shares,
# the 1080p512 A/B.
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
L=$GRAFT_REPO_ROOT/raytracinginaweekend_amd
for c in "base|" "note|"; do
  v=${c%%|*}; e=${c#*|}; lib=$L/librtw_$v.so; [ "$v" = base ] && lib=$L/librtw.so
  echo "[$v $e]" >> $O/part8.txt
  env RTW_LIBRARY=$lib $e timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube" 2 "base|" "note|" || exit $?
echo all-done
