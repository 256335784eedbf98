# Round 4, call M: the drain's cooperative trace with its leaf records software-pipelined (base) against
# the previous loop (librtw_nopipe.so: RTW_COOP_PIPE=0): parity, suzanne's 8-way rank shares (the drain is
# ~10 % of a share), two rays per pass over the leaves (librtw_pair.so: RTW_COOP_PAIR=1), coop_max 48, and the
# 1080p512 A/B.
set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
L=$GRAFT_REPO_ROOT/raytracinginaweekend_amd
RTW_LIBRARY=$L/librtw_pair.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tie or coop or suzanne or cornell" > $O/tests_pair.log 2>&1 || exit $?
for c in "base|" "nopipe|" "pair|" "base|RTW_COOP_MAX=48"; do
  v=${c%%|*}; e=${c#*|}; lib=$L/librtw_$v.so; [ "$v" = base ] && lib=$L/librtw.so
  echo "[$v $e]" >> $O/part8.txt
  env RTW_LIBRARY=$lib $e timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube" 2 "base|" "nopipe|" "pair|" || exit $?
echo all-done
