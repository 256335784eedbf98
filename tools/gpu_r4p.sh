# Round 4, call P: the drain's cooperative trace only for rays that have walked RTW_COOP_AGE loop rounds
# in a dry wave (the others keep walking side by side); 0 (unset) = every drained ray, as before.
# Parity (age 8), suzanne's 8-way rank shares per age, the 1080p512 A/B.
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RTW_COOP_AGE=8 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
for a in "" 4 8 16 32; do
  echo "[RTW_COOP_AGE=$a]" >> $O/part8.txt
  RTW_COOP_AGE=$a timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
bash tools/ab_mix.sh "suzanne cornell_cube final_scene1" 2 "base|" "base|RTW_COOP_AGE=8" "base|RTW_COOP_AGE=16" || exit $?
echo all-done
