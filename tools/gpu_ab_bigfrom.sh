# Costly-prefix batch rule: parity (cost-ordered frames), one-GPU A/B against HEAD (prev) over the
# prefix fraction RTW_BIG_BATCH_FROM (per mille), one rank's 8-way share
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log gpurun_out/part_bf.txt
for f in 1 250; do
  RTW_BIG_BATCH_FROM=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k cost_ordered --timeout 200 --timeout-method thread > gpurun_out/bf_tests_$f.log 2>&1 || exit $?
done
bash tools/ab.sh "prev" "final_scene1 suzanne cornell_cube" 1 || exit $?
for f in 1 125 250 500; do
  RTW_BIG_BATCH_FROM=$f bash tools/ab.sh "base" "final_scene1 suzanne cornell_cube" 1 || exit $?
  echo "-- above: from $f" >> gpurun_out/ab.log
done
for cfg in prev:250 base:1 base:125 base:250 base:500; do
  v=${cfg%%:*}; f=${cfg##*:}
  lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so; [ "$v" = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
  RTW_BIG_BATCH_FROM=$f RTW_LIBRARY=$lib timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --steps 2 2>&1 | grep -v amdgpu | sed "s/^/$v f$f /" >> gpurun_out/part_bf.txt || exit $?
done
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --steps 2 2>&1 | grep -v amdgpu | sed "s/^/base f250 /" >> gpurun_out/part_bf.txt || exit $?
echo all-done
