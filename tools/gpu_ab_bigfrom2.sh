# Smaller costly prefixes (RTW_BIG_BATCH_FROM per mille): one-GPU A/B, one rank's 8-way suzanne share
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log gpurun_out/part_bf2.txt
for f in 30 60 125 250; do
  RTW_BIG_BATCH_FROM=$f bash tools/ab.sh "base" "final_scene1 cornell_cube" 2 > /dev/null || exit $?
  echo "-- above: from $f" >> gpurun_out/ab.log
  RTW_BIG_BATCH_FROM=$f timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --steps 2 2>&1 | grep -v amdgpu | sed "s/^/f$f /" >> gpurun_out/part_bf2.txt || exit $?
done
echo all-done
