set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests3.log 2>&1; echo tests_rc=$? >> gpurun_out/gpu_tests3.log
for tm in 0 16 32 40 48 56; do
  RTW_TRACE_MIN=$tm timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stats > gpurun_out/sweep_$tm.log 2>&1 || break
  echo "tm=$tm $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$tm.log)" >> gpurun_out/sweep.txt
done
echo done
