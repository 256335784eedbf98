set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for sc in final_scene1 suzanne; do
  timeout -k 10 200 python bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/bench_$sc.json 2>gpurun_out/bench_$sc.err || exit $?
done
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/bench_final_scene1_b.json 2>&1 || exit $?
timeout -k 10 200 python tools/exec_counters.py --scenes final_scene1,suzanne > gpurun_out/exec.txt 2>&1
