set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; echo tests_rc=$? >> gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stats > gpurun_out/bench.log 2>&1; echo bench_rc=$?
