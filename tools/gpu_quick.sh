# Quick GPU check: parity tests, then short benches (final_scene1 and suzanne at 1080p512).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-stats > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --scene suzanne --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-stats >> gpurun_out/bench.log 2>&1
