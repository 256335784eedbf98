set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_node_pass.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
RTW_TRACE_MIN=12 bash tools/ab.sh "base prev ilp" "final_scene1" 2 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base prev ilp" "suzanne" 1 || exit $?
