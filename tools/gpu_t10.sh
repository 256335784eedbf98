set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_b1024.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stats.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base prev b1024" "suzanne" 1 || exit $?
RTW_LDS_MODE=1 RTW_TRACE_MIN=48 bash tools/ab.sh "b1024" "suzanne" 1 || exit $?
RTW_TRACE_MIN=12 bash tools/ab.sh "base b1024" "final_scene1" 1 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base prev b1024" "suzanne" 1 || exit $?
