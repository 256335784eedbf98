set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_l16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
RTW_TRACE_MIN=12 bash tools/ab.sh "base old l8 l16 l24" "final_scene1" 1 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base old l8 l16 l24" "suzanne" 1 || exit $?
RTW_TRACE_MIN=12 bash tools/ab.sh "base l16" "final_scene1" 1 || exit $?
