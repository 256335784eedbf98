set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
RTW_TRACE_MIN=12 bash tools/ab.sh "base old" "final_scene1" 2 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base old" "suzanne" 1 || exit $?
timeout -k 10 300 python tools/exec_counters.py --scenes final_scene1,suzanne --width 1920 --height 1080 --spp 32 > gpurun_out/exec.txt 2>&1
