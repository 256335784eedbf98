set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash tools/ab.sh "base prev" "final_scene1 suzanne" 2 || exit $?
