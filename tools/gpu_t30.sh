set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k cost_ordered > gpurun_out/gpu_tests.log 2>&1 || exit $?
for ch in 4 8 16; do RTW_CHUNK=$ch bash tools/ab.sh "base" "final_scene1 suzanne" 1 | sed "s/^/chunk=$ch /" || exit $?; done
