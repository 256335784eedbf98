# One GPU call: the -m gpu suite (division self-checks first), then an interleaved A/B of the
# committed kernel (librtw_head.so, tools/build_head_variant.sh) against the working tree (base).
#   bash tools/gpu_check_ab.sh "final_scene1 suzanne" reps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_division.py -x -v --timeout 200 --timeout-method thread > gpurun_out/div_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "${1:-final_scene1 suzanne cornell_cube earth_motion}" ${2:-2} "head|" "base|"
