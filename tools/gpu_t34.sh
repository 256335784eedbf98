set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log gpurun_out/part11.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
bash tools/ab.sh "base prev" "cornell_cube final_scene1 suzanne" 1 || exit $?
timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --steps 2 >> gpurun_out/part11.txt 2>&1 || exit $?
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --steps 2 >> gpurun_out/part11.txt 2>&1 || exit $?
