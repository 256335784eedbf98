set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 > gpurun_out/part.txt 2>&1 || exit $?
timeout -k 10 300 python tools/part_bench.py --scene suzanne >> gpurun_out/part.txt 2>&1
