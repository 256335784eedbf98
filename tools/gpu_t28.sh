set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log gpurun_out/part9.txt
bash tools/ab.sh "base" "final_scene1 suzanne cornell_cube" 1 || exit $?
RTW_TRACE_MIN=6 bash tools/ab.sh "base" "final_scene1" 1 | sed "s/^/tm=6 /" || exit $?
RTW_TRACE_MIN=12 bash tools/ab.sh "base" "final_scene1" 1 | sed "s/^/tm=12 /" || exit $?
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --steps 2 >> gpurun_out/part9.txt 2>&1 || exit $?
