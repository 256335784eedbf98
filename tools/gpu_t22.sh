set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/part6.txt
for tm in 12 16 24 32 48; do
RTW_TRACE_MIN=$tm timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --steps 3 | sed "s/^/tm=$tm /" >> gpurun_out/part6.txt 2>&1 || exit $?
done
for r in 1 2 3; do
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --steps 2 | sed "s/^/tuned run $r /" >> gpurun_out/part6.txt 2>&1 || exit $?
done
