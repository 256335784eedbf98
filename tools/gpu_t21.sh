set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/part5.txt
for spp in 64 128 256 512; do
RTW_TRACE_MIN=12 timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 1,8 --spp $spp --steps 3 >> gpurun_out/part5.txt 2>&1 || exit $?
done
