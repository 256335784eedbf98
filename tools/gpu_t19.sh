set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/part3.txt
for d in 50 10 4; do for spp in 128 512; do
RTW_TRACE_MIN=48 timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --spp $spp --steps 2 --max-depth $d >> gpurun_out/part3.txt 2>&1 || exit $?
done; done
