set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/part2.txt
for spp in 128 256 512 1024; do
timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --spp $spp --steps 2 >> gpurun_out/part2.txt 2>&1 || exit $?
done
for spp in 128 512; do
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --spp $spp --steps 2 >> gpurun_out/part2.txt 2>&1 || exit $?
done
