set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/part7.txt
for r in 1 2; do
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 1,8 --steps 2 | sed "s/^/run $r /" >> gpurun_out/part7.txt 2>&1 || exit $?
timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 1,8 --steps 2 | sed "s/^/run $r /" >> gpurun_out/part7.txt 2>&1 || exit $?
done
timeout -k 10 300 python tools/part_bench.py --scene cornell_cube --width 800 --height 800 --spp 1024 --parts 1,8 --steps 2 >> gpurun_out/part7.txt 2>&1 || exit $?
