set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log gpurun_out/part10.txt
for ch in 8 16 32 64; do RTW_CHUNK=$ch bash tools/ab.sh "base" "final_scene1 suzanne cornell_cube" 1 | sed "s/^/chunk=$ch /" || exit $?; done
for ch in 8 16 32; do RTW_CHUNK=$ch timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --steps 2 | sed "s/^/chunk=$ch /" >> gpurun_out/part10.txt 2>&1 || exit $?; done
