set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do for s in final_scene1 suzanne; do
timeout -k 10 120 python bench.py --scene $s --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-traffic > gpurun_out/c.out 2> gpurun_out/c_err.txt || exit $?
echo "$s $(grep -o '"value": [0-9.]*' gpurun_out/c.out) $(grep -o '"trace_min": [0-9]*' gpurun_out/c.out)" >> gpurun_out/calib.log
done; done
