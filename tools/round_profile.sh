# Round-end measurement set (one GPU): default bench line (C2, with CPU baseline + PMC traffic),
# the rocprofv3 kernel-trace summary of the same bench command, and the other BASELINE configs
# on one GPU: C4 suzanne 1080p512, C3 cornell_cube 800x800x1024, C5 earth_motion 3840x2160x2048.
set -o pipefail
mkdir -p gpurun_out/round
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > gpurun_out/round/bench_default.json 2> gpurun_out/round/bench_default.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/round/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-traffic > gpurun_out/round/kt_bench.json 2> gpurun_out/round/kt.err || exit $?
timeout -k 10 600 python bench.py --scene suzanne --no-cpu-baseline > gpurun_out/round/bench_suzanne.json 2> gpurun_out/round/bench_suzanne.err || exit $?
timeout -k 10 600 python bench.py --scene cornell_cube --width 800 --height 800 --spp 1024 --no-cpu-baseline > gpurun_out/round/bench_cornell_cube.json 2> gpurun_out/round/bench_cornell_cube.err || exit $?
timeout -k 10 900 python bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --steps 2 --no-cpu-baseline > gpurun_out/round/bench_earth_motion.json 2> gpurun_out/round/bench_earth_motion.err || exit $?
echo done
