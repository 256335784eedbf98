# Round-end measurement set: default bench line (with CPU baseline + PMC traffic), the rocprofv3
# kernel-trace summary of the same bench command, and the suzanne config line.
set -o pipefail
mkdir -p gpurun_out/round
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/round/bench_default.json 2> gpurun_out/round/bench_default.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/round/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-traffic > gpurun_out/round/kt_bench.json 2> gpurun_out/round/kt.err || exit $?
timeout -k 10 600 python bench.py --scene suzanne --no-cpu-baseline > gpurun_out/round/bench_suzanne.json 2> gpurun_out/round/bench_suzanne.err || exit $?
echo done
