# Round 4's closing measurement set on one MI355X -> gpurun_out/${ROUND_TAG:-r4final}/:
#   the full -m gpu suite, smoke(), the default bench line (C2 headline with its CPU baseline, PMC
#   roofline and HBM traffic, plus the configs leg: C4 suzanne, C3 cornell_cube, C5 earth_motion), the
#   rocprofv3 kernel-trace summary of the headline bench command, and one rank's share of 8-GPU splits.
set -o pipefail
O=gpurun_out/${ROUND_TAG:-r4final}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-configs > $O/kt_bench.json 2> $O/kt.err || exit $?
rm -f $O/part8.txt
for s in final_scene1 suzanne; do
  timeout -k 10 300 python tools/part_bench.py --scene $s --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
echo all-done
