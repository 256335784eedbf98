# Round-end measurement set on one MI355X -> gpurun_out/$ROUND_TAG/ (default r03):
#   -m gpu tests, smoke(), the default bench line (C2: CPU baseline, PMC roofline, HBM traffic),
#   the rocprofv3 kernel-trace summary of the same bench command, the other BASELINE configs on one
#   GPU (C4 suzanne, C3 cornell_cube, C5 earth_motion), one rank's share of 8-GPU splits, and
#   PMC passes of the render kernel (all four configs).
set -o pipefail
O=gpurun_out/${ROUND_TAG:-r03}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc > $O/kt_bench.json 2> $O/kt.err || exit $?
timeout -k 10 600 python bench.py --scene suzanne --no-cpu-baseline > $O/bench_suzanne.json 2> $O/bench_suzanne.err || exit $?
timeout -k 10 600 python bench.py --scene cornell_cube --width 800 --height 800 --spp 1024 --no-cpu-baseline > $O/bench_cornell_cube.json 2> $O/bench_cornell_cube.err || exit $?
timeout -k 10 900 python bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --steps 2 --no-cpu-baseline > $O/bench_earth_motion.json 2> $O/bench_earth_motion.err || exit $?
rm -f $O/part8.txt
for s in final_scene1 suzanne; do
  timeout -k 10 300 python tools/part_bench.py --scene $s --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
timeout -k 10 300 python tools/part_bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --parts 8 --steps 1 >> $O/part8.txt 2>&1 || exit $?
for SC in final_scene1 suzanne; do SCENE=$SC SPP=32 bash tools/gpu_pmc3.sh || exit $?; done
SCENE=cornell_cube W=800 H=800 SPP=128 bash tools/gpu_pmc3.sh || exit $?
SCENE=earth_motion W=3840 H=2160 SPP=32 bash tools/gpu_pmc3.sh || exit $?
echo all-done
