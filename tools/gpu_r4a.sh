# Round 4, call A: the -m gpu suite on the product build, smoke, same-call A/B of HEAD (librtw_head.so)
# against the product build on the four BASELINE worlds, the r4 phase split (librtw_pt.so) and
# WRITE_SIZE passes of head and base on suzanne / cornell_cube.
set -o pipefail
O=gpurun_out/r4a; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube earth_motion" 2 "head|" "base|" || exit $?
for s in final_scene1 suzanne cornell_cube; do
  RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_pt.so timeout -k 10 120 python tools/phase_timing.py --scene $s --spp 128 >> $O/phase.txt 2>&1 || exit $?
done
for v in head base; do
  lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so; [ $v = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
  for s in suzanne cornell_cube; do
    RTW_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_${v}_$s -o w --output-format csv -- python3 tools/prof_render.py --scene $s --spp 64 --repeat 2 > $O/w_${v}_$s.log 2>&1 || exit $?
  done
done
echo all-done
