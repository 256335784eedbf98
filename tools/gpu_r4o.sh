# Round 4, call O: the phase split of the round's closing build (librtw_pt.so) and of the same source drawing
# through rtw_scalar.h (librtw_pto.so: RTW_DEV_RNG=0), 1920x1080x128.
set -o pipefail
O=gpurun_out/r4o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in pt pto; do
  for s in final_scene1 suzanne cornell_cube; do
    echo "[$v]" >> $O/phase.txt
    RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so timeout -k 10 120 python tools/phase_timing.py --scene $s --spp 128 >> $O/phase.txt 2>&1 || exit $?
  done
done
echo all-done
