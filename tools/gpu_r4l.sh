# Round 4, call L: parity of the product build (proof boxes in LDS, whole-pixel threshold 16), then the
# wave-timing build's frame tails: suzanne 1080p512 whole frame and one 8-way share, final_scene1 share.
set -o pipefail
O=gpurun_out/r4l; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
W=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_wt.so
RTW_LIBRARY=$W timeout -k 10 200 python tools/wave_timing.py --scene suzanne --spp 512 > $O/wt.txt 2>&1 || exit $?
RTW_LIBRARY=$W timeout -k 10 200 python tools/wave_timing.py --scene suzanne --spp 512 --parts 8 --rank 3 >> $O/wt.txt 2>&1 || exit $?
RTW_LIBRARY=$W timeout -k 10 200 python tools/wave_timing.py --scene final_scene1 --spp 512 --parts 8 --rank 0 >> $O/wt.txt 2>&1 || exit $?
RTW_LIBRARY=$W timeout -k 10 200 python tools/wave_timing.py --scene final_scene1 --spp 512 >> $O/wt.txt 2>&1 || exit $?
echo all-done
