# Round 4, call K: the SAH proof boxes in LDS (RTW_NO_PROOF_LDS=1: HBM / L2) and the per-lane tile_perm
# cache (librtw_nopc.so: RTW_PERM_CACHE=0), parity first; then the whole-pixel C5 frame's fixed
# dynamic-fetch threshold (no tuning there) at 8 / 16 / 32 (default) / 48.
set -o pipefail
O=gpurun_out/r4k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube earth_motion" 2 "base|" "base|RTW_NO_PROOF_LDS=1" "nopc|" || exit $?
AB_ARGS="--width 3840 --height 2160 --spp 2048" bash tools/ab_mix.sh "earth_motion" 1 "base|" "base|RTW_TRACE_MIN=8" "base|RTW_TRACE_MIN=16" "base|RTW_TRACE_MIN=48" || exit $?
echo all-done
