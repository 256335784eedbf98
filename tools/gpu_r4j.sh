# Round 4, call J: the gfx950-written RNG draws (d_next_u64 / d_m1_1 / d_unit_*): parity on the image
# suites, then the A/B against the same source drawing through rtw_scalar.h (librtw_orng.so).
set -o pipefail
O=gpurun_out/r4j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube earth_motion" 2 "base|" "orng|" || exit $?
bash tools/ab_mix.sh "final_scene1 suzanne" 2 "base|RTW_CHUNK=2" "base|RTW_CHUNK=4" || exit $?
echo all-done
