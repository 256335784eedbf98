# Round 4, call T: leaf bodies on every third step of the one-child walk in triangle worlds (librtw_lc3.so:
# RTW_LEAF_CADENCE=3) against every other step (base), suzanne 1080p512.
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_lc3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "suzanne or tie or mesh" > $O/tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "suzanne" 3 "base|" "lc3|" || exit $?
echo all-done
