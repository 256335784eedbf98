# Round 4, call X: the two-children step's take() under the hit predicate as selects, no branch around it
# (librtw_ts.so: RTW_TAKE_SEL=1): parity, then final_scene1 1080p512.
set -o pipefail
O=gpurun_out/r4x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_ts.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1" 4 "base|" "ts|" || exit $?
echo all-done
