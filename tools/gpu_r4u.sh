# Round 4, call U: leaf pairs in the one-child SAH walk (librtw_lp.so: RTW_LEAF_PAIRS=1; a node step whose
# children are both leaves stands on the pair and one leaf step tests both): parity, then suzanne and
# cornell_cube at 1080p512.
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_lp.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "suzanne cornell_cube" 3 "base|" "lp|" || exit $?
echo all-done
