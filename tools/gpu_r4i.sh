# Round 4, call I: the SAH node test with the margin in space (smar, constants x9/8): its containment of
# the exact cull on the device, the parity suite on it, and the A/B against the product build.
set -o pipefail
O=gpurun_out/r4i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_smar.so timeout -k 10 400 python -u -m pytest tests/test_gpu_node_pass.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/smar_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube" 2 "base|" "smar|" || exit $?
echo all-done
