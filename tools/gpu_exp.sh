# One GPU call for this session's experiments: the -m gpu suite on the product build, parity of an
# experiment build (EXP, default c1i) on the SAH and mesh worlds, interleaved A/Bs (tools/ab_mix.sh),
# and a PMC pass of suzanne.
set -o pipefail
mkdir -p gpurun_out
EXP=${EXP:-c1i}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$EXP.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sah or suzanne or cornell" -x -q --timeout 200 --timeout-method thread > gpurun_out/exp_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1" 2 "base|" "c2u2|" "c2u4|" "c2u6|" || exit $?
bash tools/ab_mix.sh "suzanne cornell_cube" 2 "base|" "$EXP|" || exit $?
SCENE=suzanne SPP=32 bash tools/gpu_pmc3.sh
