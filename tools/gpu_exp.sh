# One GPU call for this session's experiments: the -m gpu suite on the product build, SAH parity of the
# inline-leaf experiment build, then interleaved A/Bs (tools/ab_mix.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_inl.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sah or scene1" -x -q --timeout 200 --timeout-method thread > gpurun_out/inl_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1" 2 "head|" "base|" "inl|" "c2u2|" "c2u4|" || exit $?
bash tools/ab_mix.sh "suzanne cornell_cube" 2 "head|" "base|" "u4|" "u8|" "base|RTW_TRACE_MIN=56" "base|RTW_TRACE_MIN=64"
