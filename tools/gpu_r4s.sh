# Round 4, call S: SAH nodes with one leaf child hold it on the left (RTW_SAH_LEAF_LEFT=1): parity, then the
# 1080p512 A/B.
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RTW_SAH_LEAF_LEFT=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or c1 or sampled" > $O/tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube" 3 "base|" "base|RTW_SAH_LEAF_LEFT=1" || exit $?
echo all-done
