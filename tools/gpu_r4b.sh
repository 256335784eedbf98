# Round 4, call B: the default bench line (with the new configs leg), GPU count without HIP, the
# self-check tests after the DevBufs change.
set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -c "import bench; print('count_gpus', bench.count_gpus())" > $O/count.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_division.py tests/test_gpu_scalar.py tests/test_gpu_node_pass.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
s=$(date +%s); timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?; e=$(date +%s); echo "bench wall $((e-s)) s" >> $O/count.txt
echo all-done
