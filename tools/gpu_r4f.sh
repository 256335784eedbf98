# Round 4, call F: the -m gpu suite (4-wide walk removed, packed two-children walk, per-pixel cost in
# whole-pixel frames), A/Bs (packed vs unpacked two-children walk; the drain's coop_max on suzanne, one
# GPU and 8-way shares), the bench line.
set -o pipefail
O=gpurun_out/r4f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1" 3 "base|" "c2np|" || exit $?
bash tools/ab_mix.sh "suzanne cornell_cube" 2 "base|" "base|RTW_COOP_MAX=16" "base|RTW_COOP_MAX=32" || exit $?
for c in 16 32; do
  echo "[RTW_COOP_MAX=$c]" >> $O/part8.txt
  RTW_COOP_MAX=$c timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
s=$(date +%s); timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?; e=$(date +%s); echo "bench wall $((e-s)) s" >> $O/count.txt
echo all-done
