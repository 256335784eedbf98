# Round 4, call D: the -m gpu suite (4-wide walk, whole-pixel items, spatial splits off by default),
# same-call A/Bs (4-wide vs two-children walk on final_scene1; spatial-split budgets on suzanne and
# cornell_cube; whole-pixel items on C5 and final_scene1), GPU count, and the default bench line.
set -o pipefail
O=gpurun_out/r4d; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -c "import bench; print('count_gpus', bench.count_gpus())" > $O/count.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1" 2 "base|" "base|RTW_SAH4=1" "w5|" "w5|RTW_SAH4=1" || exit $?
bash tools/ab_mix.sh "suzanne" 2 "base|" "base|RTW_SAH_SPLIT_BUDGET=0.1" "base|RTW_SAH_SPLIT_BUDGET=0.2" "base|RTW_SAH_SPLIT_BUDGET=0.3" || exit $?
bash tools/ab_mix.sh "cornell_cube" 1 "base|" "base|RTW_SAH_SPLIT_BUDGET=0.2" "tmk|" || exit $?
bash tools/ab_mix.sh "suzanne" 2 "tmk|" || exit $?
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_tmk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -k "suzanne or cornell or tie" --timeout 200 --timeout-method thread > $O/tmk_tests.log 2>&1 || exit $?
RTW_SAH_SPLIT_BUDGET=0.2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "sah or suzanne or cornell or tie" --timeout 200 --timeout-method thread > $O/split_tests.log 2>&1 || exit $?
B="--no-cpu-baseline --no-stats --no-pmc --no-first-frame --no-thread-count --no-configs"
for r in 1 2; do
  for env in "RTW_TRACE_MIN=40" "RTW_TRACE_MIN=40 RTW_WHOLE_PIXEL=1"; do
    echo "$r [$env] earth_motion 3840x2160x2048: $(env $env timeout -k 10 200 python bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --steps 2 --warmup 1 $B 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> $O/whole_ab.txt || exit $?
  done
done
s=$(date +%s); timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?; e=$(date +%s); echo "bench wall $((e-s)) s" >> $O/count.txt
for s in final_scene1 earth_motion suzanne; do
  RTW_SAH4=1 RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_pt.so timeout -k 10 120 python tools/phase_timing.py --scene $s --spp 128 >> $O/phase.txt 2>&1 || exit $?
done
echo all-done
