# Round 4, call E: the -m gpu suite on the new defaults (spatial splits 0.2, guard-free triangle t,
# whole-pixel items by pixels per lane), A/Bs (4-wide walk variants; whole-pixel items on final_scene1
# and their trace_min on C5), 8-way rank shares (suzanne coop_max 4/8/16, final_scene1), the bench line.
set -o pipefail
O=gpurun_out/r4e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "final_scene1" 2 "base|RTW_TRACE_MIN=6" "base|RTW_TRACE_MIN=6 RTW_WHOLE_PIXEL=1" "q4u1|RTW_SAH4=1" "q4u3|RTW_SAH4=1" "q4ns|RTW_SAH4=1" || exit $?
B="--no-cpu-baseline --no-stats --no-pmc --no-first-frame --no-thread-count --no-configs"
for r in 1 2; do
  for env in "RTW_WHOLE_PIXEL=0" "RTW_WHOLE_PIXEL=1" "RTW_WHOLE_PIXEL=1 RTW_TRACE_MIN=16" "RTW_WHOLE_PIXEL=1 RTW_TRACE_MIN=48"; do
    echo "$r [$env] earth_motion 3840x2160x2048: $(env $env timeout -k 10 200 python bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --steps 2 --warmup 1 $B 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['trace_min'])")" >> $O/whole_ab.txt || exit $?
  done
done
for c in 4 8 16; do
  echo "[RTW_COOP_MAX=$c]" >> $O/part8.txt
  RTW_COOP_MAX=$c timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
done
timeout -k 10 300 python tools/part_bench.py --scene final_scene1 --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit $?
s=$(date +%s); timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?; e=$(date +%s); echo "bench wall $((e-s)) s" >> $O/count.txt
echo all-done
