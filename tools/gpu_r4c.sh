# Round 4, call C: GPU count without HIP, the -m gpu suite (DevBufs, whole-pixel items), the default
# bench line with the configs leg, and the whole-pixel A/B (C5 4Kx2048 and final_scene1 1080p512, plus
# an 8-way rank share of C5).
set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -c "import bench; print('count_gpus', bench.count_gpus())" > $O/count.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
s=$(date +%s); timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?; e=$(date +%s); echo "bench wall $((e-s)) s" >> $O/count.txt
B="--no-cpu-baseline --no-stats --no-pmc --no-first-frame --no-thread-count --no-configs"
for r in 1 2; do
  for env in "RTW_TRACE_MIN=40" "RTW_TRACE_MIN=40 RTW_WHOLE_PIXEL=1" "RTW_TRACE_MIN=16 RTW_WHOLE_PIXEL=1"; do
    echo "$r [$env] earth_motion 3840x2160x2048: $(env $env timeout -k 10 200 python bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --steps 2 --warmup 1 $B 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> $O/whole_ab.txt || exit $?
  done
  for env in "RTW_TRACE_MIN=6" "RTW_TRACE_MIN=6 RTW_WHOLE_PIXEL=1" "RTW_TRACE_MIN=16 RTW_WHOLE_PIXEL=1"; do
    echo "$r [$env] final_scene1 1920x1080x512: $(env $env timeout -k 10 200 python bench.py --steps 2 --warmup 1 $B 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" >> $O/whole_ab.txt || exit $?
  done
done
for env in "RTW_TRACE_MIN=40" "RTW_TRACE_MIN=40 RTW_WHOLE_PIXEL=1"; do
  echo "[$env]" >> $O/whole_part8.txt
  env $env timeout -k 10 300 python tools/part_bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --parts 8 --steps 1 >> $O/whole_part8.txt 2>&1 || exit $?
done
echo all-done
