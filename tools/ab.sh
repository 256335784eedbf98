# A/B experiment builds in one GPU call: bash tools/ab.sh "base old ..." "final_scene1 suzanne" [reps]
# (env passes through, e.g. RTW_TRACE_MIN=12); appends "variant scene Msamples/s ms/frame" lines
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${3:-1}); do
for v in $1; do
  for s in $2; do
    lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so
    [ "$v" = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
    r=$(RTW_LIBRARY=$lib timeout -k 10 120 python bench.py --scene $s --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-pmc --no-first-frame --no-thread-count 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['trace_min'])") || exit $?
    echo "$v $s $r" | tee -a gpurun_out/ab.log
  done
done
done
