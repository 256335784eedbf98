# Interleaved A/B of builds x environments in one GPU call (devices differ by several per cent,
# so only same-call comparisons count):
#   bash tools/ab_mix.sh "final_scene1 suzanne" reps "head|" "base|" "base|RTW_LEAF_MIN=4" ...
# each case = "<variant>|<env>" (variant base = librtw.so, else librtw_<variant>.so); AB_ARGS: extra bench.py
# arguments for every run (e.g. AB_ARGS="--width 3840 --height 2160 --spp 2048")
set -o pipefail
mkdir -p gpurun_out
scenes=$1; reps=$2; shift 2
for r in $(seq 1 $reps); do
for c in "$@"; do
  v=${c%%|*}; e=${c#*|}
  lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so
  [ "$v" = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
  for s in $scenes; do
    out=$(env RTW_LIBRARY=$lib $e timeout -k 10 120 python bench.py --scene $s $AB_ARGS --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-pmc --no-first-frame --no-thread-count --no-configs 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['trace_min'], d['config'].get('kernel'))") || exit $?
    echo "$r $v [$e] $s $out" | tee -a ${AB_LOG:-gpurun_out/ab_mix.log}
  done
done
done
