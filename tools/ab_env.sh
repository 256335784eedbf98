# A/B of one build under several environments, in one GPU call:
#   bash tools/ab_env.sh "final_scene1 suzanne" "RTW_NO_PARK=1" "RTW_PARK_SWAP=4" ...
# (an empty string = the defaults); appends "env scene Msamples/s ms/frame trace_min" lines
set -o pipefail
mkdir -p gpurun_out
scenes=$1; shift
for e in "$@"; do
  for s in $scenes; do
    r=$(env $e timeout -k 10 120 python bench.py --scene $s --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-pmc --no-first-frame --no-thread-count 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['trace_min'])") || exit $?
    echo "[${e:-default}] $s $r" | tee -a gpurun_out/ab_env.log
  done
done
