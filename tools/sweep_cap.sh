set -o pipefail
mkdir -p gpurun_out
run() {  # scene cap
  r=$(RTW_TRACE_MIN=12 RTW_WAIT_CAP=$2 timeout -k 10 200 python bench.py --scene $1 --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-traffic 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'])") || exit $?
  echo "$1 cap=$2 $r" | tee -a gpurun_out/sweep_cap.log
}
for c in 8 16 32 64 128; do run suzanne $c; run final_scene1 $c; done
