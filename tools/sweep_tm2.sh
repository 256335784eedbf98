set -o pipefail
mkdir -p gpurun_out
run() {  # scene w h spp tm
  r=$(RTW_TRACE_MIN=$5 timeout -k 10 200 python bench.py --scene $1 --width $2 --height $3 --spp $4 --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-traffic 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'])") || exit $?
  echo "$1 tm=$5 $r" | tee -a gpurun_out/sweep_tm.log
}
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; echo rc=$? >> gpurun_out/gpu_tests.log
for tm in 12 24 32 40 48; do run suzanne 1920 1080 512 $tm; done
for tm in 12 24; do run final_scene1 1920 1080 512 $tm; done
