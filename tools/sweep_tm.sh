# trace_min sweep over configs: bash tools/sweep_tm.sh
set -o pipefail
mkdir -p gpurun_out
run() {  # scene w h spp tm
  r=$(RTW_TRACE_MIN=$5 timeout -k 10 200 python bench.py --scene $1 --width $2 --height $3 --spp $4 --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-traffic 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'])") || exit $?
  echo "$1 tm=$5 $r" | tee -a gpurun_out/sweep_tm.log
}
for tm in 12 24 40 48; do run cornell_cube 800 800 1024 $tm; done
for tm in 12 24 40 48; do run earth_motion 1080 1920 256 $tm; done
for tm in 12 24 40 48; do run final_scene2 1080 1080 128 $tm; done
