# Sweep one env knob of the render kernel: bash tools/sweep_env.sh VAR "v1 v2 ..." [scene]
set -o pipefail
mkdir -p gpurun_out
VAR=$1; VALS=$2; SCENE=${3:-final_scene1}
for v in $VALS; do
  r=$(env $VAR=$v timeout -k 10 120 python bench.py --scene $SCENE --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-first-frame --no-thread-count 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit $?
  echo "$SCENE $VAR=$v $r" | tee -a gpurun_out/sweep.log
done
