# Bench several experiment builds: bash tools/sweep_libs.sh "b1024 b256 ..." [scenes]
set -o pipefail
mkdir -p gpurun_out
for v in $1; do
  for s in ${2:-final_scene1 suzanne}; do
    lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so
    [ "$v" = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
    r=$(RTW_LIBRARY=$lib timeout -k 10 120 python bench.py --scene $s --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-first-frame --no-thread-count 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit $?
    echo "$v $s $r" | tee -a gpurun_out/sweep.log
  done
done
