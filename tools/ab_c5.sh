set -o pipefail
for v in ${VARIANTS:-head base head base}; do
  lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so; [ $v = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
  RTW_LIBRARY=$lib timeout -k 10 300 python bench.py --scene earth_motion --width 3840 --height 2160 --spp 2048 --steps 2 --warmup 1 --no-cpu-baseline --no-stats --no-pmc --no-first-frame 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/c5.log || exit 1
done
