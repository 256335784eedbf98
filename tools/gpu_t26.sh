set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for v in base prev base prev; do
RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so
[ "$v" = base ] && RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
r=$(RTW_LIBRARY=$RTW_LIBRARY timeout -k 10 120 python bench.py --scene cornell_cube --width 800 --height 800 --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-stats 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['trace_min'])") || exit $?
echo "$v cornell_cube $r" | tee -a gpurun_out/ab.log
done
