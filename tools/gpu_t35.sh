set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log gpurun_out/part12.txt
bash tools/ab.sh "base b64k8 b64k32 b256k32 b128k16" "final_scene1 suzanne cornell_cube" 1 || exit $?
for v in base b64k8 b64k32 b256k32 b128k16; do
lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so; [ "$v" = base ] && lib=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw.so
RTW_LIBRARY=$lib RTW_TRACE_MIN=40 timeout -k 10 300 python tools/part_bench.py --scene suzanne --parts 8 --steps 2 | sed "s/^/$v /" >> gpurun_out/part12.txt 2>&1 || exit $?
done
