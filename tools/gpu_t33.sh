set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
for ch in 8 32 64; do
RTW_CHUNK=$ch RTW_TRACE_MIN=6 bash tools/ab.sh "base" "final_scene1" 1 | sed "s/^/chunk=$ch tm=6 /" || exit $?
RTW_CHUNK=$ch RTW_TRACE_MIN=40 bash tools/ab.sh "base" "suzanne" 1 | sed "s/^/chunk=$ch tm=40 /" || exit $?
done
