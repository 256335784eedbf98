set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
for ch in 8 64; do for tm in 6 32; do
RTW_CHUNK=$ch RTW_TRACE_MIN=$tm bash tools/ab.sh "base" "cornell_cube" 1 | sed "s/^/chunk=$ch tm=$tm /" || exit $?
RTW_NO_REORDER=1 RTW_CHUNK=$ch RTW_TRACE_MIN=$tm bash tools/ab.sh "base" "cornell_cube" 1 | sed "s/^/noreorder chunk=$ch tm=$tm /" || exit $?
done; done
