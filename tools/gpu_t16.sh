set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
RTW_TRACE_MIN=12 bash tools/ab.sh "base pv10 pv30 plds" "final_scene1" 1 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base pv10 pv30 plds" "suzanne" 1 || exit $?
