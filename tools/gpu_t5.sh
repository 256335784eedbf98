set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
RTW_TRACE_MIN=12 bash tools/ab.sh "base b384" "final_scene1" 2 || exit $?
RTW_TRACE_MIN=48 bash tools/ab.sh "base b384" "suzanne" 1 || exit $?
for tm in 8 16 24; do RTW_TRACE_MIN=$tm bash tools/ab.sh "b384" "final_scene1" 1 || exit $?; done
