set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
for tm in 6 8 10 12; do RTW_TRACE_MIN=$tm bash tools/ab.sh "base" "final_scene1" 1 | sed "s/^/tm=$tm /" || exit $?; done
for tm in 40 48 56 64; do RTW_TRACE_MIN=$tm bash tools/ab.sh "base" "suzanne" 1 | sed "s/^/tm=$tm /" || exit $?; done
for tm in 8 12 16 24; do RTW_TRACE_MIN=$tm bash tools/ab.sh "base" "cornell_cube" 1 | sed "s/^/tm=$tm /" || exit $?; done
