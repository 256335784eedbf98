set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.log
RTW_TRACE_MIN=12 bash tools/ab.sh "base prev psq" "final_scene1" 2 || exit $?
