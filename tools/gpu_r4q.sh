# Round 4, call Q: the tuner's candidate range (6..48): final_scene1 settles at 6-8 (its low end), suzanne at
# 48 (its high end); fixed thresholds beyond both ends.
set -o pipefail
O=gpurun_out/r4q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_mix.sh "final_scene1" 2 "base|" "base|RTW_TRACE_MIN=3" "base|RTW_TRACE_MIN=4" "base|RTW_TRACE_MIN=6" || exit $?
bash tools/ab_mix.sh "suzanne" 2 "base|" "base|RTW_TRACE_MIN=48" "base|RTW_TRACE_MIN=56" "base|RTW_TRACE_MIN=64" || exit $?
echo all-done
