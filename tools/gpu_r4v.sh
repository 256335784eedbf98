# Round 4, call V: the in-frame tuner's epoch length (RTW_TUNE_LANES_X: epochs of at least 2 (default) / 8
# x the resident lanes' items): which threshold each run settles on and the frame rate, 4 fresh worlds each.
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_mix.sh "cornell_cube final_scene1 suzanne" 4 "base|" "base|RTW_TUNE_LANES_X=8" || exit $?
echo all-done
