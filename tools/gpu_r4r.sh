# Round 4, call R: steps per exit check re-measured on the round's closing kernel: the two-children walk
# (RTW_C2_UNROLL 2 / 3 default / 4: final_scene1) and the one-child walk (RTW_TRAV_UNROLL 4 / 6 default / 8:
# suzanne, cornell_cube).
set -o pipefail
O=gpurun_out/r4r; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_mix.sh "final_scene1" 2 "base|" "c2u2|" "c2u4|" || exit $?
bash tools/ab_mix.sh "suzanne cornell_cube" 2 "base|" "tu4|" "tu8|" || exit $?
echo all-done
