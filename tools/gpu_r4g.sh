# Round 4, call G: the -m gpu suite (leaf-indexed triangle records, coop_max 32), A/Bs (leaf-indexed vs
# triangle-indexed records on suzanne / cornell_cube; coop_max 32 vs 4 on final_scene1 / earth_motion;
# the two-children step without branches (c2bl) and with 2 / 4 steps per exit check).
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
bash tools/ab_mix.sh "suzanne cornell_cube" 2 "base|" "tbl0|" || exit $?
bash tools/ab_mix.sh "final_scene1 earth_motion" 2 "base|" "base|RTW_COOP_MAX=4" || exit $?
bash tools/ab_mix.sh "final_scene1" 2 "base|" "c2bl|" "c2u2|" "c2u4|" || exit $?
echo all-done
