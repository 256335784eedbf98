# Round 4, call H: speculative stack-top reads (spop) against the product build, three worlds.
set -o pipefail
O=gpurun_out/r4h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab_mix.sh "final_scene1 suzanne cornell_cube" 2 "base|" "spop|" || exit $?
echo all-done
