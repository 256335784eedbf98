# Round 4, call W: the full -m gpu suite and smoke() on the round's final tree, then the PMC passes
# (tools/gpu_pmc3.sh: instruction mix, SALU share, LDS conflicts, waits) of final_scene1 and suzanne.
set -o pipefail
O=gpurun_out/r4w; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for SC in final_scene1 suzanne; do SCENE=$SC SPP=32 bash tools/gpu_pmc3.sh || exit $?; done
echo all-done
