# Round-end set: -m gpu tests, smoke(), tools/round_profile.sh, and one rank's 8-way share
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/part8.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
bash tools/round_profile.sh || exit $?
for s in final_scene1 suzanne; do
  timeout -k 10 300 python tools/part_bench.py --scene $s --parts 8 --steps 2 >> gpurun_out/part8.txt 2>&1 || exit $?
done
echo all-done
