# One parametrised GPU runner (replaces round 4's one-shot tools/gpu_r4*.sh).  Run it through gpurun:
#   gpurun -- 'TAG=r5a bash tools/gpu_run.sh tests:parity smoke bench'
# Each argument is a step, run in order, each under its own time limit; the first failing step ends
# the call (no retries).  Output: gpurun_out/$TAG/.
#   tests[:EXPR]      pytest -m gpu (EXPR: a -k expression; "all" or none: the full suite)
#   files:F1,F2[:EXPR] pytest -m gpu on the given test files
#   smoke             __graft_entry__.smoke()
#   bench[:ARGS]      python bench.py ARGS (commas become spaces) -> bench_<n>.json
#   kt                rocprofv3 kernel-trace summary of the headline bench command -> kt/
#   part8[:SCENES]    one rank's share of 8-way splits (tools/part_bench.py), default final_scene1,suzanne
#   pmc:SCENE[:W:H:SPP]  the PMC counter passes of tools/gpu_pmc3.sh for one scene
#   env:VAR=VALUE / unenv:VAR  set / unset an environment variable for the steps that follow
#   py:SCRIPT[,ARGS]  python SCRIPT ARGS (commas become spaces) -> py_<n>.txt
#   ab:SCENES:REPS:CASE1;CASE2..  tools/ab_mix.sh (cases "<variant>|<env>"; SCENES comma-separated);
#                     AB_ARGS passes extra bench.py arguments
set -o pipefail
O=gpurun_out/${TAG:-run}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
nb=0
nf=0
np_=0
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  echo "== $step ($(date +%T))" | tee -a $O/steps.log
  case $kind in
    tests)
      if [ -z "$rest" ] || [ "$rest" = all ]; then K=(); else K=(-k "$rest"); fi
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; } ;;
    files)
      nf=$((nf + 1))
      f=${rest%%:*}; e=${rest#*:}; [ "$e" = "$rest" ] && e=""
      if [ -z "$e" ]; then K=(); else K=(-k "$e"); fi
      timeout -k 10 1100 python -u -m pytest ${f//,/ } -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > $O/gpu_tests_files_$nf.log 2>&1 || { tail -30 $O/gpu_tests_files_$nf.log; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1 ;;
    bench)
      nb=$((nb + 1))
      timeout -k 10 900 python bench.py ${rest//,/ } > $O/bench_$nb.json 2> $O/bench_$nb.err || { tail -20 $O/bench_$nb.err; exit 1; } ;;
    kt)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py \
        --no-cpu-baseline --no-pmc --no-configs > $O/kt_bench.json 2> $O/kt.err || exit 1 ;;
    part8)
      for s in $(echo ${rest:-final_scene1,suzanne} | tr , ' '); do
        timeout -k 10 300 python tools/part_bench.py --scene $s --parts 8 --ranks all --steps 2 >> $O/part8.txt 2>&1 || exit 1
      done ;;
    pmc)
      IFS=: read -r sc w h spp <<< "$rest"
      SCENE=$sc W=${w:-1920} H=${h:-1080} SPP=${spp:-32} PMC_OUT=$O/pmc_$sc bash tools/gpu_pmc3.sh || exit 1 ;;
    env)
      export "$rest" ;;  # for the steps that follow, e.g. env:RTW_COOP_MAX=8
    unenv)
      unset "$rest" ;;
    py)
      np_=$((np_ + 1))
      timeout -k 10 900 python ${rest//,/ } > $O/py_$np_.txt 2>&1 || { tail -20 $O/py_$np_.txt; exit 1; } ;;
    ab)
      IFS=: read -r sc reps cases <<< "$rest"
      IFS=';' read -r -a C <<< "$cases"
      AB_LOG=$O/ab_mix.log bash tools/ab_mix.sh "${sc//,/ }" $reps "${C[@]}" || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo all-done | tee -a $O/steps.log
