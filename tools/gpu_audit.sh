# Audit builds, made first (here, in-tree): RTW_VARIANT_FLAGS=-DRTW_SAH_AUDIT_NO_TIE bash tools/build_variant.sh notie,
# and the same with -DRTW_SAH_AUDIT_NO_BOX as nobox (tools/build_variant.sh): the SAH walk's
# tie test and leaf-box proof switched off.  The parity tests that exercise them must FAIL on these
# libraries (a failure is the expected result: it shows that the switch decides pixels).  Run through
# gpurun; output: gpurun_out/audit/.
set -o pipefail
O=gpurun_out/audit; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in notie nobox; do
  RTW_LIBRARY=$GRAFT_REPO_ROOT/raytracinginaweekend_amd/librtw_$v.so timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread \
    -k "tie or sah_tree_agrees or split or wrapped or rolling" > $O/$v.log 2>&1
  rc=$?
  echo "$v: pytest exit $rc ($(tail -1 $O/$v.log))" | tee -a $O/summary.txt
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1   # a time limit ends the call
done
exit 0
