# Round 2: full GPU suite, then the drop-in rate (no-op training).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u tools/dropin_rate.py 5 > $OUT/dropin.log 2>&1 || { echo DROPIN FAILED; tail -30 $OUT/dropin.log; exit 1; }
grep '^{' $OUT/dropin.log
echo EXIT 0
