# Round 3 (e): the whole GPU suite, then the drop-in call-surface rates (per call, batched round)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03e}; mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1; rc=$?
tail -5 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR" $OUT/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/percall_profile.py 300 > $OUT/percall.log 2>&1 && head -3 $OUT/percall.log | grep aggregate
timeout -k 10 600 python tools/dropin_rate.py 5 > $OUT/dropin.log 2>&1; grep '^{' $OUT/dropin.log
