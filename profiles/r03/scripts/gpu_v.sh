# Round 3 (v): full -m gpu suite, smoke and the driver's default bench command on the current code
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03v}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity')}, d['roofline']['frac'], d['roofline']['traffic'], d['placement']['first_pair_ms'], d['placement']['chosen_pair_ms'], d['k1_per_call']['ms'], d['cpu_baseline']['value'])"
