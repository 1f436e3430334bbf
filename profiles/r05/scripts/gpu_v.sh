# Round 5 validation (v): full -m gpu suite, smoke, the driver's default bench command, and the
# same bench command under rocprofv3 --kernel-trace --stats (kernel durations beside the bench's
# HIP events), then the drop-in rates.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05v}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ --durations=20 > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity')}, d['roofline']['frac'], d['roofline']['traffic'], (d.get('placement') or {}).get('first_pair_ms'), (d.get('placement') or {}).get('chosen_pair_ms'), d['k1_per_call']['ms'], d['cpu_baseline']['value'])"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o trace -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_trace.log 2>&1 ) || { echo FAIL c3_trace; tail -20 $OUT/c3_trace.log; exit 1; }
python3 tools/summarize_trace.py $OUT/c3_trace $OUT/c3_trace.log $OUT/prof 20 "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline" || exit 1
rm -rf $OUT/c3_trace
cat $OUT/prof/summary.json | head -20
timeout -k 10 400 python tools/dropin_rate.py 7 > $OUT/dropin.log 2>&1 || { tail -20 $OUT/dropin.log; exit 1; }
grep '^{' $OUT/dropin.log | grep -v setup
echo EXIT 0
