# Round 3 (p): the driver's bench command under rocprofv3 --kernel-trace --stats (bench line and
# kernel trace from one process), then the drop-in call-surface rates and cProfiles of both modes
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03p}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o trace -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3_trace.log 2>&1 || { echo FAIL c3_trace; tail -20 $OUT/c3_trace.log; exit 1; }
tail -1 $OUT/c3_trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity')}, d['roofline']['frac'], d.get('placement'))"
cd $R
timeout -k 10 600 python -u tools/dropin_rate.py 7 > $OUT/dropin.log 2>&1 || { echo FAIL dropin; tail -20 $OUT/dropin.log; exit 1; }
grep '^{' $OUT/dropin.log
timeout -k 10 300 python -u tools/dropin_rate.py 5 --profile > $OUT/dropin_prof_batched.log 2>&1 || { echo FAIL prof; tail -20 $OUT/dropin_prof_batched.log; exit 1; }
timeout -k 10 300 python -u tools/dropin_rate.py 5 --profile=per_call > $OUT/dropin_prof_percall.log 2>&1 || { echo FAIL prof2; exit 1; }
echo done
