# Round 3 (w): the driver's default bench command twice (K1 timing change)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03w}; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py > $OUT/bench$i.log 2>&1 || { tail -20 $OUT/bench$i.log; exit 1; }
  grep '^{' $OUT/bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity')}, d['roofline']['frac'], d['placement']['first_pair_ms'], d['placement']['chosen_pair_ms'], d['k1_per_call']['ms'], d['k1_per_call']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['ms_per_call'])"
done
