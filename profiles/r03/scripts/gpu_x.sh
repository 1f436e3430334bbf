# Round 3 (x): K1 (per-call kernel): one vs two float4 chunks per lane (probe build), interleaved,
# timed by bench.py's k1_per_call (64 back-to-back calls, rows rotated)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03x}; mkdir -p $OUT
export TMPDIR=/tmp
NT=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_k1x2.so
B="--steps 2 --warmup 1 --no-cpu-baseline --placement-trials 2 --no-tune"
run() {
  timeout -k 10 200 python bench.py $B > $OUT/k1_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/k1_$1.log; return 1; }
  grep '^{' $OUT/k1_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['k1_per_call']['ms'],4), round(d['k1_per_call']['frac'],3))"
}
run plain && TAL_LIB_PATH=$NT run x2 && run plain2 && TAL_LIB_PATH=$NT run x2b || exit 1
