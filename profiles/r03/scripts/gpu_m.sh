# Round 3 (m): bf16 image at c4 = 32 (256-B source pieces, 2 rows per wavefront) on config 5,
# the placement skew probe (config 3), the drop-in call-surface rates
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03m}; mkdir -p $OUT
export TMPDIR=/tmp
B="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 2"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'])" $OUT/c5_$1.log $1
}
P32='--plan {"c4":32,"lds":163840,"dense":0}'
TAL_NARROW_B16_IMAGE=1 run bf16_b16i_c32 "--dtype bf16 $P32" &&
run bf16_c32 "--dtype bf16 $P32" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i_c16 "--dtype bf16" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i_c32b "--dtype bf16 $P32" &&
TAL_NARROW_B16_IMAGE=1 run bf16x_b16i_c32 "--dtype bf16 --mode exact $P32" || exit 1
timeout -k 10 200 python -u tools/placement_skew_probe.py 6 > $OUT/skew.log 2>&1 || { echo SKEW FAILED; tail -20 $OUT/skew.log; exit 1; }
timeout -k 10 300 python tools/percall_profile.py 300 > $OUT/percall.log 2>&1 && head -3 $OUT/percall.log | grep aggregate
timeout -k 10 600 python -u tools/dropin_rate.py 5 > $OUT/dropin.log 2>&1; grep '^{' $OUT/dropin.log
