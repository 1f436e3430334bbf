# Round 3 (n): re-run after the container reset: bf16-image parity tests, bf16 image A/B at
# c4 = 16 / 32 on config 5, the placement skew probe, the drop-in call-surface rates
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03n}; mkdir -p $OUT
export TMPDIR=/tmp
B="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 2"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'])" $OUT/c5_$1.log $1
}
P32='--plan {"c4":32,"lds":163840,"dense":0}'
TAL_NARROW_B16_IMAGE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > $OUT/b16i_tests.log 2>&1; rc=$?
tail -3 $OUT/b16i_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/b16i_tests.log | head -20; exit $rc; }
run bf16_base "--dtype bf16" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i_c16 "--dtype bf16" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i_c32 "--dtype bf16 $P32" &&
run bf16_c32 "--dtype bf16 $P32" &&
run bf16_base2 "--dtype bf16" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i_c16b "--dtype bf16" || exit 1
timeout -k 10 200 python -u tools/placement_skew_probe.py 6 > $OUT/skew.log 2>&1 || { echo SKEW FAILED; tail -20 $OUT/skew.log; exit 1; }
tail -12 $OUT/skew.log
timeout -k 10 300 python tools/percall_profile.py 300 > $OUT/percall.log 2>&1 && head -3 $OUT/percall.log | grep aggregate
timeout -k 10 600 python -u tools/dropin_rate.py 5 > $OUT/dropin.log 2>&1; grep '^{' $OUT/dropin.log
