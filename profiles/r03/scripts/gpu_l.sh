# Round 3 (l): bf16 LDS image (TAL_NARROW_B16_IMAGE) A/B on config 5 + its parity tests, then the
# full -m gpu suite, smoke and the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03l}; mkdir -p $OUT
export TMPDIR=/tmp
B="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 2"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'])" $OUT/c5_$1.log $1
}
TAL_NARROW_B16_IMAGE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > $OUT/b16i_tests.log 2>&1; rc=$?
tail -3 $OUT/b16i_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/b16i_tests.log | head -20; exit $rc; }
run bf16_base "--dtype bf16" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i "--dtype bf16" &&
run bf16_base2 "--dtype bf16" &&
TAL_NARROW_B16_IMAGE=1 run bf16_b16i2 "--dtype bf16" &&
run bf16x_base "--dtype bf16 --mode exact" &&
TAL_NARROW_B16_IMAGE=1 run bf16x_b16i "--dtype bf16 --mode exact" || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity')}, d['roofline']['frac'], d.get('placement'), d['k1_per_call'])"
