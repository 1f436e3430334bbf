# Round 3 (q): 16-B staging lanes for bf16 narrow rounds (W16) — bf16 parity tests, then A/B on
# config 5 bf16 FMA / EXACT against TAL_NARROW_W16=0, interleaved; with / without 16-B stores (S16)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03q}; mkdir -p $OUT
export TMPDIR=/tmp
B="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 2 --no-tune"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'], d.get('plan',{}).get('spec'))" $OUT/c5_$1.log $1
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py tests/test_gpu_kernels.py -k "bf16 or narrow or b16" > $OUT/w16_tests.log 2>&1; rc=$?
tail -3 $OUT/w16_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/w16_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "config5" > $OUT/w16_full.log 2>&1; rc=$?
tail -3 $OUT/w16_full.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/w16_full.log | head -20; exit $rc; }
run bf16_ws "--dtype bf16" &&
TAL_NARROW_S16=0 run bf16_w16 "--dtype bf16" &&
TAL_NARROW_W16=0 run bf16_w8 "--dtype bf16" &&
run bf16_wsb "--dtype bf16" &&
TAL_NARROW_S16=0 run bf16_w16b "--dtype bf16" &&
TAL_NARROW_W16=0 run bf16_w8b "--dtype bf16" &&
run bf16x_ws "--dtype bf16 --mode exact" &&
TAL_NARROW_W16=0 run bf16x_w8 "--dtype bf16 --mode exact" || exit 1
timeout -k 10 240 ./tools/tune/c5_walk_probe > $OUT/walk_f32.log 2>&1 && cat $OUT/walk_f32.log &&
timeout -k 10 240 ./tools/tune/c5_walk_probe bf16 > $OUT/walk_bf16.log 2>&1 && cat $OUT/walk_bf16.log
