set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02j; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SPEC='{"c4": 16, "dense": 0, "lds": 81920}'
for dt in bf16 f32; do
  timeout -k 10 300 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype $dt --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --plan "$SPEC" > $OUT/c5_${dt}.log 2>&1 || { echo FAIL $dt; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), d['parity'], d.get('bf16_vs_fp32_reference_row0'))" $OUT/c5_${dt}.log $dt
done
echo EXIT 0
