# bf16 EXACT change check: bf16 parity tests (K1b, K3 forms, apps), then config 5 bf16 EXACT and
# bf16 FMA with the product's narrow plan.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bf16x}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --plan {\"c4\":16,\"lds\":81920,\"dense\":0}"
timeout -k 10 400 python bench.py $C5 --dtype bf16 --mode exact > $OUT/c5bf16x.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 > $OUT/c5bf16.log 2>&1 || { echo BENCH FAILED; exit 1; }
for f in c5bf16x c5bf16; do
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(r['kernel_ms'],3), round(r['frac'],3), d['parity'])
" $OUT/$f.log $f
done
echo EXIT 0
