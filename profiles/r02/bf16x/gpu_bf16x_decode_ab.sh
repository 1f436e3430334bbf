set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-decab}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --dtype bf16 --mode exact --plan {\"c4\":16,\"lds\":81920,\"dense\":0}"
for rep in 1 2; do
  for v in base dec; do
    if [ $v = base ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so; fi
    timeout -k 10 400 python bench.py $C5 >> $OUT/$v.log 2>&1 || { echo FAIL $v; exit 1; }
  done
done
export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_dec.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests_dec.log 2>&1 || { echo TESTS FAILED; tail -20 $OUT/tests_dec.log; exit 1; }
tail -1 $OUT/tests_dec.log
for v in base dec; do python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); print(sys.argv[2], round(d['roofline']['kernel_ms'],3), d['parity'])
" $OUT/$v.log $v; done
echo EXIT 0
