# GPU: full gpu test suite, then the bench default (config 3, metric config), ring-32 ResNet-18
# and config 5 fp32 / bf16 with the product default plan choice.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02m}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c3.log 2>&1 || { echo FAIL c3; exit 1; }
timeout -k 10 300 python bench.py --graph ring --devices 32 --model resnet18 --steps 20 --no-cpu-baseline --no-k1 > $OUT/c2.log 2>&1 || { echo FAIL c2; exit 1; }
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/c5.log 2>&1 || { echo FAIL c5; exit 1; }
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/c5bf16.log 2>&1 || { echo FAIL c5bf16; exit 1; }
for f in c3 c2 c5 c5bf16; do
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d.get('parity'), d.get('plan_spec') or d.get('config',{}).get('plan'))" $OUT/$f.log $f
done
echo EXIT 0
