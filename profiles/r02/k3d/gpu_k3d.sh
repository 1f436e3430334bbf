# GPU: K3d (dense row blocks over 512-B tiles) parity tests, then config 5 (SBM-256 ViT-B/16)
# fp32 EXACT and bf16 FMA with the K3d plan and with the narrow c4 = 16 plan (A/B, one board).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-k3d}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense_narrow.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 1"
D='{"c4":32,"lds":163840,"dense":8}'
N='{"c4":16,"lds":163840,"dense":0}'
for arm in d n d n; do
  P=$D; [ $arm = n ] && P=$N
  timeout -k 10 300 python bench.py $C5 --plan "$P" >> $OUT/c5_$arm.log 2>&1 || { echo FAIL c5 $arm; tail -20 $OUT/c5_$arm.log; exit 1; }
  timeout -k 10 300 python bench.py $C5 --dtype bf16 --plan "$P" >> $OUT/c5bf16_$arm.log 2>&1 || { echo FAIL c5bf16 $arm; tail -20 $OUT/c5bf16_$arm.log; exit 1; }
done
for f in c5_d c5_n c5bf16_d c5bf16_n; do
  python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],3), round(r.get('kernel_ms',0),3), round(r['frac'],3), d.get('parity'), d.get('kernel'))
" $OUT/$f.log $f
done
echo EXIT 0
