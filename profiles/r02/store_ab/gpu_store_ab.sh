# A/B of the round kernels' output store cache policy (nt = product, sc1, plain) on config 3
# (two plan specs the tuner picks) and config 5 fp32, interleaved, one board.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-storeab}; mkdir -p $OUT
for rep in 1 2 3; do
  for v in base sc1 plain; do
    if [ $v = base ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so; fi
    for spec in '{"c4": 64, "lds": 81920, "dense": 0}' '{"c4": 128, "lds": 163840, "dense": 0}'; do
      timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-k1 --plan "$spec" >> $OUT/c3_$v.log 2>&1 || { echo C3 FAILED $v; exit 1; }
    done
    [ $rep = 1 ] && { timeout -k 10 300 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --plan '{"c4": 16, "lds": 163840, "dense": 0}' >> $OUT/c5_$v.log 2>&1 || { echo C5 FAILED $v; exit 1; }; }
  done
done
for f in $OUT/c3_*.log $OUT/c5_*.log; do
  python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['plan']['spec']['c4'], round(r['kernel_ms'],3), round(r['frac'],3), d['placement'] and d['placement'].get('dest_ms'), d['parity'])
" $f
done
echo EXIT 0
