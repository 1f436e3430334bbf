# Round-4 closing table: BASELINE configs 2, 4, 5 (fp32, bf16 FMA, bf16 EXACT, degree-centrality
# weights) and the host-memory per-call path, with the product's default tuning, one board.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04cfg}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1"
timeout -k 10 300 python bench.py --graph ring --devices 32 --model resnet18 --degree 2 --steps 20 --no-cpu-baseline --no-k1 > $OUT/c2.log 2>&1 && \
timeout -k 10 300 python bench.py --graph barbell --devices 128 --model resnet50 --steps 10 --no-cpu-baseline --no-k1 > $OUT/c4.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 > $OUT/c5.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 > $OUT/c5bf16.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 --mode exact > $OUT/c5bf16x.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --weights degcent > $OUT/c5degcent.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --weights degcent --dtype bf16 > $OUT/c5degcent_bf16.log 2>&1 && \
timeout -k 10 300 python bench.py --host-path --steps 5 --no-cpu-baseline > $OUT/host.log 2>&1 || { echo FAILED; exit 1; }
for f in c2 c4 c5 c5bf16 c5bf16x c5degcent c5degcent_bf16 host; do
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['kernel'], (d.get('plan') or {}).get('spec'), d.get('host_path_per_call',{}).get('ms') if 'host_path_per_call' in d else '')
" $OUT/$f.log $f
done
echo EXIT 0
