set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-c24}; mkdir -p $OUT
timeout -k 10 300 python bench.py --graph ring --devices 32 --model resnet18 --degree 2 --steps 20 --no-cpu-baseline --no-k1 > $OUT/c2.log 2>&1 && \
timeout -k 10 300 python bench.py --graph barbell --devices 128 --model resnet50 --steps 10 --no-cpu-baseline --no-k1 > $OUT/c4.log 2>&1 || { echo FAILED; exit 1; }
for f in c2 c4; do python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; p=d.get('placement') or {}
print(sys.argv[2], round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['kernel'], p.get('chosen_pair_ms'), p.get('first_pair_ms'))
" $OUT/$f.log $f; done
echo EXIT 0
