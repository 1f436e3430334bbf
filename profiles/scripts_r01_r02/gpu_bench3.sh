# The driver's default bench command three times on one board (placement + tuning variance).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bench3}; mkdir -p $OUT
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b$rep.log 2>&1 || { echo FAIL; tail -20 $OUT/b$rep.log; exit 1; }
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; p=d['placement']
print(round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['plan']['spec'], p['dest_ms'], p['chosen'], p['chosen_pair_ms'], p['first_pair_ms'], d['parity'])
" $OUT/b$rep.log
done
echo EXIT 0
