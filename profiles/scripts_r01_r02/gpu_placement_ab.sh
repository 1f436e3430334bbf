# Placement calibration A/B on config 3: 4 vs 8 candidate output pools (bench --placement-trials),
# and in-place rounds on the best of 8; interleaved, one board.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-placeab}; mkdir -p $OUT
SPEC='{"c4": 64, "lds": 81920, "dense": 0}'
for rep in 1 2 3; do
  for t in 4 8; do
    timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-k1 --plan "$SPEC" --placement-trials $t >> $OUT/t$t.log 2>&1 || { echo FAILED t$t; exit 1; }
  done
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-k1 --plan "$SPEC" --placement-trials 8 --in-place >> $OUT/inplace8.log 2>&1 || { echo FAILED inplace; exit 1; }
done
for f in $OUT/t4.log $OUT/t8.log $OUT/inplace8.log; do
  python -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; p=d['placement'] or {}; print(sys.argv[1].split('/')[-1], round(r['kernel_ms'],3), round(r['frac'],3), p.get('dest_ms') or p.get('in_place_ms'), p.get('first_pair_ms'), d['parity'])
" $f
done
echo EXIT 0
