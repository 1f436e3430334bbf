# Round 4 (m): config 5 degree-centrality rounds with default tuning after the tuner key fix
# (c4 16 / 32 broadcast candidates kept apart), and the untimed defaults beside them.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04m}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --weights degcent"
for run in "bf16|tuned|" "bf16|default|--no-tune" "f32|tuned|" "f32|default|--no-tune"; do
  IFS='|' read -r dt name extra <<< "$run"
  timeout -k 10 400 python bench.py $C5 --dtype $dt $extra > $OUT/c5dc_${dt}_$name.log 2>&1 || { echo "FAILED $dt $name"; tail -20 $OUT/c5dc_${dt}_$name.log; exit 1; }
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
c=sorted([x for x in (d['plan'].get('candidates') or []) if x.get('ms')], key=lambda x: x['ms'])[:4]
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['plan']['spec'], [(x['c4'], x['ms']) for x in c])
" $OUT/c5dc_${dt}_$name.log ${dt}_$name
done
echo EXIT 0
