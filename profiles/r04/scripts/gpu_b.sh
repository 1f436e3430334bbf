# Round 4: broadcast-form parity tests, then config 5 with degree-centrality weights through the
# pairs form and the broadcast forms (waves x workgroups per CU), fp32 EXACT and bf16 FMA.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04b}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --weights degcent"
timeout -k 10 900 python -u -m pytest tests/test_gpu_bcast.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
summ() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['parity_k3_vs_k1']['rows_differing'])
" $1 $2; }
for dt in f32 bf16; do
  for spec in '{"c4":16,"lds":163840,"dense":0,"bcast":12,"bcwg":2}' '{"c4":16,"lds":163840,"dense":0,"bcast":16,"bcwg":2}' '{"c4":16,"lds":163840,"dense":0}'; do
    tag=$(echo "$dt$spec" | tr -dc 'a-z0-9')
    timeout -k 10 300 python bench.py $C5 --dtype $dt --plan "$spec" > $OUT/$tag.log 2>&1 || { echo "BENCH FAILED $tag"; tail -20 $OUT/$tag.log; exit 1; }
    summ $OUT/$tag.log $tag
  done
done
echo EXIT 0
