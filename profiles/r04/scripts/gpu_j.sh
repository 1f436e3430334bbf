# Round 4 (j): the two-chunk broadcast form (c4 = 32: 16 lanes per row, two float4 chunks per lane,
# one workgroup of 16 wavefronts per CU): parity, then config 5 per form and weights, fp32 / bf16.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04j}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_bcast.py "tests/test_gpu_fullsize.py::test_config5_degree_centrality_vs_reference" "tests/test_gpu_fullsize.py::test_config5_bf16_fma_full_width_within_bound" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2"
summ() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d.get('parity_k3_vs_k1',{}).get('rows_differing'))
" $1 $2; }
X2_16='{"c4":32,"lds":163840,"dense":0,"bcast":16,"bcwg":1}'
X2_12='{"c4":32,"lds":163840,"dense":0,"bcast":12,"bcwg":1}'
for rep in 1 2; do
  for run in "f32|degcent|x2_16|$X2_16" "f32|degcent|default|none" "bf16|degcent|x2_16|$X2_16" "bf16|degcent|default|none" "f32|unweighted|x2_16|$X2_16" "f32|unweighted|default|none" "bf16|unweighted|x2_16|$X2_16" "bf16|unweighted|default|none" "f32|degcent|x2_12|$X2_12"; do
    IFS='|' read -r dt wt name spec <<< "$run"
    P="--plan $spec"; [ $spec = none ] && P="--no-tune"
    tag=${dt}_${wt}_${name}_$rep
    timeout -k 10 300 python bench.py $C5 --dtype $dt --weights $wt $P > $OUT/$tag.log 2>&1 || { echo "BENCH FAILED $tag"; tail -20 $OUT/$tag.log; exit 1; }
    summ $OUT/$tag.log $tag
  done
done
echo EXIT 0
