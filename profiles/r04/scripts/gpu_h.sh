# Round 4 (h): where config 5's degree-centrality round spends its time: the broadcast form's
# memory side (nocomp: staging + stores, no row arithmetic) and compute side (noload: the first
# tile's data reused, no HBM reads) beside the full round, fp32 8x2 / 16x2 (DMA) and bf16 16x2,
# and the unweighted ROWW form for reference.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04h}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2"
summ() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'])
" $1 $2; }
BC8='{"c4":16,"lds":163840,"dense":0,"bcast":8,"bcwg":2}'
BC16='{"c4":16,"lds":163840,"dense":0,"bcast":16,"bcwg":2}'
for lib in full noload nocomp; do
  L=; [ $lib != full ] && L=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$lib.so
  for run in "f32_bc8|$BC8|f32|degcent|0" "f32_bc16dma|$BC16|f32|degcent|1" "bf16_bc16|$BC16|bf16|degcent|0" "f32_roww|none|f32|unweighted|0" "bf16_roww|none|bf16|unweighted|0"; do
    IFS='|' read -r name spec dt wt dma <<< "$run"
    P="--plan $spec"; [ $spec = none ] && P="--no-tune"
    TAL_LIB_PATH=$L TAL_BC_DMA=$dma timeout -k 10 300 python bench.py $C5 --dtype $dt --weights $wt $P > $OUT/${lib}_$name.log 2>&1 || { echo "BENCH FAILED ${lib}_$name"; tail -20 $OUT/${lib}_$name.log; exit 1; }
    summ $OUT/${lib}_$name.log ${lib}_$name
  done
done
echo EXIT 0
