# Round 4 (g): fp32 broadcast form with DMA staging (TAL_BC_DMA=1): parity (both stagings), then
# config 5 with degree-centrality weights per form, register staging vs DMA, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04g}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --weights degcent --dtype f32"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bcast.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
summ() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d.get('parity_k3_vs_k1',{}).get('rows_differing'))
" $1 $2; }
for rep in 1 2; do
  for bc in 16:2 12:2 8:2 16:1; do
    w=${bc%%:*}; g=${bc##*:}
    for dma in 1 0; do
      tag=f32_dc_bcast${w}x${g}_dma${dma}_$rep
      TAL_BC_DMA=$dma timeout -k 10 300 python bench.py $C5 --plan "{\"c4\":16,\"lds\":163840,\"dense\":0,\"bcast\":$w,\"bcwg\":$g}" > $OUT/$tag.log 2>&1 || { echo "BENCH FAILED $tag"; tail -20 $OUT/$tag.log; exit 1; }
      summ $OUT/$tag.log $tag
    done
  done
done
echo EXIT 0
