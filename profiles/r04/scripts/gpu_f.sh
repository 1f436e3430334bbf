# Round 4 (f): config 5 with degree-centrality weights through every form (pairs, K3r, broadcast
# 8x2 / 12x2 / 16x2 / 16x1), the no-prefetch probe (each tile's loads issued after the previous
# tile's math: what a single-buffered DMA staging would cost), the one-rank sharded step of both
# exchanges (own block off RCCL) and the host-memory path with pinned binding by default.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04f}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2"
summ() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d.get('exchange'), d.get('parity_k3_vs_k1'))
" $1 $2; }
run() {  # tag, extra args (lib env optional via LIBP)
  local tag=$1; shift
  TAL_LIB_PATH=$LIBP timeout -k 10 300 python bench.py $C5 "$@" > $OUT/$tag.log 2>&1 || { echo "BENCH FAILED $tag"; tail -20 $OUT/$tag.log; exit 1; }
  summ $OUT/$tag.log $tag
}
timeout -k 10 300 python -u -m pytest tests/test_cosine_threads.py tests/test_gpu_kernels.py -k cosine -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PAIRS='{"c4":16,"lds":163840,"dense":0}'
LIBP=
for dt in f32 bf16; do
  run ${dt}_dc_pairs --weights degcent --dtype $dt --plan "$PAIRS"
  for bc in 8:2 12:2 16:2 16:1; do
    w=${bc%%:*}; g=${bc##*:}
    run ${dt}_dc_bcast${w}x$g --weights degcent --dtype $dt --plan "{\"c4\":16,\"lds\":163840,\"dense\":0,\"bcast\":$w,\"bcwg\":$g}"
  done
done
run bf16_dc_reg --weights degcent --dtype bf16 --plan '{"reg":1}'
run f32_dc_default --weights degcent --dtype f32 --no-tune
run bf16_dc_default --weights degcent --dtype bf16 --no-tune
run f32_unw_default --dtype f32 --no-tune
run bf16_unw_default --dtype bf16 --no-tune
LIBP=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_nopf.so
run nopf_f32_unw_default --dtype f32 --no-tune
run nopf_bf16_unw_default --dtype bf16 --no-tune
run nopf_bf16_dc_bcast16x2 --weights degcent --dtype bf16 --plan '{"c4":16,"lds":163840,"dense":0,"bcast":16,"bcwg":2}'
run nopf_f32_dc_bcast8x2 --weights degcent --dtype f32 --plan '{"c4":16,"lds":163840,"dense":0,"bcast":8,"bcwg":2}'
LIBP=
for ex in transpose halo; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --sharded --exchange $ex --steps 10 --warmup 2 > $OUT/sharded_$ex.log 2>&1 || { echo "SHARDED FAILED $ex"; tail -20 $OUT/sharded_$ex.log; exit 1; }
  summ $OUT/sharded_$ex.log sharded_$ex
done
timeout -k 10 300 python bench.py --host-path --steps 5 --no-cpu-baseline --no-k1 --placement-trials 2 > $OUT/host.log 2>&1 || { echo HOST FAILED; tail -5 $OUT/host.log; exit 1; }
python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('host_path_per_call', d['host_path_per_call'])
" $OUT/host.log
echo EXIT 0
