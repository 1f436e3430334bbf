# Round 4: broadcast-form tests + distributed tests (virtual ranks, one-rank RCCL), config 5
# degree-centrality broadcast forms, and the one-rank transposed step (own block off RCCL).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04c}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --weights degcent"
timeout -k 10 900 python -u -m pytest tests/test_gpu_bcast.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
summ() { python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d.get('exchange'))
" $1 $2; }
for ex in transpose halo; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --sharded --exchange $ex --steps 10 --warmup 2 > $OUT/sharded_$ex.log 2>&1 || { echo "SHARDED FAILED $ex"; tail -20 $OUT/sharded_$ex.log; exit 1; }
  summ $OUT/sharded_$ex.log sharded_$ex
done
for dt in f32 bf16; do
  for spec in '{"c4":16,"lds":163840,"dense":0,"bcast":12,"bcwg":2}' '{"c4":16,"lds":163840,"dense":0,"bcast":16,"bcwg":2}'; do
    tag=$(echo "$dt$spec" | tr -dc 'a-z0-9')
    timeout -k 10 300 python bench.py $C5 --dtype $dt --plan "$spec" > $OUT/$tag.log 2>&1 || { echo "BENCH FAILED $tag"; tail -20 $OUT/$tag.log; exit 1; }
    summ $OUT/$tag.log $tag
  done
done
timeout -k 10 300 python tools/window_probe.py --windows 12 --allocs 6 > $OUT/window_c3.log 2>&1 || { echo WINDOW FAILED; tail -5 $OUT/window_c3.log; exit 1; }
tail -1 $OUT/window_c3.log
timeout -k 10 300 python bench.py --host-path --steps 5 --no-cpu-baseline --no-k1 --placement-trials 2 > $OUT/host.log 2>&1 || { echo HOST FAILED; tail -5 $OUT/host.log; exit 1; }
python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('host_path_per_call', d['host_path_per_call'])
" $OUT/host.log
echo EXIT 0
