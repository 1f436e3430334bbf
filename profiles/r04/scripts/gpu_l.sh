# Round 4 (l): the world-8 rehearsal of the weak-scaling default (random, tuned) with per-rank logs
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04l}; mkdir -p $OUT/logs
export MASTER_ADDR=127.0.0.1 OMP_NUM_THREADS=1
timeout -k 10 280 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29931 \
  --log-dir $OUT/logs --redirects 3 bench.py --gpus 8 --dist-backend gloo --graph random --model resnet50 --dtype f32 \
  --exchange auto --max-params 131072 --steps 2 --warmup 1 > $OUT/run.log 2>&1; rc=$?
echo rc=$rc
for f in $(find $OUT/logs -name "stderr.log"); do if grep -q "Error\|Traceback" $f; then echo "== $f"; grep -v "^\[Gloo\]" $f | tail -25; fi; done
echo EXIT 0
