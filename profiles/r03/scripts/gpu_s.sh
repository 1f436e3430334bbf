# Round 3 (s): the sharded bench path on a one-rank RCCL group (tests + config 3 at full size)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03s}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_distributed.py -k "one_rank" > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
for ex in transpose halo; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 1 --sharded --exchange $ex --steps 10 --warmup 3 > $OUT/c3_sharded_$ex.log 2>&1 || { echo FAIL $ex; tail -20 $OUT/c3_sharded_$ex.log; exit 1; }
  grep '^{' $OUT/c3_sharded_$ex.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ex', d['value'], d['ms_per_step'], d['parity'], d['roofline']['kernel_ms'], d['bound_model']['measured_over_predicted'], d['bound_model']['kernel_share_of_step'])"
done
