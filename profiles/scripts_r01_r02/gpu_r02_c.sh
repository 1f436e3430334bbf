# Round 2: the new interface/distributed GPU tests, the drop-in rate, config 2 under placement + SQ PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_interface.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests_interface.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests_interface.log; exit 1; }
timeout -k 10 400 python -u tools/dropin_rate.py 5 > $OUT/dropin.log 2>&1 || { echo DROPIN FAILED; tail -30 $OUT/dropin.log; exit 1; }
timeout -k 10 200 python bench.py --graph ring --model resnet18 --devices 32 --degree 2 --no-cpu-baseline --no-k1 > $OUT/c2_bench.log 2>&1 || { echo C2 FAILED; exit 1; }
SPEC=$(python -c "import json,sys; print(json.dumps([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['plan']['spec']))" $OUT/c2_bench.log)
cd /tmp
for CT in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  N=$(echo $CT | cut -c1-12 | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d $OUT/c2_pmc_$N -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --graph ring --model resnet18 --devices 32 --degree 2 --plan "$SPEC" --steps 4 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 > $OUT/c2_pmc_$N.log 2>&1 || { echo PMC FAILED $N; exit 1; }
done
echo EXIT 0
