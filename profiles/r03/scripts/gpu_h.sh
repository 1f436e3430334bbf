# Round 3 (h): K3r with ordered item tickets; pieces in flight per XCD (blocks per CU 3 / 2 / 1); HBM fetch
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reg.py > $OUT/reg_tests.log 2>&1; rc=$?
tail -2 $OUT/reg_tests.log; [ $rc -eq 0 ] || exit $rc
B="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --dtype f32"
for bpc in 3 2 1; do
  export TAL_REG_BLOCKS_PER_CU=$bpc
  timeout -k 10 300 python bench.py $B --plan '{"reg":1}' > $OUT/c5_bpc$bpc.log 2>&1 || { echo FAIL; tail -3 $OUT/c5_bpc$bpc.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('bpc', sys.argv[2], round(d['roofline']['kernel_ms'],3), d['parity'])" $OUT/c5_bpc$bpc.log $bpc
  cd /tmp
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_bpc$bpc -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $B --plan '{"reg":1}' > $OUT/pmc_bpc$bpc.log 2>&1 || { echo FAIL pmc; exit 1; }
  f=$(find $OUT/pmc_bpc$bpc -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" k_round_reg
  cd $GRAFT_REPO_ROOT
done
