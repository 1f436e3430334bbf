# Config 5 narrow kernel PMC (same-process counters per launch), by variant and dtype.
# VARIANTS (default "base noload"), DTYPES (default "f32 bf16").
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-k3npmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
SPEC='{"c4": 16, "dense": 0, "lds": 81920}'
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"
B="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_IFETCH SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE"
cd /tmp
for v in ${VARIANTS:-base noload}; do
  if [ $v = base ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so; fi
  for dt in ${DTYPES:-f32 bf16}; do
    for P in A B; do
      timeout -s KILL 180 rocprofv3 --pmc ${!P} --output-format csv -d $OUT/${v}_${dt}_$P -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --graph sbm --devices 256 --model vit_b16 --dtype $dt --steps 2 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --plan "$SPEC" > $OUT/${v}_${dt}_$P.log 2>&1 || { echo FAIL $v $dt $P; exit 1; }
      f=$(find $OUT/${v}_${dt}_$P -name '*counter_collection.csv' | head -1)
      echo "== $v $dt $P"; python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" k_round_f32_narrow
    done
  done
done
echo EXIT 0
