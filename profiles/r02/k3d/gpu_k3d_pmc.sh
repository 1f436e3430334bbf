# K3d (config 5, fp32 EXACT) PMC: where the time goes (scalar issue, scalar loads, VALU, LDS).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-k3dpmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
SPEC=${SPEC:-'{"c4": 32, "dense": 8, "lds": 163840}'}
DT=${DT:-f32}
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*SCA[A-Z_]*\|SQ_INSTS_S[A-Z]*\|SQ_INST_CYCLES_[A-Z]*\|SQ_WAIT_INST_[A-Z]*\|SQ_ACTIVE_INST_[A-Z]*\|SQ_IFETCH[A-Z_]*\|SQC_[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/names.txt || true
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES"
B="SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for P in A B; do
  timeout -s KILL 180 rocprofv3 --pmc ${!P} --output-format csv -d $OUT/$P -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --graph sbm --devices 256 --model vit_b16 --dtype $DT --steps 2 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --plan "$SPEC" > $OUT/$P.log 2>&1 || { echo FAIL $P; tail -5 $OUT/$P.log; exit 1; }
  f=$(find $OUT/$P -name '*counter_collection.csv' | head -1)
  echo "== $P"; python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" ${KNAME:-k_round_dense_narrow}
done
echo EXIT 0
