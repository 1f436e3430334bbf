# Round 3 (r): where config 5's compute side goes — SQ wave-state counters (parked / issue-stalled
# / active, VALU and LDS activity) for the full K3n round and the compute-side probe (noload),
# fp32 EXACT and bf16 FMA, one counter pass each
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03r}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
B="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --no-tune"
pmc() {  # name lib extra
  local name=$1 lib=$2; shift 2
  TAL_LIB_PATH=$lib timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/$name -o pmc -- \
    python3 $R/bench.py $B "$@" > $OUT/$name.log 2>&1 || { echo FAIL $name; tail -5 $OUT/$name.log; return 1; }
  echo ok $name
}
pmc f32_full $R/topology_aware_learning_amd/libtal_agg.so --dtype f32 &&
pmc f32_noload $R/tools/tune/libtal_agg_noload.so --dtype f32 &&
pmc bf16_full $R/topology_aware_learning_amd/libtal_agg.so --dtype bf16 &&
pmc bf16_noload $R/tools/tune/libtal_agg_noload.so --dtype bf16 || exit 1
