# Round 3 (c): K3r where-does-the-time-go probes on config 5 fp32 (base / nocomp / noload / hot
# scalar tables) and PMC of the base kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03c}; mkdir -p $OUT
export TMPDIR=/tmp
B="--graph sbm --devices 256 --model vit_b16 --dtype f32 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2"
for v in base regnocomp regnoload reghot; do
  if [ $v = base ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so; fi
  timeout -k 10 300 python bench.py $B --plan '{"reg": 1}' > $OUT/c5_$v.log 2>&1 || { echo FAIL $v; tail -5 $OUT/c5_$v.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), d['parity'])" $OUT/c5_$v.log $v
done
unset TAL_LIB_PATH
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_ANY"
P2="SQC_DCACHE_REQ SQC_DCACHE_MISSES SQC_DCACHE_HITS GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
cd /tmp
for P in P1 P2 P3; do
  timeout -s KILL 240 rocprofv3 --pmc ${!P} --output-format csv -d $OUT/pmc_$P -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $B --plan '{"reg": 1}' > $OUT/pmc_$P.log 2>&1 || { echo FAIL pmc $P; tail -5 $OUT/pmc_$P.log; exit 1; }
  f=$(find $OUT/pmc_$P -name '*counter_collection.csv' | head -1)
  echo "== $P"; python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" k_round_reg || true
done
