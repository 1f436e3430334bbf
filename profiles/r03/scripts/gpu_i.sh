# Round 3 (i): K3r v4 (pair trips as one asm loop over 16-dword records, neutral-padded): parity tests,
# config-5 fp32 / bf16 / degcent lines, nocomp / noload probes, HBM fetch PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reg.py > $OUT/reg_tests.log 2>&1; rc=$?
tail -3 $OUT/reg_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/reg_tests.log | head -20; exit $rc; }
B="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'])" $OUT/c5_$1.log $1
}
run reg_f32 "--dtype f32 --plan {\"reg\":1}" &&
run reg_bf16 "--dtype bf16 --plan {\"reg\":1}" &&
run reg_f32_degcent "--dtype f32 --weights degcent --plan {\"reg\":1}" &&
run reg_f32_fma "--dtype f32 --mode fma --plan {\"reg\":1}" &&
TAL_REG_BLOCKS_PER_CU=2 run reg_f32_bpc2 "--dtype f32 --plan {\"reg\":1}" &&
TAL_REG_BLOCKS_PER_CU=2 run reg_bf16_bpc2 "--dtype bf16 --plan {\"reg\":1}" || exit 1
for v in regnocomp regnoload; do
  export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so
  run ${v}_f32 "--dtype f32 --plan {\"reg\":1}" || exit 1
done
unset TAL_LIB_PATH
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $B --dtype f32 --plan '{"reg":1}' > $OUT/pmc_fetch.log 2>&1 || { echo FAIL pmc; exit 1; }
f=$(find $OUT/pmc_fetch -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" k_round_reg
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $OUT/pmc_sq -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $B --dtype f32 --plan '{"reg":1}' > $OUT/pmc_sq.log 2>&1 || { echo FAIL pmc; exit 1; }
f=$(find $OUT/pmc_sq -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$f" k_round_reg
