# Round 3 (t): K3n ROWW row loop as a rotating LDS-read pipeline — narrow / bf16 / full-size
# config-5 parity tests, then A/B against the previous loop (TAL_PROBE_NOPIPE build) on config 5
# fp32 EXACT, bf16 FMA, bf16 EXACT, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03t}; mkdir -p $OUT
export TMPDIR=/tmp
NP=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_nopipe.so
B="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 2 --no-tune"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'])" $OUT/c5_$1.log $1
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_bf16.py -k "narrow or bf16 or b16 or round" > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "config5 and (None or bf16)" > $OUT/full.log 2>&1; rc=$?
tail -3 $OUT/full.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/full.log | head -20; exit $rc; }
run f32_pipe "--dtype f32" &&
TAL_LIB_PATH=$NP run f32_nopipe "--dtype f32" &&
run bf16_pipe "--dtype bf16" &&
TAL_LIB_PATH=$NP run bf16_nopipe "--dtype bf16" &&
run f32_pipe2 "--dtype f32" &&
TAL_LIB_PATH=$NP run f32_nopipe2 "--dtype f32" &&
run bf16_pipe2 "--dtype bf16" &&
TAL_LIB_PATH=$NP run bf16_nopipe2 "--dtype bf16" &&
run bf16x_pipe "--dtype bf16 --mode exact" &&
TAL_LIB_PATH=$NP run bf16x_nopipe "--dtype bf16 --mode exact" || exit 1
# where the transposed exchange's local time goes: config 3 on a one-rank RCCL group, kernel trace
cd /tmp
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr1_trace -o trace -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --sharded --exchange transpose --steps 5 --warmup 2 --no-tune > $OUT/tr1_trace.log 2>&1 || { echo FAIL tr1; tail -20 $OUT/tr1_trace.log; exit 1; }
head -12 $OUT/tr1_trace/trace_kernel_stats.csv | cut -c1-200
