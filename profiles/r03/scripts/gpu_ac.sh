# Round 3 (ac): K3n in 512-thread workgroups (TAL_NARROW_PIPE512=1: pipelined row loop, =2: plain
# loop) against the product's 1024-thread form — narrow parity tests under each mode, then config
# 5 fp32 EXACT / bf16 FMA timings, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03ac}; mkdir -p $OUT
export TMPDIR=/tmp
B="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 2 --no-cpu-baseline --no-k1 --placement-trials 2 --no-tune"
run() {  # name, extra args
  timeout -k 10 300 python bench.py $B $2 > $OUT/c5_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c5_$1.log; return 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'])" $OUT/c5_$1.log $1
}
for m in 1 2; do
  TAL_NARROW_PIPE512=$m timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_bf16.py -k "narrow or bf16 or b16 or round" > $OUT/tests_$m.log 2>&1; rc=$?
  tail -2 $OUT/tests_$m.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests_$m.log | head -20; exit $rc; }
done
run f32_base "--dtype f32" &&
TAL_NARROW_PIPE512=1 run f32_p512 "--dtype f32" &&
TAL_NARROW_PIPE512=2 run f32_n512 "--dtype f32" &&
run bf16_base "--dtype bf16" &&
TAL_NARROW_PIPE512=1 run bf16_p512 "--dtype bf16" &&
TAL_NARROW_PIPE512=2 run bf16_n512 "--dtype bf16" &&
run f32_base2 "--dtype f32" &&
TAL_NARROW_PIPE512=1 run f32_p512b "--dtype f32" &&
TAL_NARROW_PIPE512=2 run f32_n512b "--dtype f32" || exit 1
