# GPU A/B of two library builds on config 5 bf16, EXACT and FMA (in-tree library vs
# tools/tune/libtal_agg_base.so), interleaved, after the kernel parity tests.
# Usage: bash profiles/scripts_r01_r02/gpu_lib_ab_bf16x.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-libx}
LIB=topology_aware_learning_amd/libtal_agg.so
cp $LIB /tmp/libtal_agg_new.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then cp tools/tune/libtal_agg_base.so $LIB; else cp /tmp/libtal_agg_new.so $LIB; fi
    for m in exact fma; do
      timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --mode $m --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_${m}_${v}_r${rep}.log 2>&1 || { cp /tmp/libtal_agg_new.so $LIB; echo FAILED; exit 1; }
    done
  done
done
cp /tmp/libtal_agg_new.so $LIB
echo EXIT 0
