# GPU A/B of two library builds on one box: parity tests with the in-tree library, then config 3
# and config 5 (fp32, bf16) with the in-tree library and with tools/tune/libtal_agg_base.so
# swapped in, interleaved.  Usage: bash profiles/scripts_r01_r02/gpu_lib_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-lib}
LIB=topology_aware_learning_amd/libtal_agg.so
cp $LIB /tmp/libtal_agg_new.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then cp tools/tune/libtal_agg_base.so $LIB; else cp /tmp/libtal_agg_new.so $LIB; fi
    timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-k1 --plan '{"c4": 32, "lds": 81920, "dense": 0}' > $OUT/${TAG}_c3_${v}_r${rep}.log 2>&1 || { echo C3 FAILED; exit 1; }
    timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5_${v}_r${rep}.log 2>&1 || { echo C5 FAILED; exit 1; }
  done
done
cp /tmp/libtal_agg_new.so $LIB
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5bf16_new.log 2>&1 || { echo C5BF16 FAILED; exit 1; }
echo EXIT 0
