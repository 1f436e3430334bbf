set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_interface.py tests/test_gpu_kernels.py tests/test_lib_abi.py -x -q -m gpu --timeout 200 --timeout-method thread -k "cosine or near_ties or app or abi or ring32" > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/cosine_bench.py resnet50 > $OUT/cos50.log 2>&1 || { echo COS FAILED; tail -20 $OUT/cos50.log; exit 1; }
timeout -k 10 300 python tools/cosine_bench.py resnet18 > $OUT/cos18.log 2>&1 || { echo COS FAILED; tail -20 $OUT/cos18.log; exit 1; }
cat $OUT/cos50.log $OUT/cos18.log | grep '^{'
echo EXIT 0
