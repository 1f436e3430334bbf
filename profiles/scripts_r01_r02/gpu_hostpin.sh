set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-hostpin}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_cache.py tests/test_gpu_interface.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python -u tools/host_round_rate.py 2 > $OUT/host_round_rate.log 2>&1 || { echo RATE FAILED; tail -20 $OUT/host_round_rate.log; exit 1; }
cat $OUT/host_round_rate.log
echo EXIT 0
