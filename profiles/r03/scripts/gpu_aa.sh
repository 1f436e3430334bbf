# Round 3 (aa): the multi-rank rehearsal and one-rank RCCL tests, including the tuned (driver
# default) variants
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03aa}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_distributed.py -k "world8_rehearsal and random" > $OUT/tests.log 2>&1; rc=$?
tail -15 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -30; exit $rc; }
