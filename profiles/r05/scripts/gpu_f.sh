# Round 5 (r05f): the per-call app path on pool rows (ops.agg_pool_rows) - its parity tests and
# the interface tests, the drop-in rates - then the round's closing measurements (gpu_e.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05f}; mkdir -p $OUT
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_pool_rows.py tests/test_gpu_interface.py tests/test_gpu_bf16.py > $OUT/t_pool.log 2>&1 || { tail -30 $OUT/t_pool.log; exit 1; }
tail -1 $OUT/t_pool.log
timeout -k 10 300 python tools/dropin_rate.py 7 > $OUT/dropin.log 2>&1 || { tail -20 $OUT/dropin.log; exit 1; }
grep '^{' $OUT/dropin.log | grep -v setup
bash profiles/r05/scripts/gpu_e.sh ${1:-r05f}
