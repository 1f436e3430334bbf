# Round 4: default-plan change (bf16 FMA per-operand weights -> broadcast form), config 5 bf16 FMA
# full-width bound tests, placement maps (windows of one arena across HBM, ballast first).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04d}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_reg.py "tests/test_gpu_fullsize.py::test_config5_bf16_fma_full_width_within_bound" -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -3
timeout -k 10 300 python tools/window_probe.py --windows 36 --allocs 4 --reps 3 > $OUT/window_map.log 2>&1 || { echo WINDOW FAILED; tail -5 $OUT/window_map.log; exit 1; }
tail -1 $OUT/window_map.log
timeout -k 10 300 python tools/window_probe.py --windows 12 --allocs 6 --reps 3 --ballast-gb 100 > $OUT/window_ballast.log 2>&1 || { echo BALLAST FAILED; tail -5 $OUT/window_ballast.log; exit 1; }
tail -1 $OUT/window_ballast.log
echo EXIT 0
