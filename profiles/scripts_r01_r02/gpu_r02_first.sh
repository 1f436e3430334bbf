# Round 2 first pass: GPU suite, smoke, bench, and the PMC counter list of this board.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/r02_counters.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/r02a_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r02a_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 4 > $OUT/r02a_bench.log 2>&1
echo EXIT $?
