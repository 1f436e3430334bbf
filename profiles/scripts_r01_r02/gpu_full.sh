# Full GPU pass: tests, smoke, bench, rocprofv3 kernel trace + PMC (FETCH_SIZE / WRITE_SIZE).
# Usage: bash profiles/scripts_r01_r02/gpu_full.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
TAG=${1:-full}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/${TAG}_bench.log 2>&1 && \
SPEC=$(python -c "import json,sys; print(json.dumps([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['plan']['spec']))" $OUT/${TAG}_bench.log) && \
echo "profiled plan: $SPEC" && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_prof -o trace -- python $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --plan "$SPEC" > $OUT/${TAG}_prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${TAG}_pmc_fetch -o pmc -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-k1 --plan "$SPEC" > $OUT/${TAG}_pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${TAG}_pmc_write -o pmc -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-k1 --plan "$SPEC" > $OUT/${TAG}_pmc_write.log 2>&1
echo EXIT $?
