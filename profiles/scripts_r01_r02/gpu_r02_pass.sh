# Round-2 full pass: GPU suite, smoke, then the profiling pass.  Usage: bash profiles/scripts_r01_r02/gpu_r02_pass.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02}
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -2 $OUT/${TAG}_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; exit 1; }
bash profiles/scripts_r01_r02/gpu_profile.sh ${TAG}prof
