# GPU check: kernel parity tests, smoke, bench (short).  Usage: bash profiles/scripts_r01_r02/gpu_check.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 6 > gpurun_out/${TAG}_bench.log 2>&1
echo EXIT $?
