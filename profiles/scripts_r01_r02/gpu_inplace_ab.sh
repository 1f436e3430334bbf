# GPU A/B: config-3 round out of place (ping-pong between two pools) vs in place on one pool.
# Usage: bash profiles/scripts_r01_r02/gpu_inplace_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-ip}
P='{"c4": 32, "lds": 81920, "dense": 0}'
for rep in 1 2; do
  timeout -k 10 200 python bench.py --plan "$P" --steps 40 --no-cpu-baseline --no-k1 > $OUT/${TAG}_oop_r${rep}.log 2>&1 || { echo BENCH FAILED; exit 1; }
  timeout -k 10 200 python bench.py --plan "$P" --steps 40 --no-cpu-baseline --no-k1 --in-place > $OUT/${TAG}_inp_r${rep}.log 2>&1 || { echo BENCH FAILED; exit 1; }
done
timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-k1 --in-place > $OUT/${TAG}_inp_tuned.log 2>&1 || { echo BENCH FAILED; exit 1; }
echo EXIT 0
