set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/tune/round_variants > gpurun_out/tune2_round.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/tune2_bench.log 2>&1
echo EXIT $?
