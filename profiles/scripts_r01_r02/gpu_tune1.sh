set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/tune/round_variants > gpurun_out/tune_round.log 2>&1 && \
timeout -k 10 300 ./tools/tune/k1_variants > gpurun_out/tune_k1.log 2>&1
echo EXIT $?
