set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/tune/round_variants 23573962 reg > gpurun_out/tune3_reg.log 2>&1 && \
timeout -k 10 300 ./tools/tune/round_variants 23573962 barbell > gpurun_out/tune3_bar.log 2>&1
echo EXIT $?
