set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tune4 -o t -- $GRAFT_REPO_ROOT/tools/tune/round_variants 23573962 reg > $GRAFT_REPO_ROOT/gpurun_out/tune4.log 2>&1
echo EXIT $?
