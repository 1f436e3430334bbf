# Activity PMC pass (one run) over one round-plan form: bash profiles/scripts_r01_r02/gpu_pmc_round2.sh <tag> <run_round.py args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/${TAG}_sq3 -o p -- python $GRAFT_REPO_ROOT/tools/run_round.py "$@" --steps 2 > $OUT/${TAG}_sq3.log 2>&1
echo EXIT $?
