# PMC passes (one run each) over one round-plan form: bash profiles/scripts_r01_r02/gpu_pmc_round.sh <tag> <run_round.py args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 python $GRAFT_REPO_ROOT/tools/run_round.py "$@" > $OUT/${TAG}_run.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $OUT/${TAG}_sq1 -o p -- python $GRAFT_REPO_ROOT/tools/run_round.py "$@" --steps 2 > $OUT/${TAG}_sq1.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SENDMSG --output-format csv -d $OUT/${TAG}_sq2 -o p -- python $GRAFT_REPO_ROOT/tools/run_round.py "$@" --steps 2 > $OUT/${TAG}_sq2.log 2>&1
echo EXIT $?
