# Placement probe: round time per output allocation + TLB / memory-side PMC in the same processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/placement
mkdir -p $OUT
export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/placement_probe.py
timeout -k 10 120 python $P 6 4 > $OUT/plain.jsonl 2>&1 && \
cd /tmp && \
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum --output-format csv -d $OUT/pmcA -o pmc -- python3 $P 6 2 > $OUT/pmcA.jsonl 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum --output-format csv -d $OUT/pmcB -o pmc -- python3 $P 6 2 > $OUT/pmcB.jsonl 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/pmcC -o pmc -- python3 $P 6 2 > $OUT/pmcC.jsonl 2>&1
echo EXIT $?
