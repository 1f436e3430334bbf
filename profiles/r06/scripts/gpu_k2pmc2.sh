#!/bin/bash
# Round 6: the streamed K2 column kernels (k_cos_col_norms, k_cos_col_prods) on one 512 x 512 x 3 x 3 tensor (8 pairs) and one
# 2048 x 1024 row tensor: timings and PMC passes (instruction mix, waits, LDS, cache accesses).
# usage: bash profiles/r06/scripts/gpu_k2pmc.sh <tag>   (writes gpurun_out/<tag>/)
set -o pipefail
t=${1:?tag}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$t
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 tools/cosine_one.py 512,512,3,3 20 > $OUT/one_col.log 2>&1 && \
timeout -k 10 120 python3 tools/cosine_one.py 2048,1024 20 > $OUT/one_row.log 2>&1 || exit 1
pass() {
  local name=$1; local shape=$2; shift; shift
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
      python3 $R/tools/cosine_one.py $shape 3 > $OUT/$name.log 2>&1 )
}
for shape in 512,512,3,3; do
  tag=${shape//,/x}
  pass sq_$tag $shape SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY || exit 1
  pass lds_$tag $shape SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
  pass mem_$tag $shape TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 1
  for kn in k_cos_col_norms k_cos_col_prods k_cosine_outputs; do python3 tools/pmc_print.py $kn $OUT/sq_$tag $OUT/lds_$tag $OUT/mem_$tag >> $OUT/pmc_$tag.jsonl || true; done
done
echo EXIT 0
