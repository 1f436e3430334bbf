#!/bin/bash
# K2's column kind on one 512 x 512 x 3 x 3 tensor (8 pairs): timings and two PMC passes.
# usage: bash profiles/r05/scripts/gpu_k2pmc.sh <tag>   (writes gpurun_out/<tag>/)
set -e
t=${1:?tag}
R=$PWD
OUT=$R/gpurun_out/$t
mkdir -p $OUT
timeout -k 10 120 python3 tools/cosine_one.py 512,512,3,3 20 > $OUT/one_col.log 2>&1
timeout -k 10 120 python3 tools/cosine_one.py 2048,1024 20 > $OUT/one_row.log 2>&1
pass() {
  local name=$1; shift
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- \
      python3 $R/tools/cosine_one.py 512,512,3,3 3 > $OUT/$name.log 2>&1 )
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD
pass ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
python3 tools/pmc_print.py k_cosine_outputs $OUT/sq $OUT/ta > $OUT/pmc.jsonl
