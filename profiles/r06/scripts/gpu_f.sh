#!/bin/bash
# Round 6 (r06f): double-buffered rounds (RoundExecutor's spare pool + storage exchange): the GPU
# tests that run the executor, the drop-in rate (double-buffered vs in place), and one PMC pass
# (FETCH_SIZE) of the bf16 wide-row form against one K1 call per row.
set -o pipefail
t=${1:-r06f}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_double_buffer.py tests/test_gpu_interface.py tests/test_gpu_reg.py tests/test_gpu_kernels.py \
  tests/test_gpu_bf16.py tests/test_gpu_wide_rows.py > $o/t.log 2>&1 && \
timeout -k 10 300 python -u tools/dropin_rate.py 5 > $o/dropin.log 2>&1 && \
grep '^{' $o/dropin.log > $o/dropin.jsonl && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d $o/wfetch -o pmc -- python3 $R/tools/wide_rows_rate.py --pmc > $o/wfetch.log 2>&1 ) && \
python3 tools/pmc_sum.py $o/wfetch k_round_wide k_agg k_round > $o/wfetch.jsonl
echo EXIT $?
