#!/bin/bash
# Round 6 (r06e): the bf16 wide-row form (tests vs the oracle, timing against one K1 per row)
set -o pipefail
t=${1:-r06e}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wide_rows.py tests/test_gpu_bf16.py > $o/t.log 2>&1 && \
timeout -k 10 300 python -u tools/wide_rows_rate.py > $o/rate.log 2>&1
echo EXIT $?
