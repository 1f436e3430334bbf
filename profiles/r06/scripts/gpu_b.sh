#!/bin/bash
# Round 6 (r06b): the multi-GPU pool through the reference's driver on virtual GPUs, the
# interface / driver tests, and K2 (hybrid: staged column tensors, direct rows) with timings.
set -o pipefail
t=${1:-r06b}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $PT tests/test_multipool.py tests/test_gpu_interface.py tests/test_fill_counter.py > $o/t_multi.log 2>&1 && \
timeout -k 10 300 $PT tests -k cosine > $o/t_cos.log 2>&1 && \
timeout -k 10 120 python tools/cosine_bench.py resnet50 > $o/bench1.log 2>&1 && \
timeout -k 10 120 python tools/cosine_kinds.py resnet50 > $o/kinds.log 2>&1
rc=$?
echo EXIT $rc
