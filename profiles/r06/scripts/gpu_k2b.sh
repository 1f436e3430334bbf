#!/bin/bash
# Round 6 K2 (cosine), second form: the streamed column kernels (k_cos_col_norms /
# k_cos_col_prods).  Cosine GPU tests (bitwise the oracle), tools/cosine_bench.py (ResNet-50 and
# ViT-B/16, one client vs 8 neighbors, pair 0 bitwise the oracle at full size), by tensor kind,
# one 512 x 512 x 3 x 3 tensor, and a kernel trace.
# usage: bash profiles/r06/scripts/gpu_k2b.sh <tag>   (writes gpurun_out/<tag>/)
set -o pipefail
t=${1:?tag}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -k cosine -x -v --timeout 200 --timeout-method thread > $o/t.log 2>&1 && \
timeout -k 10 120 python tools/cosine_bench.py resnet50 > $o/bench1.log 2>&1 && \
timeout -k 10 120 python tools/cosine_bench.py resnet50 > $o/bench2.log 2>&1 && \
timeout -k 10 120 python tools/cosine_bench.py vit_b16 > $o/bench_vit.log 2>&1 && \
timeout -k 10 120 python tools/cosine_kinds.py resnet50 > $o/kinds.log 2>&1 && \
timeout -k 10 120 python3 tools/cosine_one.py 512,512,3,3 20 > $o/one_col.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o k2 -- python3 $R/tools/cosine_bench.py resnet50 > $o/prof.log 2>&1 )
rc=$?
echo EXIT $rc
