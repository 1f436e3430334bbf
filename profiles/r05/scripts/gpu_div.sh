#!/bin/bash
# K2 experiments r05div / r05k6 / r05k7: the range tests, the exhaustive
# 2^46-pair check of the candidate division scheme, then the K2 tests and timings (gpu_k2.sh).
# (the range tests were tests/test_gpu_cosine_ranges.py then; the checker is built by hand:
# hipcc --offload-arch=gfx950 -O3 -o tools/div_exhaustive tools/div_exhaustive.hip)
# usage: bash profiles/r05/scripts/gpu_div.sh <tag>   (writes gpurun_out/<tag>/)
set -e
t=${1:?tag}
o=gpurun_out/$t
mkdir -p $o
timeout -k 10 200 python -u -m pytest tests/test_gpu_cosine_ranges.py -m gpu -x -v --timeout 120 --timeout-method thread > $o/t_div.log 2>&1
timeout -k 10 600 tools/div_exhaustive 1 > $o/exhaustive.log 2>&1
bash profiles/r05/scripts/gpu_k2.sh $t
