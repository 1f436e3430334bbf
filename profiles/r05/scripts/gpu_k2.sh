#!/bin/bash
# K2 (cosine) check and timing: the cosine GPU tests, tools/cosine_bench.py twice (ResNet-50,
# 8 pairs, bitwise pair 0 vs the oracle) and tools/cosine_kinds.py (time by tensor kind).
# usage: bash profiles/r05/scripts/gpu_k2.sh <tag>   (writes gpurun_out/<tag>/)
set -e
t=${1:?tag}
o=gpurun_out/$t
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -k cosine -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1
timeout -k 10 120 python tools/cosine_bench.py resnet50 > $o/bench1.log 2>&1
timeout -k 10 120 python tools/cosine_bench.py resnet50 > $o/bench2.log 2>&1
timeout -k 10 120 python tools/cosine_kinds.py resnet50 > $o/kinds.log 2>&1
