#!/bin/bash
# Round 6 final: the driver's bench command (N = 1), the same command under rocprofv3
# --kernel-trace --stats (kernel durations against the bench's HIP-event kernel time), the
# drop-in rate through the reference's driver, and K2 timings.
set -o pipefail
t=${1:-r06y}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
timeout -k 10 300 python -u bench.py > $o/bench.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o bench -- python3 $R/bench.py > $o/prof_bench.log 2>&1 ) && \
timeout -k 10 300 python -u tools/dropin_rate.py 5 > $o/dropin.log 2>&1 && \
timeout -k 10 120 python tools/cosine_bench.py resnet50 > $o/cos_r50.log 2>&1 && \
timeout -k 10 120 python tools/cosine_bench.py vit_b16 > $o/cos_vit.log 2>&1
echo EXIT $?
