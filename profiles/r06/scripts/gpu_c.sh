#!/bin/bash
# Round 6 (r06c): the whole GPU suite, the drop-in driver rates (per call / batched, with the
# round cache) and the default bench line.
set -o pipefail
t=${1:-r06c}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1 && \
timeout -k 10 300 python -u tools/dropin_rate.py 5 > $o/dropin.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $o/bench.log 2> $o/bench.err
rc=$?
echo EXIT $rc
