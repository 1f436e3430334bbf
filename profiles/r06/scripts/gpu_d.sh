#!/bin/bash
# Round 6 (r06d): driver-level GPU tests after the host-time changes, and the drop-in rates.
set -o pipefail
t=${1:-r06d}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_interface.py tests/test_multipool.py > $o/t.log 2>&1 && \
timeout -k 10 300 python -u tools/dropin_rate.py 5 > $o/dropin.log 2>&1
rc=$?
grep "^{" $o/dropin.log > $o/dropin.jsonl
echo EXIT $rc
