#!/bin/bash
# Round 6: K2 staged-kernel phase timing with the stamped diagnostic build (tools/cosine_stamps.py;
# built from the product source by a throwaway patch: s_memtime at each phase boundary).
set -o pipefail
t=${1:-r06s}
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/$t
mkdir -p $o
cd $R
export TAL_LIB_PATH=$R/tools/tune/libtal_agg_stamps.so
for shape in 512,512,3,3 256,256,3,3 64,64,3,3; do
  timeout -k 10 120 python tools/cosine_stamps.py $shape >> $o/stamps.log 2>&1 || exit 1
done
TAL_COS_STAGE_ROWS=1 timeout -k 10 120 python tools/cosine_stamps.py 2048,1024 >> $o/stamps.log 2>&1 && TAL_COS_STAGE_ROWS=1 timeout -k 10 120 python tools/cosine_stamps.py 512,2048 >> $o/stamps.log 2>&1
echo EXIT $?
timeout -k 10 300 python -u tools/dropin_rate.py 5 --profile > $o/dropin_profile.log 2>&1
echo EXIT $?
