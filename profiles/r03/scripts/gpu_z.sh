# Round 3 (z): closing run — full -m gpu suite, smoke, the driver's default bench command, the
# drop-in call-surface rates
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03z}; mkdir -p $OUT
bash tools/r03/gpu_v.sh ${1:-r03z} || exit 1
timeout -k 10 600 python -u tools/dropin_rate.py 7 > $OUT/dropin.log 2>&1 || { echo FAIL dropin; tail -20 $OUT/dropin.log; exit 1; }
grep '^{' $OUT/dropin.log
