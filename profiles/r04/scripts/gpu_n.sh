# Round 4 (n): the drop-in per-call round against the interpreter's thread switch interval
# (5000 us default, 500, 100): are the app threads' stalls GIL hand-offs?
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04n}; mkdir -p $OUT
for sw in 5000 500 100 5000; do
  timeout -k 10 300 python -u tools/dropin_rate.py 7 --switch-us=$sw > $OUT/dropin_sw$sw.log 2>&1 || { echo FAIL $sw; tail -20 $OUT/dropin_sw$sw.log; exit 1; }
  grep '"mode"' $OUT/dropin_sw$sw.log | tail -2 | cut -c1-160 | sed "s/^/sw=$sw /"
done
echo EXIT 0
