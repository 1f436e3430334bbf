# Round 5 (dt): after K1 on pool row addresses and direct seeding -: the drop-in per-call round under rocprofv3 --kernel-trace --stats: K1 durations in
# the driver (its bound pool's placement) and the gaps between the 64 launches of a round.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05dt}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dropin_trace -o trace -- \
  python3 $R/tools/dropin_rate.py 7 > $OUT/dropin_trace.log 2>&1 || { echo FAIL dropin_trace; tail -20 $OUT/dropin_trace.log; exit 1; }
grep '^{' $OUT/dropin_trace.log | cut -c1-300
python3 - $OUT/dropin_trace <<'PY'
import csv, glob, sys, json
p = glob.glob(sys.argv[1] + "/*kernel_trace.csv")[0]
rows = [r for r in csv.DictReader(open(p)) if "k_agg_model" in r["Kernel_Name"]]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
dur = [(e - s) / 1e3 for s, e in ev]
gaps = [(ev[i + 1][0] - ev[i][1]) / 1e3 for i in range(len(ev) - 1)]
small = sorted(g for g in gaps if g < 1000)
print(json.dumps(dict(k1_launches=len(ev), k1_us_median=sorted(dur)[len(dur) // 2], k1_us_mean=sum(dur) / len(dur),
                      gap_us_median=small[len(small) // 2] if small else None,
                      gap_us_p90=small[int(len(small) * 0.9)] if small else None, gaps_over_1ms=len(gaps) - len(small))))
PY
rm -f $OUT/dropin_trace/*kernel_trace.csv
echo EXIT 0
