# Round 5 (r05p): HBM traffic and memory-side counters of config 3's default plan in place vs
# out of place (why does the in-place round run 5-6 % slower on the same destination?).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05p}; mkdir -p $OUT
RR="$R/tools/run_round.py --graph random --devices 64 --model resnet50 --fill randn --steps 3 --plan {\"c4\":64,\"lds\":81920,\"dense\":0}"
pass() {  # name counters extra-args
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o pmc -- \
      python3 $RR $3 > $OUT/$1.log 2>&1 ) && python3 $R/tools/pmc_shrink.py $OUT/$1 || { echo "FAIL $1"; tail -5 $OUT/$1.log; return 1; }
  grep kernel $OUT/$1.log
}
for mode in out in; do
  X=""; [ $mode = in ] && X="--in-place"
  pass ${mode}_fetch FETCH_SIZE "$X" && pass ${mode}_write WRITE_SIZE "$X" && \
  pass ${mode}_ea "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" "$X" || exit 1
done
python3 - $OUT <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
res = {}
for f in sorted(glob.glob(f"{out}/*/pmc_counter_collection.csv")):
    name = f.split("/")[-2]
    for r in csv.DictReader(open(f)):
        res.setdefault(name, {})[r["Counter_Name"]] = res.get(name, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
for k, v in res.items():
    print(k, {kk: f"{vv:.4e}" for kk, vv in v.items()})
PY
echo EXIT $?
