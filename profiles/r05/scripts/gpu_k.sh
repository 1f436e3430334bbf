# Round 5 (r05k): smoke (now with one app call on pool-bound models), and HBM traffic of the
# headline plan (config 3, persistent c4 64) from FETCH_SIZE / WRITE_SIZE passes (one counter
# block per pass; tools/run_round.py --fill randn; the last round dispatch kept).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05k}; mkdir -p $OUT
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
RR="$R/tools/run_round.py --graph random --devices 64 --model resnet50 --fill randn --steps 3 --plan {\"c4\":64,\"lds\":81920,\"dense\":0}"
for ctr in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o pmc -- \
      python3 $RR > $OUT/pmc_$ctr.log 2>&1 ) && python3 $R/tools/pmc_shrink.py $OUT/pmc_$ctr || { echo "FAIL $ctr"; tail -5 $OUT/pmc_$ctr.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
v = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = list(csv.DictReader(open(glob.glob(f"{out}/pmc_{c}/*counter_collection.csv")[0])))
    v[c] = sum(float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == c)
    v["kernel"] = rows[0]["Kernel_Name"]
alg = 4 * 23573962 * (64 + 64)
hbm = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024  # kB; gfx950 FETCH_SIZE counts half of wide reads
json.dump(dict(kernel=v["kernel"], FETCH_SIZE_kB=v["FETCH_SIZE"], WRITE_SIZE_kB=v["WRITE_SIZE"], hbm_bytes=hbm,
               algorithmic_bytes=alg, ratio=hbm / alg), open(f"{out}/traffic_c3.json", "w"), indent=1)
print(json.dumps(dict(hbm_bytes=hbm, algorithmic=alg, ratio=round(hbm / alg, 6))))
PY
echo EXIT $?
