"""Summarize a `rocprofv3 --kernel-trace --stats` run of bench.py into profiles/ (not the product).

usage: python tools/summarize_trace.py <trace dir> <bench log> <out dir> [steps] [command]

The bench's timed steps are the last `steps` dispatches of the round kernel it reports (nothing
after the timed region launches that kernel again); their mean duration is compared with the
bench's own HIP-event kernel time.  Writes <out dir>/summary.json, kernel_stats.csv (copy) and
bench_line.json.
"""
import csv
import json
import shutil
import sys
from pathlib import Path


def main():
    trace, log, out = Path(sys.argv[1]), Path(sys.argv[2]), Path(sys.argv[3])
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    command = sys.argv[5] if len(sys.argv) > 5 else ""
    out.mkdir(parents=True, exist_ok=True)
    line = [json.loads(x) for x in open(log) if x.startswith("{")][-1]
    kt = next(trace.glob("*kernel_trace.csv"))
    rows = list(csv.DictReader(open(kt)))
    name_key = "Kernel_Name"
    by = {}
    for r in rows:
        by.setdefault(r[name_key], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    want = line.get("kernel") or ""
    cands = [k for k in by if k.startswith("void (anonymous namespace)::k_round")]
    if want:
        base = want.split("<")[0]
        cands = [k for k in cands if base in k] or cands
    # the round kernel the bench timed is the one dispatched last
    rk = max(cands, key=lambda k: max(s for s, _ in by[k]))
    d = sorted(by[rk])
    timed = [x for _, x in d[-steps:]]
    bpl = line["roofline"]["bytes_per_launch"]
    peak = line["roofline"]["peak"]
    mean_ms = sum(timed) / len(timed) / 1e6
    summ = dict(command=command, round_kernel=rk, timed_dispatches=len(timed), timed_mean_ms=round(mean_ms, 4),
                timed_frac=round(bpl / (mean_ms * 1e-3) / 1e9 / peak, 4),
                all_dispatches_of_that_name=len(d), all_mean_ms=round(sum(x for _, x in d) / len(d) / 1e6, 4),
                bench_hip_event_kernel_ms=round(line["roofline"]["kernel_ms"], 4), bench_frac=round(line["roofline"]["frac"], 4),
                bench_value=line["value"], bench_ms_per_step=line["ms_per_step"])
    k1 = [x for k, v in by.items() if "k_agg_model" in k for _, x in v]
    if k1 and line.get("k1_per_call"):
        k1_ms = sum(k1) / len(k1) / 1e6
        summ.update(k_agg_model_dispatches=len(k1), k_agg_model_mean_ms=round(k1_ms, 4),
                    k_agg_model_frac=round(line["k1_per_call"]["bytes"] / (k1_ms * 1e-3) / 1e9 / peak, 4)
                    if "bytes" in line["k1_per_call"] else None)
    json.dump(summ, open(out / "summary.json", "w"), indent=1)
    json.dump(line, open(out / "bench_line.json", "w"), indent=1)
    st = next(trace.glob("*kernel_stats.csv"), None)
    if st:
        shutil.copy(st, out / "kernel_stats.csv")
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
