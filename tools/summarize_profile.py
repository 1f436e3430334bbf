"""Summarize rocprofv3 outputs (kernel stats + FETCH_SIZE / WRITE_SIZE passes) into profiles/.

usage: python tools/summarize_profile.py <gpurun_out tag> <profiles subdir>
Writes <subdir>/kernel_stats.csv (copy), <subdir>/pmc_summary.json and updates
profiles/traffic.json (HBM bytes per launch of the round kernel, FETCH_SIZE corrected x2 per
MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads).
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def per_kernel(path, last=4):
    """Mean counter value per kernel name over its last `last` dispatches (the bench's timed
    steps come last; earlier dispatches include tune_plan's candidates)."""
    by = {}
    for r in csv.DictReader(open(path)):
        by.setdefault(r["Kernel_Name"], []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {k: sum(x for _, x in sorted(v)[-last:]) / len(sorted(v)[-last:]) for k, v in by.items()}


def last_round_kernel(path):
    """Name of the round kernel dispatched last (the plan the bench timed)."""
    best = (-1, None)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "k_round_" in k and "scalar" not in k and "direct" not in k and int(r["Dispatch_Id"]) > best[0]:
            best = (int(r["Dispatch_Id"]), k)
    return best[1]


def timed_steps(trace_csv, kernel, steps=20):
    """Mean duration (ns) of the kernel's last `steps` dispatches in a rocprofv3 kernel trace:
    the bench's timed steps (tuning candidates and placement trials come earlier)."""
    d = sorted((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
               for r in csv.DictReader(open(trace_csv)) if r["Kernel_Name"] == kernel)
    last = [x for _, x in d[-steps:]]
    return dict(kernel=kernel, dispatches=len(d), last_n=len(last), mean_ns_last_n=sum(last) / max(1, len(last)),
                mean_ns_all=sum(x for _, x in d) / max(1, len(d)))


def main(tag, sub, key="random-64-resnet50"):
    src = ROOT / "gpurun_out"
    dst = ROOT / "profiles" / sub
    dst.mkdir(parents=True, exist_ok=True)
    shutil.copy(src / f"{tag}_prof" / "trace_kernel_stats.csv", dst / "kernel_stats.csv")
    fetch = per_kernel(src / f"{tag}_pmc_fetch" / "pmc_counter_collection.csv")
    write = per_kernel(src / f"{tag}_pmc_write" / "pmc_counter_collection.csv")
    summ = {}
    for k in fetch:
        if "tal" in k or "anonymous namespace)::k_" in k:
            f_kb, w_kb = fetch[k], write.get(k, 0.0)
            summ[k] = dict(FETCH_SIZE_kB_raw=f_kb, WRITE_SIZE_kB=w_kb,
                           hbm_bytes_corrected=2 * f_kb * 1024 + w_kb * 1024)
    (dst / "pmc_summary.json").write_text(json.dumps(summ, indent=1))
    stats = {r["Name"]: r for r in csv.DictReader(open(dst / "kernel_stats.csv"))}
    k = last_round_kernel(src / f"{tag}_pmc_fetch" / "pmc_counter_collection.csv")
    if k is not None:
        trace = src / f"{tag}_prof" / "trace_kernel_trace.csv"
        if trace.exists():
            (dst / "round_kernel_timed_steps.json").write_text(json.dumps(timed_steps(trace, k), indent=1))
        t = ROOT / "profiles" / "traffic.json"
        d = json.loads(t.read_text()) if t.exists() else {}
        d.pop("resnet50", None)  # round-1 key, superseded by workload keys
        d[key] = dict(kernel=k, bytes_per_launch=summ[k]["hbm_bytes_corrected"],
                        fetch_kB_raw=summ[k]["FETCH_SIZE_kB_raw"], write_kB=summ[k]["WRITE_SIZE_kB"],
                        correction="FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); units kB=1024 B",
                        rocprof_avg_ns=float(stats[k]["AverageNs"]) if k in stats else None,
                        source=f"profiles/{sub}")
        t.write_text(json.dumps(d, indent=1))
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
