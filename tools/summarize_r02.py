"""Summarize a round-2 profiling pass (profiles/scripts_r01_r02/gpu_profile.sh) into profiles/<sub>/ and
profiles/traffic.json.

Inputs under gpurun_out/<tag>/:
  c3_trace/            rocprofv3 --kernel-trace --stats of the driver's own bench command
  c3_trace.log         that run's bench JSON line (same process as the trace)
  pmc_<name>_fetch/    rocprofv3 --pmc FETCH_SIZE of bench.py --plan <spec> (one per plan spec)
  pmc_<name>_write/    rocprofv3 --pmc WRITE_SIZE of the same
  pmc_<name>.spec      the spec and workload key of that pair of passes

traffic.json keys are bench.traffic_key(kernel, spec, workload): the bench reports a PMC byte
count only for the kernel and plan that produced it.  FETCH_SIZE is doubled (gfx950: it counts
half the bytes of wide coalesced reads; MI355X_MICROARCH.md HBM section); kB = 1024 B.

usage: python tools/summarize_r02.py <tag> <profiles subdir>
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def bench_line(log: Path) -> dict:
    return [json.loads(l) for l in open(log) if l.startswith("{")][-1]


def dispatches(trace_csv: Path, short: str):
    """(dispatch id, ns, full name) of every dispatch whose name contains `short`<."""
    out = []
    for r in csv.DictReader(open(trace_csv)):
        if f"::{short}<" in r["Kernel_Name"] or r["Kernel_Name"].startswith(f"{short}<"):
            out.append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"]))
    return sorted(out)


def pmc_mean(path: Path, short: str, last: int):
    """Mean counter value over the kernel's last `last` dispatches (the timed steps)."""
    v = sorted((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"])
               for r in csv.DictReader(open(path)) if f"::{short}<" in r["Kernel_Name"])
    v = v[-last:]
    names = {n for _, _, n in v}
    return sum(x for _, x, _ in v) / max(1, len(v)), names


def main(tag, sub):
    import bench

    src = ROOT / "gpurun_out" / tag
    dst = ROOT / "profiles" / sub
    dst.mkdir(parents=True, exist_ok=True)
    report = {}
    # (1) the driver's command under the kernel trace: bench line and rocprof from one process
    if (src / "c3_trace.log").exists():
        b = bench_line(src / "c3_trace.log")
        shutil.copy(src / "c3_trace" / "trace_kernel_stats.csv", dst / "c3_kernel_stats.csv")
        (dst / "c3_bench_under_rocprof.json").write_text(json.dumps(b, indent=1))
        d = dispatches(src / "c3_trace" / "trace_kernel_trace.csv", b["kernel"])
        full = d[-1][2]
        same = [x for x in d if x[2] == full]
        timed = same[-b["steps"]:]
        stats = {r["Name"]: r for r in csv.DictReader(open(dst / "c3_kernel_stats.csv"))}
        B = b["roofline"]["bytes_per_launch"]
        t_ns = sum(x for _, x, _ in timed) / len(timed)
        a_ns = float(stats[full]["AverageNs"]) if full in stats else None
        report["c3_same_process"] = dict(
            kernel=full, spec=b["plan"]["spec"], bench_ms_per_step=b["ms_per_step"],
            bench_kernel_ms_hip_events=b["roofline"]["kernel_ms"], bench_frac=b["roofline"]["frac"],
            rocprof_dispatches=len(same), rocprof_avg_ms_all=a_ns / 1e6 if a_ns else None,
            rocprof_avg_ms_timed_steps=t_ns / 1e6,
            frac_from_rocprof_timed=B / (t_ns * 1e-9) / 1e9 / bench.HBM_PEAK_GBPS,
            frac_from_rocprof_all=B / (a_ns * 1e-9) / 1e9 / bench.HBM_PEAK_GBPS if a_ns else None,
            bytes_per_launch=B, placement=b.get("placement"))
    # (2) PMC byte counts per plan spec
    t = ROOT / "profiles" / "traffic.json"
    traffic = {}  # rewritten: round-1 workload-only keys are superseded
    for spec_file in sorted(src.glob("pmc_*.spec")):
        name = spec_file.stem[4:]
        meta = json.loads(spec_file.read_text())
        f_log, w_log = src / f"pmc_{name}_fetch.log", src / f"pmc_{name}_write.log"
        b = bench_line(f_log)
        short = b["kernel"]
        f_kb, fn = pmc_mean(src / f"pmc_{name}_fetch" / "pmc_counter_collection.csv", short, b["steps"])
        w_kb, wn = pmc_mean(src / f"pmc_{name}_write" / "pmc_counter_collection.csv", short, b["steps"])
        hbm = 2 * f_kb * 1024 + w_kb * 1024
        key = bench.traffic_key(short, b["plan"]["spec"], meta["workload"])
        traffic[key] = dict(kernel=sorted(fn)[0], bytes_per_launch=hbm, algorithmic_bytes=b["roofline"]["bytes_per_launch"],
                            ratio=hbm / b["roofline"]["bytes_per_launch"], fetch_kB_raw=f_kb, write_kB=w_kb,
                            correction="FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); kB = 1024 B",
                            source=f"profiles/{sub}")
        shutil.copy(f_log, dst / f"pmc_{name}_fetch.log")
        shutil.copy(w_log, dst / f"pmc_{name}_write.log")
    if traffic:
        t.write_text(json.dumps(traffic, indent=1, sort_keys=True))
        report["traffic"] = traffic
    (dst / "summary.json").write_text(json.dumps(report, indent=1))
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
