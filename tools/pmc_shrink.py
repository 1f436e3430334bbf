"""Shrink a rocprofv3 --pmc output directory in place (not part of the product): keep only the
rows of the last round-kernel dispatch (k_round_f32_narrow / k_round_reg / k_round_f32_persistent,
not the scalar tail kernels) in pmc_counter_collection.csv, so a GPU run's outputs stay under
gpurun's 64 MiB copy-back limit.  usage: python tools/pmc_shrink.py <dir>"""
import csv
import sys
from pathlib import Path


def main(d):
    d = Path(d)
    p = next(d.rglob("*counter_collection.csv"))
    rows = list(csv.DictReader(open(p)))
    keep = [r for r in rows if any(k in r["Kernel_Name"] for k in ("k_round_f32_narrow", "k_round_reg", "k_round_f32_persistent"))
            and "scalar" not in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in keep)
    keep = [r for r in keep if int(r["Dispatch_Id"]) == last]
    for f in d.rglob("*"):
        if f.is_file():
            f.unlink()
    with open(d / "pmc_counter_collection.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(keep)


if __name__ == "__main__":
    main(sys.argv[1])
