"""Mean per-dispatch PMC values of the kernels matching a name filter.

usage: python tools/pmc_summary.py <pmc_counter_collection.csv> [name-substring]
"""
import collections
import csv
import sys

path = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "k_round"
agg = collections.defaultdict(float)
disp = set()
for r in csv.DictReader(open(path)):
    if flt not in r["Kernel_Name"] or "direct" in r["Kernel_Name"]:
        continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    disp.add(r["Dispatch_Id"])
n = max(1, len(disp))
print(f"{len(disp)} dispatches")
for k, v in sorted(agg.items()):
    print(f"  {k:28s} {v / n:.4g}")
