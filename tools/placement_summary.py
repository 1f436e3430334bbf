"""Join tools/placement_probe.py's per-launch times with the rocprofv3 PMC rows of the same
process (round-kernel dispatches in launch order; the first is the warm-up)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main(d):
    d = Path(d)
    for tag in ("pmcA", "pmcB", "pmcC"):
        js = [json.loads(l) for l in open(d / f"{tag}.jsonl") if l.startswith('{"launch"')]
        rows = defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(d / tag / "pmc_counter_collection.csv")):
            if "k_round_f32_persistent" not in r["Kernel_Name"]:
                continue
            did = int(r["Dispatch_Id"])
            rows[did][r["Counter_Name"]] = float(r["Counter_Value"])
            names[did] = r["Kernel_Name"][:40]
        ids = sorted(rows)[1:]  # drop the warm-up
        print(f"== {tag}")
        for j, did in zip(js, ids):
            c = rows[did]
            print(j["pool"], j["rep"], j["ms"], " ".join(f"{k.replace('_sum','')}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1])
