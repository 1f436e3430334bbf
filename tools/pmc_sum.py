"""Sum rocprofv3 --pmc counters over every dispatch, per kernel (not part of the product): one
JSON line per kernel name (template arguments dropped) with the dispatch count and each
counter's total.  usage: python tools/pmc_sum.py <dir> [<kernel-substring> ...]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main(d, subs):
    p = next(Path(d).rglob("*counter_collection.csv"))
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"].removeprefix("void ").replace("(anonymous namespace)::", "").split("<")[0].split("(")[0]
        if subs and not any(s in name for s in subs):
            continue
        tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    for name in sorted(tot):
        print(json.dumps(dict(kernel=name, dispatches=len(disp[name]), **tot[name])), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
