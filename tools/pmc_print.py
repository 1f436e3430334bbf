"""Print one kernel's counters from rocprofv3 --pmc output directories (not part of the
product): the last dispatch whose name contains the substring, one JSON line per directory.
usage: python tools/pmc_print.py <kernel-substring> <dir> [<dir> ...]"""
import csv
import json
import sys
from pathlib import Path


def main(sub, dirs):
    for d in dirs:
        p = next(Path(d).rglob("*counter_collection.csv"))
        rows = [r for r in csv.DictReader(open(p)) if sub in r["Kernel_Name"]]
        last = max(int(r["Dispatch_Id"]) for r in rows)
        vals = {}
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        print(json.dumps(dict(dir=str(d), kernel=sub, dispatch=last, **vals)), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
