"""Round-3 PMC traffic summary (not part of the product): FETCH_SIZE / WRITE_SIZE passes of
tools/r03/gpu_u.sh -> profiles/r03/pmc/summary.json, and the matching profiles/traffic.json keys
(kernel | plan spec | workload, the key bench.py looks up for `roofline.traffic`).

HBM bytes per launch = 2 x 1024 x FETCH_SIZE + 1024 x WRITE_SIZE (FETCH_SIZE is in kB and counts
half the bytes of wide coalesced reads on gfx950, MI355X_MICROARCH.md HBM section), averaged over
the round kernel's last 4 dispatches (the bench's timed steps).

usage: python tools/summarize_r03_pmc.py [gpurun_out tag]"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def per_dispatch(path):
    by = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "k_round_" in k and "scalar" not in k and "direct" not in k:
            d = int(r["Dispatch_Id"])
            by[d] += float(r["Counter_Value"])
            names[d] = k
    return by, names


def main(tag="r03u"):
    src = ROOT / "gpurun_out" / tag
    out = {}
    traffic_path = ROOT / "profiles" / "traffic.json"
    traffic = json.loads(traffic_path.read_text())
    for spec_file in sorted(glob.glob(str(src / "pmc_*.spec"))):
        name = Path(spec_file).stem[len("pmc_"):]
        meta = json.loads(Path(spec_file).read_text())
        f, fn = per_dispatch(src / f"pmc_{name}_fetch" / "pmc_counter_collection.csv")
        w, _ = per_dispatch(src / f"pmc_{name}_write" / "pmc_counter_collection.csv")
        last_f = sorted(f)[-4:]
        last_w = sorted(w)[-4:]
        kernel = fn[last_f[-1]]
        f_kb = sum(f[d] for d in last_f) / len(last_f)
        w_kb = sum(w[d] for d in last_w) / len(last_w)
        bench = [json.loads(l) for l in open(src / f"pmc_{name}_fetch.log") if l.startswith("{")][-1]
        alg = bench["roofline"]["bytes_per_launch"]
        hbm = 2 * 1024 * f_kb + 1024 * w_kb
        short = bench["kernel"]
        key = f"{short}|{json.dumps(meta['spec'], sort_keys=True)}|{meta['workload']}"
        out[name] = dict(key=key, kernel=kernel, fetch_kB_raw=f_kb, write_kB=w_kb, hbm_bytes_per_launch=hbm,
                         algorithmic_bytes=alg, ratio=hbm / alg, parity=bench["parity"])
        traffic[key] = dict(kernel=kernel, bytes_per_launch=hbm, algorithmic_bytes=alg, ratio=hbm / alg,
                            fetch_kB_raw=f_kb, write_kB=w_kb,
                            correction="FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); kB = 1024 B",
                            source="profiles/r03/pmc")
        print(name, key, f"ratio {hbm / alg:.6f}")
    dst = ROOT / "profiles" / "r03" / "pmc"
    dst.mkdir(parents=True, exist_ok=True)
    (dst / "summary.json").write_text(json.dumps(out, indent=1))
    traffic_path.write_text(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
