"""Round-4 PMC summary (not part of the product): profiles/r04/scripts/gpu_pmc.sh's passes over
config 5 with degree-centrality weights, before (K3n pairs form, K3r) and after (the broadcast
form) -> profiles/r04/pmc/summary.json, plus the traffic keys bench.py looks up
(profiles/traffic.json: kernel | plan spec | workload).

Per run: the wave-state fractions (8 SQ counters), SQ_LDS_IDX_ACTIVE / SQ_INSTS_VALU /
SQ_INSTS_LDS / bank conflicts per launch, and HBM bytes per launch = 2 x 1024 x FETCH_SIZE +
1024 x WRITE_SIZE (FETCH_SIZE in kB, half-counted on gfx950: MI355X_MICROARCH.md HBM section),
each from the last round-kernel dispatch of its pass (the bench's last timed step).

usage: python tools/summarize_r04_pmc.py [gpurun_out tag]"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def last_dispatch(path):
    """Counters summed over every agent/XCD instance of the last round-kernel dispatch."""
    by = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if ("k_round_f32_narrow" in k or "k_round_reg" in k) and "scalar" not in k:
            d = int(r["Dispatch_Id"])
            by[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = k
    d = max(by)
    return dict(by[d]), names[d]


def bench_line(log):
    return [json.loads(l) for l in open(log) if l.startswith("{")][-1]


def main(tag="r04pmc"):
    src = ROOT / "gpurun_out" / tag
    out = {}
    traffic_path = ROOT / "profiles" / "traffic.json"
    traffic = json.loads(traffic_path.read_text())
    for spec_file in sorted(glob.glob(str(src / "*.spec"))):
        name = Path(spec_file).stem
        meta = json.loads(Path(spec_file).read_text())
        rec = dict(spec=meta["spec"], dtype=meta["dtype"])
        ws, kernel = last_dispatch(src / f"{name}_ws" / "pmc_counter_collection.csv")
        wc = ws["SQ_WAVE_CYCLES"]
        rec["kernel"] = kernel
        rec["wave_states"] = {k: ws[k] for k in sorted(ws)}
        rec["frac_of_wave_cycles"] = dict(wait_any=ws["SQ_WAIT_ANY"] / wc, wait_inst_any=ws["SQ_WAIT_INST_ANY"] / wc,
                                          active_any=ws["SQ_ACTIVE_INST_ANY"] / wc,
                                          active_valu=ws["SQ_ACTIVE_INST_VALU"] / wc,
                                          active_lds=ws["SQ_ACTIVE_INST_LDS"] / wc,
                                          wait_inst_lds=ws["SQ_WAIT_INST_LDS"] / wc)
        lv, _ = last_dispatch(src / f"{name}_lv" / "pmc_counter_collection.csv")
        rec["lds_valu"] = {k: lv[k] for k in sorted(lv)}
        if "GRBM_GUI_ACTIVE" in lv and lv["GRBM_GUI_ACTIVE"]:
            # SQ_LDS_IDX_ACTIVE summed over CUs; GRBM_GUI_ACTIVE summed over the 8 XCDs
            rec["lds_array_busy"] = lv["SQ_LDS_IDX_ACTIVE"] / 256 / (lv["GRBM_GUI_ACTIVE"] / 8)
        b = bench_line(src / f"{name}_lv.log")
        rec["kernel_ms_under_pmc"] = b["roofline"]["kernel_ms"]
        rec["parity"] = b["parity"]
        fetch = src / f"{name}_fetch" / "pmc_counter_collection.csv"
        if fetch.exists():
            f, _ = last_dispatch(fetch)
            w, _ = last_dispatch(src / f"{name}_write" / "pmc_counter_collection.csv")
            hbm = 2 * 1024 * f["FETCH_SIZE"] + 1024 * w["WRITE_SIZE"]
            bf = bench_line(src / f"{name}_fetch.log")
            alg = bf["roofline"]["bytes_per_launch"]
            rec.update(hbm_bytes_per_launch=hbm, algorithmic_bytes=alg, ratio=hbm / alg)
            wl = "sbm-256-vit_b16" + ("-bf16" if meta["dtype"] == "bf16" else "") + "-degcent"
            key = f"{bf['kernel']}|{json.dumps(meta['spec'], sort_keys=True)}|{wl}"
            rec["traffic_key"] = key
            traffic[key] = dict(kernel=kernel, bytes_per_launch=hbm, algorithmic_bytes=alg, ratio=hbm / alg,
                                fetch_kB_raw=f["FETCH_SIZE"], write_kB=w["WRITE_SIZE"],
                                correction="FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); kB = 1024 B",
                                source="profiles/r04/pmc")
        out[name] = rec
        print(name, kernel[:60], round(rec["kernel_ms_under_pmc"], 3),
              {k: round(v, 3) for k, v in rec["frac_of_wave_cycles"].items()}, round(rec.get("ratio", 0), 5))
    dst = ROOT / "profiles" / "r04" / "pmc"
    dst.mkdir(parents=True, exist_ok=True)
    (dst / "summary.json").write_text(json.dumps(out, indent=1))
    traffic_path.write_text(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
