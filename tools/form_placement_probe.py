"""Probe (not part of the product): which round-plan form holds its time wherever the pool it
writes sits in HBM?  VERDICT r04 item 3.

One input pool (config 3: 64 x ResNet-50), then destinations: `windows` pool-sized windows of
ONE arena allocation (round 4: 22 of 24 such windows ran the default plan slow, 2.30-2.48 ms)
and `allocs` separate allocations made after it (mostly fast).  Every plan form below is timed
writing into every destination, `reps` times, interleaved over forms and destinations; median
kept.  One JSON line per (form, destination) and one summary line per form.

Round 5 also timed every form under three other tile walks (runs of 2 and 8 tiles per workgroup,
one contiguous range per workgroup; a kernel switch since removed): slow windows stayed slow under
every walk (profiles/r05/r05c/walk_probe.jsonl).

Usage: python tools/form_placement_probe.py [--windows 8] [--allocs 4] [--reps 3]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from topology_aware_learning_amd import ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import StateLayout  # noqa: E402
from topology_aware_learning_amd.round import csr_from_lists  # noqa: E402

FORMS = [
    {"c4": 64, "lds": 81920, "dense": 0},     # the default / tuner pick on config 3
    {"c4": 128, "lds": 163840, "dense": 0},
    {"c4": 32, "lds": 81920, "dense": 0},     # narrow c4 32
    {"c4": 16, "lds": 81920, "dense": 0},     # narrow c4 16
    {"c4": 16, "lds": 163840, "dense": 0, "bcast": 8, "bcwg": 2},
    {"c4": 16, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 2},
    {"c4": 32, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 1},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--skip-windows", type=int, default=4, help="arena windows allocated but not timed (in front)")
    ap.add_argument("--allocs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--in-place", action="store_true", help="also time each form in place on every target")
    ap.add_argument("--forms", default="", help="comma-separated indices into FORMS (default: all)")
    a = ap.parse_args()
    forms = [FORMS[int(i)] for i in a.forms.split(",")] if a.forms else FORMS
    dev = torch.device("cuda", 0)
    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    n, ld = lay.n_f32, lay.ld_f32
    orders, ws = bench.round_spec(64, 8)
    rows = len(orders)
    rp, col, w = csr_from_lists(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    plans = []
    for spec in forms:
        try:
            plans.append((spec, ops.plan_from_spec(rp, col, w, out_rows, spec).to(dev)))
        except Exception as exc:  # a form this round cannot build
            print(json.dumps(dict(spec=spec, error=str(exc))), flush=True)
    src = torch.randn(rows, ld, device=dev)
    pool = rows * ld
    total = a.skip_windows + a.windows
    arena = torch.empty(total * pool, dtype=torch.float32, device=dev)
    targets = [("arena", k, arena[k * pool:(k + 1) * pool].view(rows, ld)) for k in range(a.skip_windows, total)]
    targets += [("alloc", k, torch.empty(rows, ld, device=dev)) for k in range(a.allocs)]
    for _, _, t in targets:
        t.copy_(src)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _, p in plans:
        ops.round_f32(src, targets[0][2], p, n=n)
    torch.cuda.synchronize()
    modes = [False, True] if a.in_place else [False]
    ms = {(i, j, ip): [] for i in range(len(plans)) for j in range(len(targets)) for ip in modes}
    for _ in range(a.reps):
        for j, (_, _, t) in enumerate(targets):
            for i, (_, p) in enumerate(plans):
                for ip in modes:
                    if ip and not p.single_group:
                        continue
                    s.record()
                    ops.round_f32(t if ip else src, t, p, n=n)
                    e.record()
                    e.synchronize()
                    ms[(i, j, ip)].append(s.elapsed_time(e))
    for i, (spec, p) in enumerate(plans):
        for ip in modes:
            per = []
            for j, (kind, k, t) in enumerate(targets):
                m = ms[(i, j, ip)]
                if not m:
                    continue
                v = float(np.median(m))
                per.append(v)
                print(json.dumps(dict(spec=spec, in_place=ip, kind=kind, index=k, ms=round(v, 4),
                                      all_ms=[round(x, 4) for x in m])), flush=True)
            if per:
                win = [v for v, (kind, _, _) in zip(per, targets) if kind == "arena"]
                alc = [v for v, (kind, _, _) in zip(per, targets) if kind == "alloc"]
                print(json.dumps(dict(summary=True, spec=spec, kernel=ops.round_kernel_name(p), in_place=ip,
                                      groups=p.info.n_groups, windows_ms=[round(v, 3) for v in win],
                                      allocs_ms=[round(v, 3) for v in alc], worst=round(max(per), 4),
                                      median=round(float(np.median(per)), 4), best=round(min(per), 4))), flush=True)


if __name__ == "__main__":
    main()
