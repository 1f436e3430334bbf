"""Probe (not part of the product): is the slow / fast round placement a property of the
allocation or of where in HBM a pool's bytes sit?  VERDICT r03 item 3.

One input pool (config 3: 64 x ResNet-50, its own allocation), then
  arena   one allocation of `windows` pool-sized windows back to back; the round is timed
          writing into each window (GB-scale offsets inside ONE allocation);
  allocs  `allocs` separate pool allocations made after the arena, timed the same way.
Every target is timed `reps` times, interleaved over targets, median kept.  One JSON line per
target and a summary line.

With --step-mb the arena is one pool plus --span-gb and the windows slide by --step-mb inside
it (sub-pool offsets: is the fast / slow boundary finer than a pool?).

Usage: python tools/window_probe.py [--model resnet50] [--windows 12] [--allocs 6] [--reps 3]
       python tools/window_probe.py --step-mb 128 --span-gb 4
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--graph", default="random")
    ap.add_argument("--devices", type=int, default=64)
    ap.add_argument("--windows", type=int, default=12)
    ap.add_argument("--allocs", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ballast-gb", type=float, default=0.0, help="allocate (and keep) this much first")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--mode", default="exact", choices=["exact", "fma"])
    ap.add_argument("--step-mb", type=int, default=0, help="slide windows by this much (0: back to back)")
    ap.add_argument("--span-gb", type=float, default=4.0, help="with --step-mb: arena = pool + span")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ballast = torch.empty(int(a.ballast_gb * (1 << 30)), dtype=torch.uint8, device=dev) if a.ballast_gb else None
    lay = synth.get_layout(a.model)
    bf16 = a.dtype == "bf16"
    mode = ops.MODE_EXACT if a.mode == "exact" else ops.MODE_FMA
    lay = StateLayout.from_layout(synth.as_bf16(lay) if bf16 else lay)
    n, ld = (lay.n_b16, lay.ld_b16) if bf16 else (lay.n_f32, lay.ld_f32)
    dt = torch.bfloat16 if bf16 else torch.float32
    run = ops.round_bf16 if bf16 else ops.round_f32
    orders, ws = bench.round_spec(a.devices, 8, kind=a.graph)
    rows = len(orders)
    rp, col, w = csr_from_lists(orders, ws)
    plan = ops.default_plan(rp, col, w, np.arange(rows, dtype=np.int32), bf16=bf16, mode=mode).to(dev)
    src = torch.randn(rows, ld, device=dev, dtype=dt)  # in its dtype: no fp32 temporary of the pool's size
    pool_elems = rows * ld
    if a.step_mb:
        step = a.step_mb * (1 << 20) // src.element_size()
        span = int(a.span_gb * (1 << 30)) // src.element_size() // step * step
        arena = torch.empty(pool_elems + span, dtype=dt, device=dev)
        offs = range(0, span + 1, step)
    else:
        arena = torch.empty(a.windows * pool_elems, dtype=dt, device=dev)
        offs = range(0, a.windows * pool_elems, pool_elems)
    targets = [("arena", k, arena[o:o + pool_elems].view(rows, ld)) for k, o in enumerate(offs)]
    targets += [("alloc", k, torch.empty(rows, ld, dtype=dt, device=dev)) for k in range(a.allocs)]
    for _, _, t in targets:
        t.zero_()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    run(src, targets[0][2], plan, n=n, mode=mode)
    torch.cuda.synchronize()
    ms = [[] for _ in targets]
    for _ in range(a.reps):
        for i, (_, _, t) in enumerate(targets):
            s.record()
            run(src, t, plan, n=n, mode=mode)
            e.record()
            e.synchronize()
            ms[i].append(s.elapsed_time(e))
    base = arena.data_ptr()
    out = []
    for (kind, k, t), m in zip(targets, ms):
        rec = dict(kind=kind, index=k, ms=round(float(np.median(m)), 4), all_ms=[round(x, 4) for x in m],
                   offset_gb=round((t.data_ptr() - base) / 2 ** 30, 3) if kind == "arena" else None,
                   ptr=hex(t.data_ptr()))
        out.append(rec)
        print(json.dumps(rec), flush=True)
    arena_ms = [r["ms"] for r in out if r["kind"] == "arena"]
    alloc_ms = [r["ms"] for r in out if r["kind"] == "alloc"]
    print(json.dumps(dict(summary=True, model=a.model, dtype=a.dtype, rows=rows,
                          pool_gb=round(pool_elems * src.element_size() / 2 ** 30, 2),
                          plan=plan.spec, step_mb=a.step_mb, arena_ms=arena_ms, alloc_ms=alloc_ms, ballast_gb=a.ballast_gb,
                          arena_spread=round(max(arena_ms) / min(arena_ms), 3),
                          alloc_spread=round(max(alloc_ms) / min(alloc_ms), 3) if alloc_ms else None)), flush=True)
    del ballast


if __name__ == "__main__":
    main()
