"""Run one round plan form a few times (profiling driver, not a benchmark).

usage: python tools/run_round.py --graph sbm --devices 256 --model vit_b16 --c4 16 --lds 163840 [--steps 5]
       (--stream-rows R for a streamed plan; --dense 8 for dense row blocks; --plan JSON for a
       plan spec as bench.py --plan takes it, --dtype bf16 --mode fma for the bf16 tolerance run,
       --fill randn to fill the input pool with torch.randn instead of bench.fill_pool)
Prints the plan and the mean kernel time; rocprofv3 runs wrap it.
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from topology_aware_learning_amd import ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import ModelPool, StateLayout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="random")
    ap.add_argument("--devices", type=int, default=64)
    ap.add_argument("--degree", type=int, default=8)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--c4", type=int, default=64)
    ap.add_argument("--lds", type=int, default=160 * 1024)
    ap.add_argument("--dense", type=int, default=0)
    ap.add_argument("--stream-rows", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--plan", default="")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--mode", default="exact", choices=["exact", "fma"])
    ap.add_argument("--fill", default="pool", choices=["pool", "randn"])
    ap.add_argument("--in-place", action="store_true", help="round in place on the input pool (single-group plans)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lay = synth.get_layout(a.model)
    layout = StateLayout.from_layout(synth.as_bf16(lay) if a.dtype == "bf16" else lay)
    mode = ops.MODE_FMA if a.mode == "fma" else ops.MODE_EXACT
    orders, weights = bench.round_spec(a.devices, a.degree, kind=a.graph)
    rows = len(orders)
    row_ptr, col, w = bench._round_csr(orders, weights)
    out_rows = np.arange(rows, dtype=np.int32)
    if a.plan:
        import json
        plan = ops.plan_from_spec(row_ptr, col, w, out_rows, json.loads(a.plan))
    elif a.stream_rows:
        plan = ops.build_stream_plan(row_ptr, col, w, out_rows, a.stream_rows)
    else:
        plan = ops.build_plan(row_ptr, col, w, out_rows, c4=a.c4, lds_bytes=a.lds, dense=a.dense)
    plan.to(dev)
    i = plan.info
    print(f"plan c4={i.c4} groups={i.n_groups} staged={i.total_src} max_src={i.max_src} dense_rb={i.dense_rb} "
          f"stream_cs={i.stream_cs} lds={i.lds_bytes} kernel={ops.round_kernel_name(i)}", flush=True)
    pin = ModelPool(layout, rows, dev)
    pout = pin if a.in_place else ModelPool(layout, rows, dev)
    if a.fill == "randn":
        for _, t, _ in pin.segments():
            if t.dtype.is_floating_point:
                t.normal_()
    else:
        bench.fill_pool(pin, 1)
    seg, n = ("b16", layout.n_b16) if a.dtype == "bf16" else ("f32", layout.n_f32)
    fn = ops.round_bf16 if a.dtype == "bf16" else ops.round_f32

    def run():
        fn(getattr(pin, seg), getattr(pout, seg), plan, n=n, mode=mode)

    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(a.steps):
        s.record()
        run()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ms = float(np.mean(ts))
    gb = (2.0 if a.dtype == "bf16" else 4.0) * n * (i.total_src + rows) / 1e9
    print(f"kernel {ms:.3f} ms  {gb / ms:.1f} TB/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
