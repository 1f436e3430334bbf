"""Run one round plan form a few times (profiling driver, not a benchmark).

usage: python tools/run_round.py --graph sbm --devices 256 --model vit_b16 --c4 16 --lds 163840 [--steps 5]
       (--stream-rows R for a streamed plan; --dense 8 for dense row blocks)
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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    layout = StateLayout.from_layout(synth.get_layout(a.model))
    orders, weights = bench.round_spec(a.devices, a.degree, kind=a.graph)
    rows = len(orders)
    row_ptr, col, w = bench._round_csr(orders, weights)
    out_rows = np.arange(rows, dtype=np.int32)
    if a.stream_rows:
        plan = ops.build_stream_plan(row_ptr, col, w, out_rows, a.stream_rows)
    else:
        plan = ops.build_plan(row_ptr, col, w, out_rows, c4=a.c4, lds_bytes=a.lds, dense=a.dense)
    plan.to(dev)
    i = plan.info
    print(f"plan c4={i.c4} groups={i.n_groups} staged={i.total_src} max_src={i.max_src} dense_rb={i.dense_rb} "
          f"stream_cs={i.stream_cs} lds={i.lds_bytes} kernel={ops.round_kernel_name(i)}", flush=True)
    pin = ModelPool(layout, rows, dev)
    pout = ModelPool(layout, rows, dev)
    bench.fill_pool(pin, 1)
    ops.round_f32(pin.f32, pout.f32, plan, n=layout.n_f32)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(a.steps):
        s.record()
        ops.round_f32(pin.f32, pout.f32, plan, n=layout.n_f32)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ms = float(np.mean(ts))
    gb = 4.0 * layout.n_f32 * (i.total_src + rows) / 1e9
    print(f"kernel {ms:.3f} ms  {gb / ms:.1f} TB/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
