"""K2 time by tensor kind (not part of the product): the ResNet-50 cosine plan split into its
1-D (elementwise), row (B = 1: 1x1 convs, fc) and column (B > 1: 3x3 / 7x7 convs) tensors, and
per single tensor for the heaviest ones; one client against 8 neighbors, HIP events, median of
10.  One JSON line per plan.

usage: python tools/cosine_kinds.py [layout]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from topology_aware_learning_amd import ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import ModelPool, StateLayout  # noqa: E402


def timed(plan, a, b):
    ops.cosine(a, b, plan)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        s.record()
        ops.cosine(a, b, plan)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


def main():
    dev = torch.device("cuda", 0)
    lay = synth.get_layout(sys.argv[1] if len(sys.argv) > 1 else "resnet50")
    layout = StateLayout.from_layout(lay)
    segs = layout.param_segments(synth.param_names(lay))
    pool = ModelPool(layout, 9, dev)
    pool.f32.normal_()
    a = [pool.row_f32(0)] * 8
    b = [pool.row_f32(j) for j in range(1, 9)]
    kind = lambda s: "elem" if s[2] == 1 and s[3] == 1 else ("row" if s[3] == 1 else "col")  # noqa: E731
    groups = {"all": segs}
    for k in ("elem", "row", "col"):
        groups[k] = [s for s in segs if kind(s) == k]
    for name, g in groups.items():
        if not g:
            continue
        plan = ops.build_cosine_plan(g)
        print(json.dumps(dict(plan=name, tensors=len(g), params=int(sum(s[1] * s[2] * s[3] for s in g)),
                              n_chunks=plan.n_chunks, ms=round(timed(plan, a, b), 4))), flush=True)
    heavy = sorted(segs, key=lambda s: -s[1] * s[2] * s[3])[:6]
    for s in heavy:
        plan = ops.build_cosine_plan([s])
        print(json.dumps(dict(plan="one", kind=kind(s), A=int(s[1]), I=int(s[2]), B=int(s[3]), n_chunks=plan.n_chunks,
                              ms=round(timed(plan, a, b), 4))), flush=True)


if __name__ == "__main__":
    main()
