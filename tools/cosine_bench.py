"""K2 (exact-order cosine) timing on BASELINE config 3's layout (not part of the product):
ResNet-50, one client vs its 8 neighbors (sim_centrality_module_avg's K2 launch), checked bit
for bit against the C oracle on the first pair at full size.  One JSON line."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402  (the checker)
from topology_aware_learning_amd import ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import ModelPool, StateLayout  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    lay = synth.get_layout(sys.argv[1] if len(sys.argv) > 1 else "resnet50")
    layout = StateLayout.from_layout(lay)
    segs = layout.param_segments(synth.param_names(lay))
    plan = ops.build_cosine_plan(segs)
    pool = ModelPool(layout, 9, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    pool.f32.normal_(generator=g)
    pool.f32[1:].mul_(0.3).add_(pool.f32[0:1])  # neighbors similar to the client
    a = [pool.row_f32(0)] * 8
    b = [pool.row_f32(j) for j in range(1, 9)]
    out = ops.cosine(a, b, plan)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        s.record()
        ops.cosine(a, b, plan)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ref = oracle.cosine_model(pool.row_f32(0).cpu().numpy(), pool.row_f32(1).cpu().numpy(), segs)
    got = out[0].cpu().numpy()
    print(json.dumps(dict(layout=sys.argv[1] if len(sys.argv) > 1 else "resnet50", pairs=8,
                          ms=round(float(np.median(ts)), 4), values=[float(x) for x in out.cpu()],
                          bitwise_vs_oracle_pair0=bool(got.view(np.uint32) == ref.view(np.uint32)),
                          params=layout.n_f32, tensors=len(segs), n_chunks=plan.n_chunks)), flush=True)


if __name__ == "__main__":
    main()
