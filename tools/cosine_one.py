"""K2 on one tensor shape (not part of the product): 8 pairs of random rows holding one
parameter of the given shape, the one-tensor cosine plan run `reps` times (for rocprofv3 PMC
passes and kernel traces).  usage: python tools/cosine_one.py [A,I,kh,kw] [reps]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from topology_aware_learning_amd import ops  # noqa: E402


def main():
    shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "512,512,3,3").split(","))
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = int(np.prod(shape))
    seg = (0, shape[0], shape[1] if len(shape) > 1 else 1, int(np.prod(shape[2:])) if len(shape) > 2 else 1)
    g = torch.Generator(device="cuda").manual_seed(0)
    rows = torch.randn(9, n, device="cuda", generator=g)
    plan = ops.build_cosine_plan([seg])
    a, b = [rows[0]] * 8, [rows[1 + j] for j in range(8)]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        ops.cosine(a, b, plan)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    print(f"shape={shape} seg={seg} n_chunks={plan.n_chunks} ms_median={float(np.median(ts)):.4f}", flush=True)


if __name__ == "__main__":
    main()
