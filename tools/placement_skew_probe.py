"""Probe (not part of the product): can the output pool's layout remove the config-3 placement
lottery?  K output allocations, each with slack; into each, the round
(c4 = 64 sparse plan, the bench's plan for config 3) writes pools that start at a byte offset
inside the allocation (0 .. 2 MiB) and/or use a skewed row pitch (ld + 64 / + 1024 elements:
every row start rotated across channels).  A layout that is fast in every allocation makes the
placement deterministic; one JSON line per (allocation, offset, pitch) with the mean of 3
launches.

Usage: python tools/placement_skew_probe.py [K]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from topology_aware_learning_amd import ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import StateLayout  # noqa: E402
from topology_aware_learning_amd.round import csr_from_lists  # noqa: E402


def main():
    import networkx as nx

    k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    n, ld = lay.n_f32, lay.ld_f32
    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    rp, col, w = csr_from_lists(orders, [[1 / 9] * 9] * 64)
    dev = torch.device("cuda", 0)
    plan = ops.plan_from_spec(rp, col, w, np.arange(64, dtype=np.int32),
                              {"c4": 64, "lds": 81920, "dense": 0}).to(dev)
    src = torch.randn(64, ld, device=dev)
    offsets = [0, 64, 1024, 16384, 262144, 524288]  # elements: 0, 256 B, 4 KiB, 64 KiB, 1 MiB, 2 MiB
    pitches = [ld, ld + 64, ld + 1024]
    slack = max(offsets) + 64 * (max(pitches) - ld) + 1024
    bufs = [torch.zeros(64 * ld + slack, device=dev) for _ in range(k)]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ref = torch.empty(64, ld, device=dev)
    ops.round_f32(src, ref, plan, n=n)
    torch.cuda.synchronize()
    for i, b in enumerate(bufs):
        for off in offsets:
            for pitch in pitches:
                out = torch.as_strided(b, (64, pitch), (pitch, 1), off)
                ops.round_f32(src, out, plan, n=n)  # warm
                s.record()
                for _ in range(3):
                    ops.round_f32(src, out, plan, n=n)
                e.record()
                e.synchronize()
                ok = bool(torch.equal(out[:, :n], ref[:, :n]))
                print(json.dumps(dict(alloc=i, off_B=4 * off, pitch_skew=pitch - ld, ms=round(s.elapsed_time(e) / 3, 4),
                                      base=hex(b.data_ptr()), ok=ok)), flush=True)


if __name__ == "__main__":
    main()
