"""Probe (not part of the product): why does the config-3 round run ~2.0 or ~2.4 ms depending
on which allocation it writes?  One input pool and K output pools of config 3's size; the round
(c4 = 64 sparse plan) is timed into each, `reps` launches per pool in a fixed order, and each
launch's time is printed as one JSON line so a rocprofv3 --pmc pass of this same process
(same allocations) can be matched launch by launch (profiles/scripts_r01_r02/gpu_placement.sh).

Usage: python tools/placement_probe.py [K] [reps]"""
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

    k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    n, ld = lay.n_f32, lay.ld_f32
    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    rp, col, w = csr_from_lists(orders, [[1 / 9] * 9] * 64)
    dev = torch.device("cuda", 0)
    plan = ops.plan_from_spec(rp, col, w, np.arange(64, dtype=np.int32),
                              {"c4": 64, "lds": 81920, "dense": 0}).to(dev)
    src = torch.randn(64, ld, device=dev)
    outs = [torch.empty(64, ld, device=dev) for _ in range(k)]
    for o in outs:
        o.zero_()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ops.round_f32(src, outs[0], plan, n=n)  # warm
    torch.cuda.synchronize()
    launch = 0
    for rep in range(reps):
        for i, o in enumerate(outs):
            s.record()
            ops.round_f32(src, o, plan, n=n)
            e.record()
            e.synchronize()
            print(json.dumps(dict(launch=launch, pool=i, rep=rep, ms=round(s.elapsed_time(e), 4),
                                  base=hex(o.data_ptr()))), flush=True)
            launch += 1
    # sequential streaming write of each pool (fill) and read (sum) for contrast
    for i, o in enumerate(outs):
        o.fill_(1.0)
        s.record()
        o.fill_(2.0)
        e.record()
        e.synchronize()
        wr = o.numel() * 4 / (s.elapsed_time(e) * 1e-3) / 1e9
        print(json.dumps(dict(pool=i, fill_GBps=round(wr, 1))), flush=True)


if __name__ == "__main__":
    main()
