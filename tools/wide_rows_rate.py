"""bf16 rounds whose rows are wider than one LDS tile (not part of the product): the reference's
`unweighted_fl` over 700 clients (every other client a neighbor), CIFAR-CNN-sized bf16 rows
(5,851,338 elements), EXACT and FMA: the wide-row form (k_round_wide, the default since round 6)
against round 5's one K1 call per row (RowCallPlan), kernel time by HIP events.  One JSON line
per measurement.  --pmc: one EXACT launch of each form only, for a rocprofv3 --pmc FETCH_SIZE
pass (source reads once per group against once per row)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

from topology_aware_learning_amd import ops  # noqa: E402
from topology_aware_learning_amd.round import csr_from_lists  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    nc, n = 700, 5_851_338
    ld = (n + 63) // 64 * 64
    g = nx.complete_graph(nc)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(nc)]
    ws = [[1.0 / len(o)] * len(o) for o in orders]
    rp, col, w = csr_from_lists(orders, ws)
    rows = np.arange(nc, dtype=np.int32)
    pin = torch.randn(nc, ld, device=dev).to(torch.bfloat16)
    pout = torch.empty_like(pin)
    wide = ops.default_plan(rp, col, w, rows, bf16=True)
    percall = ops.row_call_plan(rp, col, w, rows)
    if "--pmc" in sys.argv:  # one EXACT launch of each form, nothing else (for rocprofv3 --pmc)
        ops.round_bf16(pin, pout, wide, n=n, mode=ops.MODE_EXACT)
        torch.cuda.synchronize()
        ops.round_bf16(pin, pout, percall, n=n, mode=ops.MODE_EXACT)
        torch.cuda.synchronize()
        print(json.dumps(dict(pmc_pass=True, groups=wide.info.n_groups,
                              wide_source_bytes=2 * n * nc * wide.info.n_groups,
                              per_row_source_bytes=2 * n * nc * nc, out_bytes=2 * n * nc)), flush=True)
        return
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for mode, name in ((ops.MODE_EXACT, "exact"), (ops.MODE_FMA, "fma")):
        res = {}
        for label, plan in (("wide", wide), ("k1_per_row", percall)):
            ops.round_bf16(pin, pout, plan, n=n, mode=mode)
            torch.cuda.synchronize()
            s.record()
            ops.round_bf16(pin, pout, plan, n=n, mode=mode)
            e.record()
            e.synchronize()
            res[label] = s.elapsed_time(e)
            if label == "wide":
                ref = pout.clone()
        same = bool(torch.equal(ref.view(torch.int16), pout.view(torch.int16)))
        src_bytes_wide = 2 * n * nc * wide.info.n_groups  # each source read once per group
        print(json.dumps(dict(mode=name, clients=nc, elements=n, groups=wide.info.n_groups, wide_ms=round(res["wide"], 3),
                              k1_per_row_ms=round(res["k1_per_row"], 3), speedup=round(res["k1_per_row"] / res["wide"], 1),
                              bitwise_equal=same, wide_source_GB=round(src_bytes_wide / 1e9, 1),
                              per_row_source_GB=round(2 * n * nc * nc / 1e9, 1))), flush=True)


if __name__ == "__main__":
    main()
