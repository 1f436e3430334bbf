"""GPU: rounds with a row of more distinct sources than one LDS tile holds (the reference's
`unweighted_fl` strategy - every other client a neighbor, decentralized_app.py:386-389 - over
> ~620 clients).  fp32 pools take the streamed form, bf16 pools one K1 call per row; either way
RoundExecutor's round equals the per-call oracle on the pre-round snapshot, bit for bit."""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from topology_aware_learning_amd import ops
from topology_aware_learning_amd.arena import ModelPool, StateLayout
from topology_aware_learning_amd.round import RoundExecutor

pytestmark = pytest.mark.gpu

N_CLIENTS = 700


def _fl_round():
    g = nx.complete_graph(N_CLIENTS)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(N_CLIENTS)]
    return orders, [[1.0 / len(o)] * len(o) for o in orders]


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_unweighted_fl_round_700_clients(cuda, dtype):
    lay = StateLayout.from_layout([("w", (1000,), dtype), ("b", (7,), dtype), ("n", (), "int64")])
    pool = ModelPool(lay, N_CLIENTS, cuda)
    g = torch.Generator(device=cuda).manual_seed(3)
    pool.f32.normal_(generator=g)
    pool.b16.copy_(torch.randn(pool.b16.shape, generator=g, device=cuda))
    pool.i64.random_(0, 10 ** 6, generator=g)
    orders, ws = _fl_round()
    seg = "b16" if dtype == "bfloat16" else "f32"
    n = lay.n_b16 if seg == "b16" else lay.n_f32
    if seg == "b16":
        x = pool.b16[:, :n].view(torch.int16).cpu().numpy().view(np.uint16)
    else:
        x = pool.f32[:, :n].cpu().numpy()
    xi = pool.i64[:, :lay.n_i64].cpu().numpy()
    ex = RoundExecutor(pool, placement_trials=1)
    plan = ex.plan(orders, ws, list(range(N_CLIENTS)))
    assert ops.round_kernel_name(plan) == ("k_round_stream" if seg == "f32" else "k_agg (one call per row)")
    ex.run(orders, ws)
    torch.cuda.synchronize()
    got = getattr(pool, seg)[:, :n].cpu()
    got_i = pool.i64[:, :lay.n_i64].cpu().numpy()
    for r in (0, 1, N_CLIENTS // 2, N_CLIENTS - 1):
        xs = [x[j] for j in orders[r]]
        if seg == "f32":
            exp = oracle.agg_f32(xs, ws[r])
            assert np.array_equal(exp.view(np.uint32), got[r].numpy().view(np.uint32)), r
        else:
            exp = oracle.agg_bf16(xs, ws[r], exact=True)
            assert np.array_equal(exp, got[r].view(torch.int16).numpy().view(np.uint16)), r
        exp_i = oracle.agg_i64([xi[j] for j in orders[r]], ws[r])
        assert np.array_equal(exp_i, got_i[r]), r
