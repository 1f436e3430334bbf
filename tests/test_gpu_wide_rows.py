"""GPU: rounds with a row of more distinct sources than one LDS tile holds (the reference's
`unweighted_fl` strategy - every other client a neighbor, decentralized_app.py:386-389 - over
> ~620 clients).  fp32 pools take the streamed form (k_round_stream), bf16 pools the wide-row form
(k_round_wide, round 6; round 5 ran one K1 call per row); either way RoundExecutor's round equals
the per-call oracle on the pre-round snapshot, bit for bit (bf16: EXACT and FMA)."""
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
    assert ops.round_kernel_name(plan, bf16=seg == "b16") == ("k_round_stream" if seg == "f32" else "k_round_wide")
    ex.run(orders, ws)
    torch.cuda.synchronize()
    got = getattr(pool, seg)[:, :n].cpu()
    got_i = pool.i64[:, :lay.n_i64].cpu().numpy()
    for r in (0, 1, 15, 16, 17, N_CLIENTS // 2, N_CLIENTS - 2, N_CLIENTS - 1):
        xs = [x[j] for j in orders[r]]
        if seg == "f32":
            exp = oracle.agg_f32(xs, ws[r])
            assert np.array_equal(exp.view(np.uint32), got[r].numpy().view(np.uint32)), r
        else:
            exp = oracle.agg_bf16(xs, ws[r], exact=True)
            assert np.array_equal(exp, got[r].view(torch.int16).numpy().view(np.uint16)), r
        exp_i = oracle.agg_i64([xi[j] for j in orders[r]], ws[r])
        assert np.array_equal(exp_i, got_i[r]), r


@pytest.mark.parametrize("m", [257, 600])
@pytest.mark.parametrize("kind", ["bf16_exact", "bf16_fma", "i64", "f32"])
def test_k1_past_256_operands(cuda, kind, m):
    """K1 (the per-call path) on more operands than one kernel-argument table holds: bitwise the
    oracle's single ordered chain, with out aliasing the last operand (the app's own model)."""
    rng = np.random.default_rng(m)
    n = 3001
    w = rng.uniform(0.0, 2.0 / m, m)
    if kind == "i64":
        x = rng.integers(-10 ** 6, 10 ** 6, (m, n)).astype(np.int64)
        exp = oracle.agg_i64(list(x), w)
        dev = torch.from_numpy(x).to(cuda)
        ops.agg_i64([dev[j] for j in range(m)], w.tolist(), dev[m - 1])
        got = dev[m - 1].cpu().numpy()
        assert np.array_equal(got, exp)
        return
    if kind == "f32":
        x = rng.standard_normal((m, n)).astype(np.float32)
        exp = oracle.agg_f32(list(x), w)
        dev = torch.from_numpy(x).to(cuda)
        ops.agg_f32([dev[j] for j in range(m)], w.tolist(), dev[m - 1])
        assert np.array_equal(dev[m - 1].cpu().numpy().view(np.uint32), exp.view(np.uint32))
        return
    exact = kind == "bf16_exact"
    bits = oracle.f32_to_bf16(rng.standard_normal((m, n)).astype(np.float32))
    exp = oracle.agg_bf16(list(bits), w, exact=exact)
    dev = torch.from_numpy(bits.view(np.int16)).to(cuda).view(torch.bfloat16)
    ops.agg_bf16([dev[j] for j in range(m)], w.tolist(), dev[m - 1], mode=ops.MODE_EXACT if exact else ops.MODE_FMA)
    got = dev[m - 1].view(torch.int16).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, exp)


def test_pool_rows_app_past_256_operands(cuda):
    """The per-call app path on pool rows (agg_pool_rows) with 300 operands of a ResNet-like
    fp32 + int64 layout: bitwise the oracle (fp32 chain and int64 truncation)."""
    m = 300
    lay = StateLayout.from_layout([("w", (2000,), "float32"), ("n", (), "int64")])
    pool = ModelPool(lay, m, cuda)
    g = torch.Generator(device=cuda).manual_seed(9)
    pool.f32.normal_(generator=g)
    pool.i64.random_(0, 10 ** 6, generator=g)
    x = pool.f32[:, :lay.n_f32].cpu().numpy()
    xi = pool.i64[:, :lay.n_i64].cpu().numpy()
    w = [1.0 / m] * m
    ops.agg_pool_rows(pool, list(range(m)), w, m - 1)
    exp = oracle.agg_f32(list(x), w)
    exp_i = oracle.agg_i64(list(xi), w)
    assert np.array_equal(pool.f32[m - 1, :lay.n_f32].cpu().numpy().view(np.uint32), exp.view(np.uint32))
    assert np.array_equal(pool.i64[m - 1, :lay.n_i64].cpu().numpy(), exp_i)


@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("n", [4099, 64 * 4 + 2])
def test_wide_rows_bf16_dense_graph(cuda, exact, n):
    """k_round_wide on a dense random graph of 660 clients (rows of 300-420 operands, several
    64-source chunks per group), output rows permuted, odd widths (the n % 4 tail by the direct kernel), per-operand
    weights: every row bitwise the oracle's per-call bf16 aggregation on the snapshot."""
    rng = np.random.default_rng(n + exact)
    nc = 660
    g = nx.gnp_random_graph(nc, 0.55, seed=5)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(nc)]
    ws = [list(rng.uniform(0.1, 1.0, len(o)) / len(o)) for o in orders]
    lay = StateLayout.from_layout([("w", (n,), "bfloat16")])
    pin = ModelPool(lay, nc, cuda)
    pout = ModelPool(lay, nc, cuda)
    bits = oracle.f32_to_bf16(rng.standard_normal((nc, n)).astype(np.float32))
    pin.b16[:, :n].view(torch.int16).copy_(torch.from_numpy(bits.view(np.int16)))
    out_rows = rng.permutation(nc).astype(np.int32)
    from topology_aware_learning_amd.round import csr_from_lists

    rp, col, w = csr_from_lists(orders, ws)
    plan = ops.build_stream_plan(rp, col, w, out_rows, max_group_rows=ops.WIDE_ROWS)  # the form default_plan
    assert plan.info.stream_cs and plan.info.max_rows <= ops.WIDE_ROWS and plan.info.n_groups > 1  # takes past a tile
    ops.round_bf16(pin.b16, pout.b16, plan, n=n, mode=ops.MODE_EXACT if exact else ops.MODE_FMA)
    torch.cuda.synchronize()
    got = pout.b16[:, :n].view(torch.int16).cpu().numpy().view(np.uint16)
    for r in list(range(0, nc, 37)) + [nc - 1]:
        exp = oracle.agg_bf16([bits[j] for j in orders[r]], ws[r], exact=exact)
        assert np.array_equal(exp, got[out_rows[r]]), r
