"""K3r (tal_agg_round_reg): rounds over register-resident source groups, against the oracle.

The kernel reads each group's sources from VGPRs through the VGPR index mode; these tests pin
it bit for bit: fp32 EXACT against oracle.round_f32 (the reference's arithmetic,
decentralized_client.py:399-413), fp32 FMA and bf16 FMA against K1 in the same mode row by
row (same fused chain), on the config-5 topology (SBM, 8 x 32, max 64 sources per group) and on
graphs whose groups need 1, 2 or 3 register blocks, at piece-boundary widths (n = 1, 127, 128,
129, odd n), per-operand weights, fp32 specials, padded and permuted output rows.
"""
from __future__ import annotations

import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from _pools import dev_rows, host
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops

pytestmark = pytest.mark.gpu


def _sbm(blocks=8, size=32, seed=0):
    p = [[14 / 31 if a == b else 2 / 224 for b in range(blocks)] for a in range(blocks)]
    return nx.stochastic_block_model([size] * blocks, p, seed=seed)


_GRAPHS = {
    "sbm256": lambda: _sbm(),
    "sbm64": lambda: _sbm(4, 16, 3),
    "regular12": lambda: nx.random_regular_graph(4, 12, seed=1),       # one block (<= 16 sources)
    "regular40": lambda: nx.random_regular_graph(6, 40, seed=2),       # groups of <= 32 / 48
    "ring9": lambda: nx.cycle_graph(9),                                 # an odd row count (a lone row)
}


def _csr(g, weights="unweighted"):
    orders, ws = [], []
    cent = nx.degree_centrality(g)
    for i in sorted(g.nodes):
        o = sorted(g.neighbors(i)) + [i]
        orders.append(o)
        ws.append(ra.unweighted_weights(len(o)) if weights == "unweighted" else ra.centrality_weights(o, cent, True, 10.0))
    row_ptr, col, w = ra.round_csr(orders, ws)
    return orders, ws, row_ptr, col, w


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


def _pool(rng, rows, n, special=False):
    x = (rng.standard_normal((rows, n)) * 3).astype(np.float32)
    if special and n > 8:
        x[0, :5] = [1e-40, -0.0, 3e38, -1e-45, 65504.0]
        x[1, :3] = [-0.0, -0.0, 1e-38]
    return x


@pytest.mark.parametrize("graph,n", [("sbm256", 129), ("sbm256", 8195), ("sbm64", 1), ("sbm64", 127),
                                     ("sbm64", 128), ("regular12", 1000), ("regular40", 4097), ("ring9", 300)])
@pytest.mark.parametrize("weights", ["unweighted", "degcent"])
def test_reg_round_exact_vs_oracle(cuda, graph, n, weights):
    g = _GRAPHS[graph]()
    orders, ws, row_ptr, col, w = _csr(g, weights)
    rows = len(orders)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = ops.build_reg_plan(row_ptr, col, w, out_rows)
    assert plan is not None and plan.max_src <= 64
    rng = np.random.default_rng(n + rows)
    pool = _pool(rng, rows, n, special=True)
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    for pad in (True, False):  # even row stride (K3r) / odd n contiguous (K3r or the full plan)
        pin = dev_rows(pool, cuda, pad)
        pout = torch.full_like(pin, float("nan"))
        ops.round_f32(pin, pout, plan, n=n)
        assert _bits_equal(host(pout, n), ref), pad


def test_reg_round_groups_use_every_register_block():
    """The grouping: SBM-256 needs the 64-source groups (4 register blocks); the small graphs
    exercise groups of <= 16, <= 32 and <= 48 sources (1, 2, 3 blocks)."""
    got = set()
    for name in _GRAPHS:
        _, _, row_ptr, col, w = _csr(_GRAPHS[name]())
        rows = len(row_ptr) - 1
        for cap in (16, 32, 48, 64):
            p = ops.build_reg_plan(row_ptr, col, w, np.arange(rows, dtype=np.int32), max_src=cap)
            if p is not None:
                got.add((p.max_src + 15) // 16)
    assert got == {1, 2, 3, 4}


@pytest.mark.parametrize("cap", [16, 32, 48, 64])
def test_reg_round_each_block_count(cuda, cap):
    """The same round built with groups of <= cap sources (NB = cap / 16 register blocks) is
    bitwise the oracle for each kernel instantiation."""
    orders, ws, row_ptr, col, w = _csr(_GRAPHS["regular40" if cap < 64 else "sbm64"]())
    rows = len(orders)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = ops.build_reg_plan(row_ptr, col, w, out_rows, max_src=cap)
    assert plan is not None and (plan.max_src + 15) // 16 == cap // 16
    pool = _pool(np.random.default_rng(cap), rows, 3001)
    pin = dev_rows(pool, cuda)  # an even row stride: K3r itself (odd rows take the full plan)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=3001)
    assert _bits_equal(host(pout, 3001), oracle.round_f32(pool, row_ptr, col, w, out_rows))


@pytest.mark.parametrize("graph", ["sbm256", "regular40"])
def test_reg_round_fma_equals_k1_fma(cuda, graph):
    orders, ws, row_ptr, col, w = _csr(_GRAPHS[graph](), "degcent")
    rows = len(orders)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = ops.build_reg_plan(row_ptr, col, w, out_rows)
    n = 1031
    pin = torch.from_numpy(_pool(np.random.default_rng(7), rows, n)).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, mode=ops.MODE_FMA)
    chk = torch.empty(n, device=cuda)
    for r in range(rows):
        ops.agg_f32([pin[j] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
        assert torch.equal(chk.view(torch.int32), pout[r].view(torch.int32)), r


@pytest.mark.parametrize("n", [129, 5001])
def test_reg_round_bf16_fma_equals_k1(cuda, n):
    """bf16 pools, FMA mode (BASELINE config 5's bf16 run): every row bitwise K1-bf16-FMA on the
    same operands (fp32 fused chain, one rounding, NaN stored as 0xFFFF); bf16 EXACT takes the
    full plan (narrow kernel) and is bitwise the bf16 oracle."""
    orders, ws, row_ptr, col, w = _csr(_GRAPHS["sbm256"]())
    rows = len(orders)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = ops.build_reg_plan(row_ptr, col, w, out_rows)
    x = torch.from_numpy(_pool(np.random.default_rng(n), rows, n)).to(torch.bfloat16)
    x[3, 0] = float("nan")
    pin = x.to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_bf16(pin, pout, plan, mode=ops.MODE_FMA)
    chk = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    for r in range(rows):
        ops.agg_bf16([pin[j] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
        assert torch.equal(chk.view(torch.int16), pout[r].view(torch.int16)), r
    ops.round_bf16(pin, pout, plan, mode=ops.MODE_EXACT)
    ref = oracle.round_bf16(pin.cpu().view(torch.int16).numpy().view(np.uint16), row_ptr, col, w, out_rows)
    assert np.array_equal(pout.cpu().view(torch.int16).numpy().view(np.uint16), ref)


def test_reg_round_padded_permuted_rows(cuda):
    """Pools with a pitch beyond n (odd n: the last lane reads one padding element) and an
    output permutation; rows not in the round keep their bytes."""
    orders, ws, row_ptr, col, w = _csr(_GRAPHS["sbm64"]())
    rows = len(orders)
    perm = np.random.default_rng(1).permutation(rows + 5)[:rows].astype(np.int32)
    plan = ops.build_reg_plan(row_ptr, col, w, perm)
    n, ld = 1001, 1088
    base = torch.from_numpy(_pool(np.random.default_rng(2), rows, ld)).to(cuda)
    pout = torch.full((rows + 5, ld), 7.0, device=cuda)
    ops.round_f32(base, pout, plan, n=n)
    ref = oracle.round_f32(base[:, :n].cpu().numpy(), row_ptr, col, w, np.arange(rows, dtype=np.int32))
    got = pout.cpu().numpy()
    assert _bits_equal(got[perm, :n], ref)
    untouched = np.setdiff1d(np.arange(rows + 5), perm)
    assert np.all(got[untouched] == 7.0) and np.all(got[perm, n:] == 7.0)


def test_reg_plan_spec_roundtrip_and_i64(cuda):
    """plan_from_spec({'reg': 1}) rebuilds the plan; the int64 segment runs the full plan."""
    orders, ws, row_ptr, col, w = _csr(_GRAPHS["sbm64"]())
    rows = len(orders)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = ops.plan_from_spec(row_ptr, col, w, out_rows, {"reg": 1})
    assert isinstance(plan, ops.RegPlan) and ops.round_kernel_name(plan) == "k_round_reg"
    xi = np.random.default_rng(4).integers(0, 10 ** 6, size=(rows, 53)).astype(np.int64)
    iin = torch.from_numpy(xi).to(cuda)
    iout = torch.zeros_like(iin)
    ops.round_i64(iin, iout, plan)
    assert np.array_equal(iout.cpu().numpy(), oracle.round_i64(xi, row_ptr, col, w, out_rows))


def test_round_executor_bf16_fma_per_operand_weights(cuda):
    """The product's untimed default for a bf16 FMA round with per-operand (degree-centrality)
    weights is the narrow kernel's broadcast form since round 4 (ops.default_plan; K3r before):
    RoundExecutor on bf16 model rows of the SBM-256 topology runs it in place (one group, no
    scratch pool), every row bitwise the bf16 FMA oracle (fp32 fused chain, one rounding), the
    int64 segment through the plan's scalar form, bitwise the oracle's truncation."""
    from topology_aware_learning_amd.arena import ModelPool, StateLayout
    from topology_aware_learning_amd.round import RoundExecutor

    orders, ws, row_ptr, col, w = _csr(_GRAPHS["sbm256"](), weights="degcent")
    rows = len(orders)
    lay = StateLayout.from_layout([("w", [1003], "bfloat16"), ("n", [3], "int64")])
    pool = ModelPool(lay, rows, cuda)
    rng = np.random.default_rng(5)
    x = torch.from_numpy(_pool(rng, rows, lay.n_b16)).to(torch.bfloat16)
    xi = torch.from_numpy(rng.integers(0, 10 ** 6, (rows, lay.n_i64)))
    pool.b16[:, :lay.n_b16].copy_(x.to(cuda))
    pool.i64[:, :lay.n_i64].copy_(xi.to(cuda))
    ex = RoundExecutor(pool, mode=ops.MODE_FMA)
    plan = ex.plan(orders, ws, list(range(rows)))
    assert isinstance(plan, ops.RoundPlan) and plan.info.narrow_bcast and plan.single_group
    bits = x.view(torch.int16).numpy().view(np.uint16)
    ref = oracle.round_bf16(bits, row_ptr, col, w, np.arange(rows, dtype=np.int32), exact=False)
    iref = oracle.round_i64(xi.numpy(), row_ptr, col, w, np.arange(rows, dtype=np.int32))
    ex.run(orders, ws)
    torch.cuda.synchronize(cuda)
    got = pool.b16[:, :lay.n_b16].cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(got, ref)
    assert np.array_equal(pool.i64[:, :lay.n_i64].cpu().numpy(), iref)
