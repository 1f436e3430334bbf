"""GPU parity of the HIP kernels (through the C-ABI) against the C oracle.

Bar: bit-exact in EXACT mode (fp32 and int64), M*2^-24*sum|w x| in FMA mode.
"""
import hashlib
import json

import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from _pools import dev_rows, host
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops, synth
from topology_aware_learning_amd.arena import ModelPool, StateLayout
from topology_aware_learning_amd.round import RoundExecutor

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _rand_f32(rng, n, special=False):
    x = rng.standard_normal(n).astype(np.float32) * np.float32(3.0)
    if special and n > 8:
        x[0] = 1e-40
        x[1] = -0.0
        x[2] = 3e38
        x[3] = -1e-45
        x[4] = 65504.0
    return x


def _bits_equal(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype == np.float32:
        na, nb = np.isnan(a), np.isnan(b)
        assert np.array_equal(na, nb)
        return np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))
    return np.array_equal(a, b)


@pytest.mark.parametrize("m", [1, 2, 3, 4, 8, 9, 16, 17, 18, 33, 64, 65, 130, 256, 300])
@pytest.mark.parametrize("n", [1, 3, 4, 5, 1027, 262147])
def test_agg_f32_exact(cuda, m, n):
    rng = np.random.default_rng(m * 1000 + n)
    xs = [_rand_f32(rng, n, special=(i == 0)) for i in range(m)]
    w = rng.random(m)
    w = list(w / w.sum())
    ref = oracle.agg_f32(xs, w)
    dx = [torch.from_numpy(x).to(cuda) for x in xs]
    out = torch.empty(n, dtype=torch.float32, device=cuda)
    ops.agg_f32(dx, w, out)
    assert _bits_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("m", [1, 3, 9, 17, 70])
def test_agg_f32_in_place_self_last(cuda, m):
    """The aggregating client is the last operand and the output (decentralized_app.py:625)."""
    rng = np.random.default_rng(m)
    n = 100003
    xs = [_rand_f32(rng, n) for _ in range(m)]
    w = [1 / m] * m
    ref = oracle.agg_f32(xs, w)
    dx = [torch.from_numpy(x).to(cuda) for x in xs]
    ops.agg_f32(dx, w, dx[-1])
    assert _bits_equal(dx[-1].cpu().numpy(), ref)


def test_agg_f32_unaligned(cuda):
    rng = np.random.default_rng(5)
    n, m = 50001, 9
    base = [torch.from_numpy(_rand_f32(rng, n + 1)).to(cuda) for _ in range(m)]
    xs = [b[1:] for b in base]  # 4-byte offset: scalar path
    w = [1 / m] * m
    ref = oracle.agg_f32([x.cpu().numpy() for x in xs], w)
    out = torch.empty(n + 1, dtype=torch.float32, device=cuda)[1:]
    ops.agg_f32(xs, w, out)
    assert _bits_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("m", [2, 9, 17])
def test_agg_f32_fma_tolerance(cuda, m):
    rng = np.random.default_rng(11 + m)
    n = 200000
    xs = [_rand_f32(rng, n) for _ in range(m)]
    w = list(rng.random(m))
    ref = oracle.agg_f32(xs, w).astype(np.float64)
    dx = [torch.from_numpy(x).to(cuda) for x in xs]
    out = torch.empty(n, dtype=torch.float32, device=cuda)
    ops.agg_f32(dx, w, out, mode=ops.MODE_FMA)
    bound = m * 2.0 ** -24 * sum(abs(np.float32(wi) * x.astype(np.float64)) for wi, x in zip(w, xs))
    assert np.all(np.abs(out.cpu().numpy().astype(np.float64) - ref) <= 2 * bound + 1e-45)


@pytest.mark.parametrize("m", [1, 3, 9, 17, 200])
def test_agg_i64_truncation(cuda, m):
    rng = np.random.default_rng(m)
    n = 4099
    xs = [rng.integers(-(2 ** 40), 2 ** 40, size=n).astype(np.int64) for _ in range(m)]
    for x in xs:
        x[:10] = [0, 1, 7, 10, 1000, 123456789, 2 ** 24 + 1, 2 ** 31 + 5, -1000, 999]
    w = [1 / m] * m
    ref = oracle.agg_i64(xs, w)
    dx = [torch.from_numpy(x).to(cuda) for x in xs]
    out = torch.empty(n, dtype=torch.int64, device=cuda)
    ops.agg_i64(dx, w, out)
    assert np.array_equal(out.cpu().numpy(), ref)
    if m == 9:
        assert ref[4] == 999  # nine copies of 1000 at w=1/9 come back as 999


@pytest.mark.parametrize("m", [1, 2, 9, 17, 18, 40, 64, 65])
@pytest.mark.parametrize("n", [1, 3, 4, 7, 1024, 1026, 4096 * 4 + 2, 262147])
@pytest.mark.parametrize("n_i", [0, 53, 300])
def test_agg_model_f32_one_launch(cuda, m, n, n_i):
    """K1m (tal_agg_model_f32): fp32 segment + int64 segment of one call in one launch, bitwise
    the oracle for every n % 4 tail, a last block full of chunks (n / 4 a multiple of 256), small
    n, m past the fused limit (two segment launches), int64 truncation and specials."""
    rng = np.random.default_rng(m * 7919 + n + n_i)
    xs = [_rand_f32(rng, n, special=(i == 0)) for i in range(m)]
    xis = [rng.integers(-(2 ** 40), 2 ** 40, size=n_i).astype(np.int64) for _ in range(m)]
    for x in xis:
        x[:min(n_i, 3)] = [1000, 2 ** 31 + 5, -999][:min(n_i, 3)]
    w = list(rng.random(m))
    dx = [torch.from_numpy(x).to(cuda) for x in xs]
    dxi = [torch.from_numpy(x).to(cuda) for x in xis]
    out = torch.empty(n, dtype=torch.float32, device=cuda)
    out_i = torch.empty(n_i, dtype=torch.int64, device=cuda)
    ops.agg_model_f32(dx, dxi, w, out, out_i)
    assert _bits_equal(out.cpu().numpy(), oracle.agg_f32(xs, w))
    if n_i:
        assert np.array_equal(out_i.cpu().numpy(), oracle.agg_i64(xis, w))


@pytest.mark.parametrize("mode", [ops.MODE_EXACT, ops.MODE_FMA])
def test_agg_model_f32_in_place_and_fma(cuda, mode):
    """The aggregating model is the last operand and the output (both segments), and FMA mode
    equals agg_f32's FMA mode bit for bit."""
    rng = np.random.default_rng(3)
    n, n_i, m = 100003, 53, 9
    xs = [torch.from_numpy(_rand_f32(rng, n)).to(cuda) for _ in range(m)]
    xis = [torch.from_numpy(rng.integers(0, 10 ** 6, size=n_i)).to(cuda) for _ in range(m)]
    w = [1 / m] * m
    ref = torch.empty(n, device=cuda)
    ops.agg_f32(xs, w, ref, mode=mode)
    ref_i = torch.empty(n_i, dtype=torch.int64, device=cuda)
    ops.agg_i64(xis, w, ref_i)
    ops.agg_model_f32(xs, xis, w, xs[-1], xis[-1], mode=mode)
    assert torch.equal(xs[-1].view(torch.int32), ref.view(torch.int32))
    assert torch.equal(xis[-1], ref_i)


def test_agg_model_f32_unaligned_falls_back(cuda):
    rng = np.random.default_rng(8)
    n, m = 5001, 9
    base = [torch.from_numpy(_rand_f32(rng, n + 1)).to(cuda) for _ in range(m)]
    xs = [b[1:] for b in base]
    xis = [torch.from_numpy(rng.integers(0, 10 ** 6, size=20)).to(cuda) for _ in range(m)]
    w = [1 / m] * m
    out = torch.empty(n + 1, device=cuda)[1:]
    out_i = torch.empty(20, dtype=torch.int64, device=cuda)
    ops.agg_model_f32(xs, xis, w, out, out_i)
    assert _bits_equal(out.cpu().numpy(), oracle.agg_f32([x.cpu().numpy() for x in xs], w))
    assert np.array_equal(out_i.cpu().numpy(), oracle.agg_i64([x.cpu().numpy() for x in xis], w))


def _graph_csr(g, weights="unweighted"):
    orders, ws = [], []
    cent = nx.degree_centrality(g)
    for i in sorted(g.nodes):
        o = sorted(g.neighbors(i)) + [i]
        orders.append(o)
        if weights == "unweighted":
            ws.append(ra.unweighted_weights(len(o)))
        else:
            ws.append(ra.centrality_weights(o, cent, True, 10.0))
    return orders, ws


@pytest.mark.parametrize("dense", [0, 8])
@pytest.mark.parametrize("graph,n,c4,lds", [
    ("ring", 1000, 0, 0),
    ("regular", 4099, 64, ops.LDS_BUDGET),
    ("regular", 4099, 128, 160 * 1024),
    ("regular", 70001, 64, 24 * 1024),      # forces several row groups
    ("regular", 70001, 128, 40 * 1024),     # several groups, 2 float4 columns per lane
    ("regular", 1000003, 64, 48 * 1024),    # persistent kernel with J < 8
    ("barbell", 3001, 0, 0),
    ("complete", 515, 0, 160 * 1024),
])
def test_round_f32_vs_oracle(cuda, graph, n, c4, lds, dense):
    g = {
        "ring": nx.cycle_graph(16),
        "regular": nx.random_regular_graph(8, 64, seed=0),
        "barbell": nx.barbell_graph(12, 4),
        "complete": nx.complete_graph(40),
    }[graph]
    orders, ws = _graph_csr(g, "softmax" if graph == "regular" else "unweighted")
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    rng = np.random.default_rng(rows + n)
    pool = np.stack([_rand_f32(rng, n) for _ in range(rows)])
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=lds, dense=dense)
    assert plan.info.dense_rb == dense
    pin = dev_rows(pool, cuda)  # rows strided like ModelPool's: the vector kernel + scalar tail
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=n)
    assert _bits_equal(host(pout, n), ref)
    if plan.single_group:  # in place is snapshot-safe with one group
        ops.round_f32(pin, pin, plan, n=n)
        assert _bits_equal(host(pin, n), ref)


_NARROW_GRAPHS = {
    "ring": lambda: nx.cycle_graph(16),
    "regular": lambda: nx.random_regular_graph(8, 64, seed=0),
    "sbm": lambda: nx.stochastic_block_model([32] * 4, [[0.45 if a == b else 0.01 for b in range(4)] for a in range(4)], seed=0),
    "barbell": lambda: nx.barbell_graph(12, 4),
    "complete": lambda: nx.complete_graph(40),
    "gnp": lambda: nx.gnp_random_graph(150, 0.08, seed=2),
}


@pytest.mark.parametrize("pad", [True, False], ids=["vec", "scalar"])
@pytest.mark.parametrize("c4,lds", [(16, 160 * 1024), (32, 160 * 1024), (16, 80 * 1024), (32, 24 * 1024)])
@pytest.mark.parametrize("n", [4099, 70001])
@pytest.mark.parametrize("graph", list(_NARROW_GRAPHS))
def test_round_narrow_vs_oracle(cuda, graph, n, c4, lds, pad):
    """Narrow-tile kernel (c4 16 / 32: 64/c4 rows per wavefront, per-lane plan from LDS).  pad:
    rows strided by a multiple of 64 elements (the narrow kernel computes the float4 body, the
    scalar kernel the n % 4 tail) or contiguous odd rows (all by the scalar kernel)."""
    g = _NARROW_GRAPHS[graph]()
    orders, ws = _graph_csr(g, "softmax" if graph in ("regular", "gnp", "sbm") else "unweighted")
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.random.default_rng(rows).permutation(rows).astype(np.int32)
    rng = np.random.default_rng(rows + n + c4)
    pool = np.stack([_rand_f32(rng, n, special=(rows % 3 == 0)) for _ in range(rows)])
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    try:
        plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=lds)
    except ops._lib.TalError:  # a row alone does not fit this budget
        assert lds < 64 * 1024
        return
    assert plan.info.c4 == c4 and plan.info.dense_rb == 0
    assert ops.round_kernel_name(plan.info) == "k_round_f32_narrow"
    pin = dev_rows(pool, cuda, pad)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=n)
    assert _bits_equal(host(pout, n), ref)
    ops.round_f32(pin, pout, plan, n=n, mode=ops.MODE_FMA)
    m = max(len(o) for o in orders)
    fin = np.isfinite(ref)
    tol = m * 2.0 ** -24 * np.abs(np.where(np.isfinite(pool), pool, 0)).max() + 1e-30
    got = host(pout, n)
    assert np.max(np.abs(got[fin] - ref[fin])) <= tol
    if plan.single_group:
        ops.round_f32(pin, pin, plan, n=n)
        assert _bits_equal(host(pin, n), ref)


@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_round_narrow_row_uniform_weights_signed_zero(cuda, sign):
    """ROWW encoding (one weight per row): padding reads a zero tile chosen by the weight's sign
    so fl(w * 0) == -0 and -0 results survive (rows of all-zero and -0.0 inputs)."""
    g = nx.random_regular_graph(6, 40, seed=3)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(40)]
    ws = [[sign / len(o)] * len(o) for o in orders]
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    n = 4099
    rng = np.random.default_rng(7)
    pool = rng.standard_normal((rows, n)).astype(np.float32)
    pool[:, :4] = np.float32(-0.0)
    pool[::2, 4:8] = np.float32(0.0)
    pool[1::2, 4:8] = np.float32(-0.0)
    pool[:, 8] = np.float32(1e-45)
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    for c4 in (16, 32):
        plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=80 * 1024)
        assert plan.info.narrow_roww == 1
        pin = dev_rows(pool, cuda)  # the narrow (ROWW) kernel takes the body, the scalar one the tail
        pout = torch.zeros_like(pin)
        ops.round_f32(pin, pout, plan, n=n)
        assert _bits_equal(host(pout, n), ref), c4
        bits = oracle.f32_to_bf16(pool)
        refb = oracle.round_bf16(bits, row_ptr, col, w, out_rows, exact=True)
        pb = dev_rows(bits, cuda)
        ob = torch.zeros_like(pb)
        ops.round_bf16(pb, ob, plan, n=n)
        assert np.array_equal(host(ob, n), refb), c4
        # FMA mode: the accumulator starts at -0.0 and padding is fma(w, +-0, acc); bitwise
        # against the bf16 oracle's fused chain and, for fp32, against K1-FMA row by row
        refbf = oracle.round_bf16(bits, row_ptr, col, w, out_rows, exact=False)
        ops.round_bf16(pb, ob, plan, n=n, mode=ops.MODE_FMA)
        assert np.array_equal(host(ob, n), refbf), c4
        ops.round_f32(pin, pout, plan, n=n, mode=ops.MODE_FMA)
        chk = torch.empty(n, dtype=torch.float32, device=cuda)
        for r in range(rows):
            ops.agg_f32([pin[j, :n] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
            assert torch.equal(chk.view(torch.int32), pout[r, :n].view(torch.int32)), (c4, r)


@pytest.mark.parametrize("c4", [16, 32])
def test_round_narrow_sbm256_one_group(cuda, c4):
    """BASELINE config 5's topology (256-device SBM) fits one narrow group: each source read once.
    Unweighted, so the row-uniform-weight encoding runs (16-bit slots up to the zero tiles at
    slot 256 * c4, decoded by v_mad_u32_u16 incl. its high-half form); c4 = 16: two resident
    workgroups per CU (row extents from LDS), c4 = 32: one (extents in registers)."""
    sizes = [32] * 8
    p = [[14 / 31 if a == b else 2 / 224 for b in range(8)] for a in range(8)]
    g = nx.stochastic_block_model(sizes, p, seed=0)
    orders, ws = _graph_csr(g)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=160 * 1024)
    assert plan.info.narrow_roww == 1 and plan.info.c4 == c4
    if c4 == 16:
        assert plan.info.n_groups == 1 and plan.info.total_src == rows
    n = 8195
    rng = np.random.default_rng(5)
    pool = rng.standard_normal((rows, n)).astype(np.float32)
    pin = dev_rows(pool, cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=n)
    assert _bits_equal(host(pout, n), oracle.round_f32(pool, row_ptr, col, w, out_rows))


_STREAM_GRAPHS = {
    "ring": lambda: nx.cycle_graph(16),
    "regular": lambda: nx.random_regular_graph(8, 64, seed=0),
    "barbell": lambda: nx.barbell_graph(30, 4),
    "complete40": lambda: nx.complete_graph(40),
    "complete100": lambda: nx.complete_graph(100),
    "gnp": lambda: nx.gnp_random_graph(150, 0.08, seed=2),
}


@pytest.mark.parametrize("grouping", [(64, 0), (128, 0), (16, 24)])
@pytest.mark.parametrize("n", [4099, 70001])
@pytest.mark.parametrize("graph", list(_STREAM_GRAPHS))
def test_round_stream_vs_oracle(cuda, graph, n, grouping):
    g = _STREAM_GRAPHS[graph]()
    orders, ws = _graph_csr(g, "softmax" if graph in ("regular", "gnp") else "unweighted")
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.random.default_rng(rows).permutation(rows).astype(np.int32)
    rng = np.random.default_rng(rows + n)
    pool = np.stack([_rand_f32(rng, n, special=(rows % 3 == 0)) for _ in range(rows)])
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    plan = ops.build_stream_plan(row_ptr, col, w, out_rows, *grouping)
    assert plan.info.stream_cs in (16, 32) and ops.round_kernel_name(plan.info) == "k_round_stream"
    pin = dev_rows(pool, cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=n)
    assert _bits_equal(host(pout, n), ref)
    if plan.single_group:
        ops.round_f32(pin, pin, plan, n=n)
        assert _bits_equal(host(pin, n), ref)


def test_round_stream_large_and_fma(cuda):
    g = nx.barbell_graph(60, 8)
    orders, ws = _graph_csr(g)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    n = 1 << 20
    rng = np.random.default_rng(11)
    pool = rng.standard_normal((rows, n)).astype(np.float32)
    plan = ops.build_stream_plan(row_ptr, col, w, out_rows, 64, 0)
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan)
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    assert _bits_equal(pout.cpu().numpy(), ref)
    ops.round_f32(pin, pout, plan, mode=ops.MODE_FMA)
    m = max(len(o) for o in orders)
    tol = m * 2.0 ** -24 * np.abs(pool).max() * 1.0 + 1e-30
    assert np.max(np.abs(pout.cpu().numpy() - ref)) <= tol


def test_round_stream_padded_ld_tail_unaligned_i64(cuda):
    g = nx.barbell_graph(9, 2)
    orders, ws = _graph_csr(g)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)[::-1].copy()
    plan = ops.build_stream_plan(row_ptr, col, w, out_rows, 8, 0)
    assert plan.info.n_groups > 1
    n, ld = 1030, 1088
    rng = np.random.default_rng(4)
    pool = np.zeros((rows, ld), np.float32)
    pool[:, :n] = rng.standard_normal((rows, n)).astype(np.float32)
    ref = oracle.round_f32(pool[:, :n].copy(), row_ptr, col, w, out_rows)
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.full_like(pin, 7.0)
    ops.round_f32(pin, pout, plan, n=n)
    got = pout.cpu().numpy()
    assert _bits_equal(got[:, :n], ref)
    assert np.all(got[:, n:] == 7.0)
    pin2 = torch.from_numpy(np.ascontiguousarray(pool[:, :n + 1])).to(cuda)  # odd ld: scalar path
    pout2 = torch.zeros_like(pin2)
    ops.round_f32(pin2, pout2, plan, n=n)
    assert _bits_equal(pout2.cpu().numpy()[:, :n], ref)
    ipool = rng.integers(0, 10 ** 6, size=(rows, 53)).astype(np.int64)
    ipool[:, 0] = 1000
    iref = oracle.round_i64(ipool, row_ptr, col, w, out_rows)
    ipin = torch.from_numpy(ipool).to(cuda)
    ipout = torch.zeros_like(ipin)
    ops.round_i64(ipin, ipout, plan)
    assert np.array_equal(ipout.cpu().numpy(), iref)


def test_round_gossip_matrix(cuda):
    """A reference gossip matrix (Metropolis weights) run as a device round: K3 resident and
    streamed plans are bitwise the oracle, and the oracle is W . X within fp32 rounding."""
    from topology_aware_learning_amd import gossip
    g = nx.barabasi_albert_graph(60, 3, seed=1)
    W = gossip.gossip_matrix(g).double().numpy()
    orders, weights = gossip.orders_from_matrix(W)
    row_ptr, col, w = ra.round_csr(orders, weights)
    out_rows = np.arange(len(W), dtype=np.int32)
    rng = np.random.default_rng(21)
    X = rng.standard_normal((len(W), 10007)).astype(np.float32)
    ref = oracle.round_f32(X, row_ptr, col, w, out_rows)
    pin = dev_rows(X, cuda)
    for plan in (ops.build_plan(row_ptr, col, w, out_rows), ops.build_stream_plan(row_ptr, col, w, out_rows)):
        pout = torch.zeros_like(pin)
        ops.round_f32(pin, pout, plan, n=10007)
        assert _bits_equal(host(pout, 10007), ref)
    bound = np.abs(W) @ np.abs(X.astype(np.float64)) * 64 * 2.0 ** -24
    assert np.all(np.abs(ref - W @ X.astype(np.float64)) <= bound)


def test_round_f32_padded_ld_and_tail(cuda):
    g = nx.random_regular_graph(4, 20, seed=1)
    orders, ws = _graph_csr(g)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(20, dtype=np.int32)
    n, ld = 1030, 1088
    rng = np.random.default_rng(3)
    pool = np.zeros((20, ld), np.float32)
    pool[:, :n] = rng.standard_normal((20, n)).astype(np.float32)
    ref = oracle.round_f32(pool[:, :n].copy(), row_ptr, col, w, out_rows)
    plan = ops.build_plan(row_ptr, col, w, out_rows)
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.full_like(pin, 7.0)
    ops.round_f32(pin, pout, plan, n=n)
    got = pout.cpu().numpy()
    assert _bits_equal(got[:, :n], ref)
    assert np.all(got[:, n:] == 7.0)  # padding untouched
    # odd ld -> scalar tiled path
    pin2 = torch.from_numpy(np.ascontiguousarray(pool[:, :n + 1])).to(cuda)
    pout2 = torch.zeros_like(pin2)
    ops.round_f32(pin2, pout2, plan, n=n)
    assert _bits_equal(pout2.cpu().numpy()[:, :n], ref)


def test_round_i64(cuda):
    g = nx.random_regular_graph(8, 64, seed=0)
    orders, ws = _graph_csr(g)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(64, dtype=np.int32)
    rng = np.random.default_rng(9)
    pool = rng.integers(0, 10 ** 6, size=(64, 53)).astype(np.int64)
    pool[:, 0] = 1000
    ref = oracle.round_i64(pool, row_ptr, col, w, out_rows)
    plan = ops.build_plan(row_ptr, col, w, out_rows)
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_i64(pin, pout, plan)
    assert np.array_equal(pout.cpu().numpy(), ref)
    assert np.all(ref[:, 0] == 999)


def test_round_sequential_matches_reference_fixture(cuda):
    """Sequential in-place 4-ring round driven through the reference (tests/golden/round_4ring)."""
    meta = json.loads((GOLDEN / "round_4ring.json").read_text())
    z = np.load(GOLDEN / "round_4ring.npz")
    layout = StateLayout.from_layout([(n, tuple(s), d) for n, s, d in meta["layout"]])
    pool = ModelPool(layout, 4, cuda)
    for i in range(4):
        pool.load_row(i, {n: torch.from_numpy(z[f"in{i}_{n}"]) for n, _, _ in meta["layout"]})
    ex = RoundExecutor(pool)
    orders = meta["orders"]
    ex.run(orders, [ra.unweighted_weights(len(o)) for o in orders], sequential=True)
    for i in range(4):
        sd = pool.state_dict(i)
        for n, _, _ in meta["layout"]:
            assert _bits_equal(sd[n].cpu().numpy(), z[f"seq{i}_{n}"]), (i, n)


def test_big_sha256_k1(cuda):
    """ResNet-18 M=3 / ResNet-50 M=9 reference outputs (sha256 per entry) through K1."""
    meta = json.loads((GOLDEN / "big_sha256.json").read_text())
    layouts = json.loads((GOLDEN / "layouts.json").read_text())
    cent = {k: {int(i): v for i, v in d.items()} for k, d in meta["centrality"].items()}
    for case in meta["cases"]:
        lay = [(n, tuple(s), d) for n, s, d in layouts[case["model"]]]
        layout = StateLayout.from_layout(lay)
        order = case["order"]
        if case["fn"] == "unweighted_module_avg":
            w = ra.unweighted_weights(len(order))
        elif case["fn"] == "weighted_module_avg":
            w = ra.weighted_weights(case["data_lens"])
        else:
            w = ra.centrality_weights(order, cent[case["centrality_metric"]], case["softmax"], case["softmax_coeff"])
        pool = ModelPool(layout, len(order), cuda)
        for r, seed in enumerate(case["seeds"]):
            pool.load_row(r, synth.synth_state_dict(lay, seed))
        ops.agg_f32([pool.row_f32(r) for r in range(len(order))], w, pool.row_f32(len(order) - 1))
        ops.agg_i64([pool.row_i64(r) for r in range(len(order))], w, pool.row_i64(len(order) - 1))
        sd = pool.state_dict(len(order) - 1)
        for name, digest in case["sha256"].items():
            a = sd[name].cpu().numpy()
            assert hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() == digest, (case["fn"], name)


def test_cosine_kernel_vs_numpy(cuda):
    lay = synth.get_layout("resnet18")
    layout = StateLayout.from_layout(lay)
    names = synth.param_names(lay)
    segs = layout.param_segments(names)
    plan = ops.build_cosine_plan(segs)
    a = synth.synth_state_dict(lay, 1)
    bs = [synth.synth_state_dict(lay, 2 + j) for j in range(3)]
    # make one pair strongly similar
    for k in bs[0]:
        if bs[0][k].dtype == torch.float32:
            bs[0][k] = a[k] * 2 + 0.01 * bs[0][k]
    pool = ModelPool(layout, 4, cuda)
    pool.load_row(0, a)
    for j, b in enumerate(bs):
        pool.load_row(1 + j, b)
    got = ops.cosine([pool.row_f32(0)] * 3, [pool.row_f32(1 + j) for j in range(3)], plan).cpu().numpy()
    fa = pool.row_f32(0).cpu().numpy()
    for j, b in enumerate(bs):
        ref = oracle.cosine_model(fa, pool.row_f32(1 + j).cpu().numpy(), segs)  # torch's order, bitwise
        assert got[j].view(np.uint32) == ref.view(np.uint32), (j, got[j], ref)
        assert abs(got[j] - ra.cosine_similarity([a[n].numpy() for n in names], [b[n].numpy() for n in names])) < 2e-5


_CLIQUE_GRAPHS = {
    "barbell60": lambda: nx.barbell_graph(60, 8),   # BASELINE config 4's topology (m = 60)
    "barbell20": lambda: nx.barbell_graph(20, 3),   # m = 20: the 32-register kernel
    "complete64": lambda: nx.complete_graph(64),    # m = 64: the largest block
    "complete9": lambda: nx.complete_graph(9),      # m = 9: the 16-register kernel
    "complete37": lambda: nx.complete_graph(37),    # m = 37: the 40-member instantiation, a partial row group
    "barbell45": lambda: nx.barbell_graph(45, 2),   # m = 45: the 48-member instantiation, bridges attached
    "complete53": lambda: nx.complete_graph(53),    # m = 53: the 56-member instantiation
    "mixed": lambda: nx.disjoint_union(nx.complete_graph(12), nx.random_regular_graph(4, 30, seed=1)),
}


@pytest.mark.parametrize("n", [1, 7, 4098, 70001])
@pytest.mark.parametrize("graph", list(_CLIQUE_GRAPHS))
def test_round_clique_vs_oracle(cuda, graph, n):
    """K3c (shared products, prefix-extended chains): bitwise the oracle round in EXACT mode and
    bitwise K1-FMA in FMA mode, signed weights, fp32 specials, odd n (scalar tail), permuted and
    padded output rows, the rest rows through their regular plan."""
    g = _CLIQUE_GRAPHS[graph]()
    orders = [sorted(g.neighbors(i)) + [i] for i in sorted(g.nodes)]
    rows = len(orders)
    sign = -1.0 if n % 2 else 1.0
    ws = [[sign / len(o)] * len(o) for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = (np.random.default_rng(rows).permutation(rows) + 2).astype(np.int32)
    plan = ops.build_clique_plan(row_ptr, col, w, out_rows)
    assert plan is not None and plan.n_cliques >= 1
    rng = np.random.default_rng(rows + n)
    pool = np.stack([_rand_f32(rng, n, special=True) for _ in range(rows)])
    if n > 8:
        pool[:, 5] = np.float32(-0.0)
        pool[::3, 6] = np.float32(np.inf)
    ld = n + (3 if n % 2 else 2)  # even, padded stride
    pin = torch.zeros(rows, ld, device=cuda)
    pin[:, :n] = torch.from_numpy(pool).to(cuda)
    pout = torch.full((rows + 2, ld), 7.0, device=cuda)
    got = pout
    ops.round_f32(pin, got, plan, n=n)
    full = oracle.round_f32(pool, row_ptr, col, w, out_rows - 2)
    assert _bits_equal(got[2:, :n].cpu().numpy(), full)
    assert torch.all(got[:2] == 7.0) and torch.all(got[:, n:] == 7.0)  # nothing else written
    # FMA mode: the same chains fused, bitwise K1 in FMA mode on the same operands
    ops.round_f32(pin, got, plan, n=n, mode=ops.MODE_FMA)
    chk = torch.empty(n, device=cuda)
    for r in (0, rows // 2, rows - 1):
        ops.agg_f32([pin[j, :n] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
        assert torch.equal(chk.view(torch.int32), got[out_rows[r], :n].contiguous().view(torch.int32))
    with pytest.raises(ValueError):
        ops.round_f32(pin, pin, plan, n=n)


def test_round_clique_through_tuner_and_i64(cuda):
    """tune_plan offers the clique plan for a barbell round; the int64 segment of a clique plan
    runs through its full regular plan."""
    g = nx.barbell_graph(24, 4)
    orders = [sorted(g.neighbors(i)) + [i] for i in sorted(g.nodes)]
    rows = len(orders)
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    rng = np.random.default_rng(3)
    pool = rng.standard_normal((rows, 20001)).astype(np.float32)
    pin = dev_rows(pool, cuda)
    pout = torch.zeros_like(pin)
    plan = ops.tune_plan(row_ptr, col, w, out_rows, pin, pout, n=20001)
    assert any((c["spec"] or {}).get("clique") for c in plan.candidates)
    cp = ops.plan_from_spec(row_ptr, col, w, out_rows, {"clique": 1}).to(cuda)
    ops.round_f32(pin, pout, cp, n=20001)
    assert _bits_equal(host(pout, 20001), oracle.round_f32(pool, row_ptr, col, w, out_rows))
    ip = rng.integers(0, 10 ** 6, size=(rows, 5)).astype(np.int64)
    ipo = torch.zeros(rows, 5, dtype=torch.int64, device=cuda)
    ops.round_i64(torch.from_numpy(ip).to(cuda), ipo, cp)
    assert np.array_equal(ipo.cpu().numpy(), oracle.round_i64(ip, row_ptr, col, w, out_rows))


@pytest.mark.parametrize("n", [5, 4097])
def test_round_clique_attached_rows_general(cuda, n):
    """Attached rows with two non-member neighbors interleaved among the members, a member or a
    non-member as own model, and their own weights: bitwise the oracle (EXACT) and K1 (FMA)."""
    members = list(range(0, 40, 2))  # 20 members: even pool rows 0..38
    orders, ws = [], []
    for i in members:  # the clique rows, weight 1/20
        orders.append([j for j in members if j != i] + [i])
        ws.append([1 / 20] * 20)
    # attached: member self, externals 5 and 31 (interleaved), weight -0.3
    orders.append([j for j in members if j not in (10,)] [:12] + [5, 31])
    orders[-1] = sorted(orders[-1]) + [10]
    ws.append([-0.3] * len(orders[-1]))
    # attached: non-member self (41), one external below every member? (none) and one above (45)
    orders.append(sorted(members[3:15] + [45]) + [41])
    ws.append([0.07] * len(orders[-1]))
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    cliques, rest = ops.find_cliques(row_ptr, col, w, out_rows)
    assert len(cliques) == 1 and len(cliques[0][3]) == 2 and rest == []
    plan = ops.build_clique_plan(row_ptr, col, w, out_rows)
    pool = np.random.default_rng(n).standard_normal((48, n)).astype(np.float32)
    pin = dev_rows(pool, cuda)
    pout = torch.zeros(rows, pin.shape[1], device=cuda)
    ops.round_f32(pin, pout, plan, n=n)
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows, pool_out=np.zeros((rows, n), np.float32))
    assert _bits_equal(host(pout, n), ref)
    ops.round_f32(pin, pout, plan, n=n, mode=ops.MODE_FMA)
    chk = torch.empty(n, device=cuda)
    for r in (rows - 2, rows - 1, 3):
        ops.agg_f32([pin[j, :n] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
        assert torch.equal(chk.view(torch.int32), pout[r, :n].view(torch.int32))


@pytest.mark.parametrize("spec", [None, {"c4": 128, "lds": 81920, "dense": 0}, {"c4": 64, "lds": 81920, "dense": 0},
                                  {"c4": 32, "lds": 81920, "dense": 0}, {"c4": 16, "lds": 81920, "dense": 0}])
def test_full_size_ring32_round_vs_reference(cuda, spec):
    """BASELINE config 2 at full size (32-ring, ResNet-18, M = 3): one K3 round over the
    device pool equals the REFERENCE's outputs (sha256 per output model, generated by its own
    unweighted_module_avg; tests/golden/make_golden.py big_round) for every plan form the tuner
    can pick (None = default_plan)."""
    from test_oracle_golden import RING32, ring32_pools

    f, i = ring32_pools()
    orders = [r["order"] for r in RING32["rows"]]
    rp, col, w = ra.round_csr(orders, [ra.unweighted_weights(len(o)) for o in orders])
    out_rows = np.arange(32, dtype=np.int32)
    plan = ops.default_plan(rp, col, w, out_rows) if spec is None else ops.plan_from_spec(rp, col, w, out_rows, spec)
    n = f.shape[1]  # 11,183,562: odd rows would run the scalar kernel; ModelPool's stride instead
    pin = dev_rows(f, cuda)
    pout = torch.empty_like(pin)
    iin = torch.from_numpy(i).to(cuda)
    iout = torch.empty_like(iin)
    ops.round_f32(pin, pout, plan, n=n)
    ops.round_i64(iin, iout, plan)
    got, igot = host(pout, n), iout.cpu().numpy()
    for r, row in enumerate(RING32["rows"]):
        assert hashlib.sha256(got[r].tobytes()).hexdigest() == row["sha256_f32"], r
        assert hashlib.sha256(igot[r].tobytes()).hexdigest() == row["sha256_i64"], r
