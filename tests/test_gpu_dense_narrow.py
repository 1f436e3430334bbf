"""GPU parity of K3d (dense row blocks over 512-B source tiles: plan c4 = 32, dense_rb = 8)
against the C oracle, through the C-ABI.

K3d computes each row's operands in the row's reference order (sorted neighbours, own model
last) from wave-uniform block tables, so EXACT mode is bit-exact (fp32, bf16, int64 through the
staged scalar kernel) and FMA mode is the fused chain starting at -0.0, bitwise equal to K1-FMA.
"""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops

from test_gpu_kernels import _NARROW_GRAPHS, _bits_equal, _graph_csr, _rand_f32

pytestmark = pytest.mark.gpu

_SBM = dict(sizes=[32] * 8, p=[[14 / 31 if a == b else 2 / 224 for b in range(8)] for a in range(8)])


def _sbm256():
    return nx.stochastic_block_model(_SBM["sizes"], _SBM["p"], seed=0)


_GRAPHS = dict(_NARROW_GRAPHS, sbm256=_sbm256)


def _dense_plan(row_ptr, col, w, out_rows, lds=160 * 1024):
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=32, lds_bytes=lds, dense=8)
    assert plan.info.c4 == 32 and plan.info.dense_rb == 8
    assert ops.round_kernel_name(plan.info) == "k_round_dense_narrow"
    return plan


@pytest.mark.parametrize("n", [4099, 70001])
@pytest.mark.parametrize("weights", ["unweighted", "softmax"])
@pytest.mark.parametrize("graph", list(_GRAPHS))
def test_dense_narrow_f32_vs_oracle(cuda, graph, weights, n):
    g = _GRAPHS[graph]()
    orders, ws = _graph_csr(g, weights)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.random.default_rng(rows).permutation(rows).astype(np.int32)
    rng = np.random.default_rng(rows + n)
    pool = np.stack([_rand_f32(rng, n, special=(r % 5 == 0)) for r in range(rows)])
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    plan = _dense_plan(row_ptr, col, w, out_rows)
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan)
    assert _bits_equal(pout.cpu().numpy(), ref)
    # FMA: the fused chain from -0.0, bitwise K1-FMA on the same operands (a few rows)
    ops.round_f32(pin, pout, plan, mode=ops.MODE_FMA)
    chk = torch.empty(n, dtype=torch.float32, device=cuda)
    for r in range(0, rows, max(1, rows // 6)):
        ops.agg_f32([pin[j] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
        assert torch.equal(chk.view(torch.int32), pout[out_rows[r]].view(torch.int32)), r
    if plan.single_group:  # one group: in place is snapshot-safe
        ops.round_f32(pin, pin, plan)
        assert _bits_equal(pin.cpu().numpy(), ref)


@pytest.mark.parametrize("lds", [24 * 1024, 40 * 1024])
def test_dense_narrow_several_groups(cuda, lds):
    """Budgets below the graph's source count: several row groups (grid.y), J = 1 / 4 staging."""
    g = nx.random_regular_graph(8, 96, seed=4)
    orders, ws = _graph_csr(g, "softmax")
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = _dense_plan(row_ptr, col, w, out_rows, lds=lds)
    assert plan.info.n_groups > 1
    rng = np.random.default_rng(lds)
    pool = np.stack([_rand_f32(rng, 20483) for _ in range(rows)])
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan)
    assert _bits_equal(pout.cpu().numpy(), oracle.round_f32(pool, row_ptr, col, w, out_rows))


@pytest.mark.parametrize("sign", [1.0, -1.0])
def test_dense_narrow_uniform_products_signed_zero(cuda, sign):
    """A random regular graph under one weight: most entries are shared products (compact entry
    flag 0x100, one rounded w * x added to every row taking it); -0 inputs and results survive."""
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
    plan = _dense_plan(row_ptr, col, w, out_rows)
    h, i = plan.host, plan.info
    assert i.narrow_roww == 1  # one weight per row: compact tables {n, pad, w[8], entries}
    assert any((h[t + 16: t + 16 + h[t]] & 0x100).any() for t in h[i.off_blk_tab: i.off_blk_tab + i.n_blocks])
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan)
    assert _bits_equal(pout.cpu().numpy(), oracle.round_f32(pool, row_ptr, col, w, out_rows))
    bits = oracle.f32_to_bf16(pool)
    pb = torch.from_numpy(bits.view(np.int16)).view(torch.bfloat16).to(cuda)
    ob = torch.zeros_like(pb)
    for exact, mode in ((True, ops.MODE_EXACT), (False, ops.MODE_FMA)):
        ops.round_bf16(pb, ob, plan, mode=mode)
        refb = oracle.round_bf16(bits, row_ptr, col, w, out_rows, exact=exact)
        assert np.array_equal(ob.cpu().view(torch.int16).numpy().view(np.uint16), refb), exact


@pytest.mark.parametrize("weights", ["unweighted", "softmax"])
@pytest.mark.parametrize("graph", ["sbm256", "sbm", "gnp", "barbell"])
def test_dense_narrow_bf16_vs_oracle(cuda, graph, weights):
    """bf16 pools: EXACT = the reference's own bf16 ops (bitwise), FMA = fp32 fused chain rounded
    once (bitwise the oracle's fused chain); NaN stored as 0xFFFF."""
    g = _GRAPHS[graph]()
    orders, ws = _graph_csr(g, weights)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.random.default_rng(rows + 1).permutation(rows).astype(np.int32)
    n = 8195
    rng = np.random.default_rng(rows)
    pool = np.stack([_rand_f32(rng, n, special=True) for _ in range(rows)])
    pool[1, 20] = np.nan
    bits = oracle.f32_to_bf16(pool)
    plan = _dense_plan(row_ptr, col, w, out_rows)
    pb = torch.from_numpy(bits.view(np.int16)).view(torch.bfloat16).to(cuda)
    ob = torch.zeros_like(pb)
    for exact, mode in ((True, ops.MODE_EXACT), (False, ops.MODE_FMA)):
        ops.round_bf16(pb, ob, plan, mode=mode)
        refb = oracle.round_bf16(bits, row_ptr, col, w, out_rows, exact=exact)
        assert np.array_equal(ob.cpu().view(torch.int16).numpy().view(np.uint16), refb), exact
    if plan.single_group:
        ops.round_bf16(pb, pb, plan)
        refb = oracle.round_bf16(bits, row_ptr, col, w, out_rows, exact=True)
        assert np.array_equal(pb.cpu().view(torch.int16).numpy().view(np.uint16), refb)


def test_dense_narrow_i64_and_tail(cuda):
    """The int64 segment and the fp32 n % 4 tail of a K3d plan run the staged scalar kernel with
    a c4 = 16 tile (a 256-source group plus its plan slice fits 160 KiB)."""
    g = _sbm256()
    orders, ws = _graph_csr(g)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    plan = _dense_plan(row_ptr, col, w, out_rows)
    assert plan.info.n_groups == 1 and plan.info.max_src == rows
    assert plan.info.scalar_lds_bytes <= 160 * 1024
    rng = np.random.default_rng(9)
    xi = rng.integers(-(2 ** 40), 2 ** 40, size=(rows, 37)).astype(np.int64)
    xi[:, :3] = [1000, 7, -1000]
    pin = torch.from_numpy(xi).to(cuda)
    pout = torch.zeros_like(pin)
    ops.round_i64(pin, pout, plan)
    assert np.array_equal(pout.cpu().numpy(), oracle.round_i64(xi, row_ptr, col, w, out_rows))
    # a row stride that is not a multiple of 4: everything on the scalar kernel
    pool = rng.standard_normal((rows, 1031)).astype(np.float32)
    base = torch.from_numpy(pool).to(cuda)
    out = torch.zeros_like(base)
    ops.round_f32(base, out, plan)
    assert _bits_equal(out.cpu().numpy(), oracle.round_f32(pool, row_ptr, col, w, out_rows))


def test_dense_narrow_matches_narrow_sbm256(cuda):
    """Config 5's topology at a reduced width: K3d and the narrow kernel give the same bits
    (both the oracle's) in EXACT mode, fp32 and bf16."""
    g = _sbm256()
    orders, ws = _graph_csr(g)
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    n = 65536 + 12
    rng = np.random.default_rng(3)
    pin = torch.from_numpy(rng.standard_normal((rows, n)).astype(np.float32)).to(cuda)
    a, b = torch.empty_like(pin), torch.empty_like(pin)
    ops.round_f32(pin, a, _dense_plan(row_ptr, col, w, out_rows))
    ops.round_f32(pin, b, ops.build_plan(row_ptr, col, w, out_rows, c4=16, lds_bytes=160 * 1024))
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    pb = pin.to(torch.bfloat16)
    a, b = torch.empty_like(pb), torch.empty_like(pb)
    ops.round_bf16(pb, a, _dense_plan(row_ptr, col, w, out_rows))
    ops.round_bf16(pb, b, ops.build_plan(row_ptr, col, w, out_rows, c4=16, lds_bytes=160 * 1024))
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
