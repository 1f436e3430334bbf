"""GPU parity of the narrow kernel's broadcast form (build_plan(bcast=8 / 16)): per-lane operand
records in VGPRs, handed to each row's lanes by DPP row broadcasts.  Bar: bitwise the C oracle
in EXACT mode (fp32 and bf16), bitwise K1-FMA / the oracle's fused bf16 chain in FMA mode."""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops

import bench
from _pools import dev_rows, host

pytestmark = pytest.mark.gpu

_GRAPHS = {
    "ring": lambda: nx.cycle_graph(16),
    "regular": lambda: nx.random_regular_graph(8, 64, seed=0),
    "sbm": lambda: nx.stochastic_block_model([32] * 4, [[0.45 if a == b else 0.01 for b in range(4)] for a in range(4)], seed=0),
    "barbell": lambda: nx.barbell_graph(12, 4),
    "complete": lambda: nx.complete_graph(40),
    "gnp": lambda: nx.gnp_random_graph(150, 0.08, seed=2),
    "star": lambda: nx.star_graph(70),  # one row of 71 operands: five records in one pass
}


def _csr(g, weights):
    cent = nx.degree_centrality(g)
    orders = [sorted(g.neighbors(i)) + [i] for i in sorted(g.nodes)]
    if weights == "unweighted":
        ws = [ra.unweighted_weights(len(o)) for o in orders]
    else:
        ws = [ra.centrality_weights(o, cent, True, 10.0) for o in orders]
    return orders, ws


def _pool(rng, rows, n, special):
    x = rng.standard_normal((rows, n)).astype(np.float32) * np.float32(3.0)
    if special:
        x[:, 0] = 1e-40
        x[:, 1] = -0.0
        x[::2, 2] = 3e38
        x[:, 3] = -1e-45
        x[1::3, 4] = np.float32(np.nan)
        x[::5, 5] = np.float32(np.inf)
    return x


def _bits_equal(a, b):
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint32), b[~nb].view(np.uint32))


FORMS = [(8, 2), (12, 2), (16, 2), (16, 1)]  # (wavefronts per workgroup, workgroups per CU)


@pytest.mark.parametrize("pad", [True, False], ids=["vec", "scalar"])
@pytest.mark.parametrize("waves,wg", FORMS)
@pytest.mark.parametrize("c4", [16, 32])
@pytest.mark.parametrize("n", [4099, 70001])
@pytest.mark.parametrize("graph", list(_GRAPHS))
def test_round_bcast_f32_vs_oracle(cuda, graph, n, c4, waves, wg, pad):
    """pad: rows strided by a multiple of 64 elements (the broadcast kernel computes the float4
    body, the scalar kernel the n % 4 tail) or contiguous odd rows (all by the scalar kernel)."""
    g = _GRAPHS[graph]()
    orders, ws = _csr(g, "degcent" if graph in ("regular", "gnp", "sbm", "star") else "unweighted")
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.random.default_rng(rows).permutation(rows).astype(np.int32)
    rng = np.random.default_rng(rows + n + c4 + waves)
    pool = _pool(rng, rows, n, special=(n == 4099))
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=80 * 1024, bcast=waves, bcast_wg=wg)
    assert plan.info.narrow_bcast == waves and plan.info.bc_wg_per_cu == wg
    pin = dev_rows(pool, cuda, pad)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=n)
    assert _bits_equal(host(pout, n), ref)
    # FMA: -0.0 start then one fused chain: bitwise K1-FMA on the same operands
    ops.round_f32(pin, pout, plan, n=n, mode=ops.MODE_FMA)
    chk = torch.empty(n, dtype=torch.float32, device=cuda)
    for r in range(0, rows, max(1, rows // 9)):
        ops.agg_f32([pin[j, :n] for j in orders[r]], ws[r], chk, mode=ops.MODE_FMA)
        assert torch.equal(chk.view(torch.int32), pout[out_rows[r], :n].view(torch.int32)), r
    if plan.single_group:  # in place: every source staged before any row of a tile is written
        ops.round_f32(pin, pin, plan, n=n)
        assert _bits_equal(host(pin, n), ref)


@pytest.mark.parametrize("waves,wg", FORMS)
@pytest.mark.parametrize("c4", [16, 32])
@pytest.mark.parametrize("graph", ["regular", "sbm", "star", "ring"])
def test_round_bcast_bf16_vs_oracle(cuda, graph, c4, waves, wg):
    g = _GRAPHS[graph]()
    orders, ws = _csr(g, "unweighted" if graph == "ring" else "degcent")
    rows = len(orders)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)[::-1].copy()
    n = 8200  # 2050 chunks: the 16-B staging lanes; 8196 (2049 chunks) the 8-B ones; 8198 + tail
    rng = np.random.default_rng(rows + c4)
    bits = oracle.f32_to_bf16(_pool(rng, rows, n, special=True))
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=80 * 1024, bcast=waves, bcast_wg=wg)
    for nn, pad in ((n, False), (n - 4, False), (n - 2, True), (n - 2, False)):
        b = np.ascontiguousarray(bits[:, :nn])
        pb = dev_rows(b, cuda, pad)
        ob = torch.zeros_like(pb)
        for exact in (True, False):
            ops.round_bf16(pb, ob, plan, n=nn, mode=ops.MODE_EXACT if exact else ops.MODE_FMA)
            ref = oracle.round_bf16(b, row_ptr, col, w, out_rows, exact=exact)
            assert np.array_equal(host(ob, nn), ref), (nn, pad, exact)


def test_round_bcast_padded_ld_and_tail(cuda):
    """Rows padded past n (ld > n) and n % 4 != 0: the float4 body by the broadcast kernel, the
    tail and the int64 segment by the plan's scalar kernels."""
    orders, ws = bench.round_spec(64, 8, weights="degcent")
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(64, dtype=np.int32)
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=16, lds_bytes=80 * 1024, bcast=16)
    rng = np.random.default_rng(11)
    n, ld = 5003, 5120
    pool = rng.standard_normal((64, ld)).astype(np.float32)
    ref = oracle.round_f32(np.ascontiguousarray(pool[:, :n]), row_ptr, col, w, out_rows)
    pin = torch.from_numpy(pool).to(cuda)
    pout = torch.full_like(pin, 7.0)
    ops.round_f32(pin, pout, plan, n=n)
    got = pout.cpu().numpy()
    assert _bits_equal(got[:, :n], ref)
    assert np.all(got[:, n:] == 7.0)
    xi = rng.integers(0, 10 ** 6, size=(64, 53)).astype(np.int64)
    oi = torch.zeros(64, 53, dtype=torch.int64, device=cuda)
    ops.round_i64(torch.from_numpy(xi).to(cuda), oi, plan)
    assert np.array_equal(oi.cpu().numpy(), oracle.round_i64(xi, row_ptr, col, w, out_rows))


@pytest.mark.parametrize("waves,wg", FORMS)
def test_round_bcast_config5_topology(cuda, waves, wg):
    """BASELINE config 5's topology with degree-centrality weights (the per-operand-weight case
    this form is for): one group of 256 sources at c4 = 16, every source read once per tile."""
    orders, ws = bench.round_spec(256, 8, kind="sbm", weights="degcent")
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(256, dtype=np.int32)
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=16, lds_bytes=160 * 1024, bcast=waves, bcast_wg=wg)
    assert plan.info.n_groups == 1 and plan.info.total_src == 256
    n = 16387
    rng = np.random.default_rng(5)
    pool = rng.standard_normal((256, n)).astype(np.float32)
    pin = dev_rows(pool, cuda)
    pout = torch.zeros_like(pin)
    ops.round_f32(pin, pout, plan, n=n)
    assert _bits_equal(host(pout, n), oracle.round_f32(pool, row_ptr, col, w, out_rows))


def _limit_round(k, shape):
    """A round needing k distinct sources: "wide" = ceil(k / 4) rows of 4 consecutive sources
    each (the planner's greedy grouping keeps them in one group while the union fits), "single"
    = one row of all k sources (plus rows for every source's own output)."""
    if shape == "wide":
        orders = [list(range(4 * r, min(k, 4 * r + 4))) for r in range(-(-k // 4))]
    else:
        orders = [list(range(k))]
    ws = [[1.0 / (len(o) + j) + 1e-3 * j for j in range(len(o))] for o in orders]  # per-operand weights
    return orders, ws


@pytest.mark.parametrize("shape", ["wide", "single"])
@pytest.mark.parametrize("waves,wg", FORMS)
@pytest.mark.parametrize("c4", [16, 32])
def test_round_bcast_staging_limit(cuda, c4, waves, wg, shape):
    """Each broadcast form at its largest admissible group (the library's staging table,
    tal_round_bcast_max_loads, which the planner and the launcher both read) and one source past
    it: whatever plan the planner returns launches (TAL_OK) and is bitwise the oracle; a group
    at the limit stays one group; past it the planner splits the group or - a single row that
    cannot be split - refuses with TAL_ERR_CAPACITY.  The launcher never refuses a planned
    round (the failure behind round 4's call_r04j and world-8 rehearsal)."""
    L = ops._lib.load()
    limit = L.tal_round_bcast_max_loads(c4, waves, wg) // c4  # sources per group
    n = 2 * 64 * c4 + 12  # two column tiles of every width, and a scalar tail
    for k in (limit, limit + 1):
        orders, ws = _limit_round(k, shape)
        rows = len(orders)
        row_ptr, col, w = ra.round_csr(orders, ws)
        out_rows = np.arange(rows, dtype=np.int32) + k  # outputs after the sources
        try:
            plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=160 * 1024, bcast=waves, bcast_wg=wg)
        except ops._lib.TalError as exc:
            assert exc.code == ops._lib.TAL_ERR_CAPACITY and shape == "single", (k, str(exc))
            continue
        if k == limit and shape == "wide":
            assert plan.info.n_groups == 1 and plan.info.max_src == limit
        assert plan.info.max_src <= limit
        rng = np.random.default_rng(k + c4 + waves)
        pool = rng.standard_normal((k + rows, n)).astype(np.float32)
        ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
        pin = dev_rows(pool, cuda, True)
        pout = pin.clone()
        ops.round_f32(pin, pout, plan, n=n)  # raises on any launch refusal
        assert _bits_equal(host(pout, n), ref), (k, shape)
