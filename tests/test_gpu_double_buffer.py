"""Double-buffered rounds on the GPU (RoundExecutor's default since round 6): each round reads the
pool, writes the spare, copies the rows it does not aggregate, and exchanges the two pools'
storages; bitwise the oracle's snapshot round applied round after round, for fp32 / int64 and
bf16 segments, single- and multi-group plans, partial participation, and models bound to the
pool (their parameters read the round's output through the exchange)."""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops
from topology_aware_learning_amd.arena import ModelPool, StateLayout, bound_row
from topology_aware_learning_amd.round import RoundExecutor

pytestmark = pytest.mark.gpu


def _graph(n, seed):
    g = nx.random_regular_graph(8, n, seed=seed)
    return [sorted(g.neighbors(i)) + [i] for i in range(n)]


@pytest.mark.parametrize("n_rows", [64, 1000])  # one LDS group / several groups
def test_double_buffered_rounds_vs_oracle(cuda, n_rows):
    orders = _graph(n_rows, 3)
    out_rows = [r for r in range(n_rows) if r % 7 != 3]  # partial participation
    ords = [orders[r] for r in out_rows]
    ws = [ra.unweighted_weights(len(o)) for o in ords]
    lay = StateLayout.from_layout([("w", (4093,), "float32"), ("nbt", (3,), "int64")])
    pool = ModelPool(lay, n_rows, cuda)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((n_rows, 4093)).astype(np.float32)
    xi = rng.integers(0, 10 ** 6, (n_rows, 3))
    pool.f32[:, :4093] = torch.from_numpy(x).to(cuda)
    pool.i64[:, :3] = torch.from_numpy(xi).to(cuda)
    ex = RoundExecutor(pool, placement_trials=2)
    assert ex.double_buffer
    rp, col, w = ra.round_csr(ords, ws)
    rows = np.asarray(out_rows, np.int32)
    ptr0 = pool.f32.data_ptr()
    for k in range(3):
        x = oracle.round_f32(x, rp, col, w, rows)
        xi = oracle.round_i64(xi, rp, col, w, rows)
        ex.run(ords, ws, out_rows)
        assert np.array_equal(pool.f32[:, :4093].cpu().numpy().view(np.uint32), x.view(np.uint32)), k
        assert np.array_equal(pool.i64[:, :3].cpu().numpy(), xi), k
    assert ex.swaps == 3 and ex.spare is not None and pool.f32.data_ptr() != ptr0


def test_double_buffered_bf16_round(cuda):
    orders = _graph(128, 8)
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    lay = StateLayout.from_layout([("w", (2051,), "bfloat16")])
    pool = ModelPool(lay, 128, cuda)
    rng = np.random.default_rng(6)
    bits = oracle.f32_to_bf16(rng.standard_normal((128, 2051)).astype(np.float32))
    pool.b16[:, :2051] = torch.from_numpy(bits.view(np.int16)).view(torch.bfloat16).to(cuda)
    ex = RoundExecutor(pool, placement_trials=1)
    rp, col, w = ra.round_csr(orders, ws)
    for k in range(2):
        bits = oracle.round_bf16(bits, rp, col, w, np.arange(128, dtype=np.int32))
        ex.run(orders, ws)
        got = pool.b16[:, :2051].cpu().view(torch.int16).numpy().view(np.uint16)
        assert np.array_equal(got, bits), k
    assert ex.swaps == 2


def test_bound_models_read_the_round(cuda):
    """Models bound to the pool read each round's output through their own parameters, stay
    bound across the exchanges, and a K1 call on them (the per-call path) after a
    double-buffered round reads the new rows."""
    torch.manual_seed(0)
    models = [torch.nn.Sequential(torch.nn.Linear(31, 17), torch.nn.BatchNorm1d(17)).to(cuda) for _ in range(16)]
    pool = ModelPool(StateLayout.from_state_dict(models[0].state_dict()), 16, cuda)
    for r, m in enumerate(models):
        pool.bind(m, r)
    orders = [[(i + 1) % 16, (i + 15) % 16, i] for i in range(16)]
    ws = [ra.unweighted_weights(3)] * 16
    x = pool.f32.cpu().numpy().copy()
    rp, col, w = ra.round_csr(orders, ws)
    ex = RoundExecutor(pool, placement_trials=1)
    for _ in range(2):
        x = oracle.round_f32(x, rp, col, w, np.arange(16, dtype=np.int32))
        ex.run(orders, ws)
    for r, m in enumerate(models):
        assert bound_row(m) == (pool, r)
        flat = torch.cat([v.reshape(-1).float() for k, v in m.state_dict().items() if v.dtype == torch.float32])
        assert np.array_equal(flat.cpu().numpy().view(np.uint32), x[r, :flat.numel()].view(np.uint32))
    out = torch.empty(pool.layout.n_f32, device=cuda)
    out_i = torch.empty(pool.layout.n_i64, dtype=torch.int64, device=cuda)
    ops.agg_model_f32([pool.row_f32(j) for j in orders[4]], [pool.row_i64(j) for j in orders[4]], ws[4], out, out_i)
    ref = oracle.agg_f32([x[j, :pool.layout.n_f32] for j in orders[4]], ws[4])
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
