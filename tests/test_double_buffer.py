"""Double-buffered rounds (RoundExecutor, round 6): the storage exchange behind ModelPool.swap_with
(csrc/storage_swap.cpp, libtal_swap.so) and the executor's round -> copy the rest -> swap logic,
on CPU pools (no GPU: the kernel launch is replaced by the torch restatement of the round)."""
import ctypes

import numpy as np
import pytest
import torch

from topology_aware_learning_amd import arena
from topology_aware_learning_amd.arena import ModelPool, StateLayout, bound_row

from _models import TinyNet


def _pool_of(models):
    pool = ModelPool(StateLayout.from_state_dict(models[0].state_dict()), len(models), "cpu")
    for r, m in enumerate(models):
        pool.bind(m, r)
    return pool


def test_swap_library_exports():
    from topology_aware_learning_amd.build import SWAP_LIB

    lib = ctypes.CDLL(str(SWAP_LIB))
    assert hasattr(lib, "tal_swap_storage")


def test_swap_storage_moves_every_view():
    a = torch.arange(12, dtype=torch.float32).view(3, 4)
    b = torch.full((3, 4), -1.0)
    va, vb = a[1, 1:3], b[2]
    pa, pb = a.data_ptr(), b.data_ptr()
    arena.swap_storage(a, b)
    assert a.data_ptr() == pb and b.data_ptr() == pa
    assert torch.equal(a, torch.full((3, 4), -1.0)) and torch.equal(va, torch.tensor([-1.0, -1.0]))
    assert torch.equal(vb, torch.tensor([8.0, 9.0, 10.0, 11.0]))
    with pytest.raises(ValueError):
        arena.swap_storage(a, a[0])  # the same storage
    with pytest.raises(ValueError):
        arena.swap_storage(a, torch.zeros(5))  # sizes differ


def test_bound_models_follow_a_swap():
    """After swap_with the bound models read the other pool's bytes and are still bound (the
    binding records offsets from the segment base, not addresses): the O(1) check and the full
    check after a hook event both pass; a module re-pointed elsewhere is still caught."""
    torch.manual_seed(0)
    models = [TinyNet() for _ in range(3)]
    pool = _pool_of(models)
    spare = ModelPool(pool.layout, 3, "cpu")
    spare.f32.normal_()
    spare.i64.random_(0, 100)
    want = {k: v.clone() for k, v in spare.state_dict(1).items()}
    pool.swap_with(spare)
    for k, v in models[1].state_dict().items():
        assert torch.equal(v, want[k]), k
    assert bound_row(models[1]) == (pool, 1)  # O(1) path
    torch.nn.Linear(2, 2)  # a registration hook fires: the next check is the full one
    assert all(bound_row(m) == (pool, r) for r, m in enumerate(models))
    models[2].fc.weight.data = models[2].fc.weight.data.clone()
    assert bound_row(models[2]) is None
    with pytest.raises(ValueError):
        pool.swap_with(ModelPool(pool.layout, 2, "cpu"))
    part = ModelPool(pool.layout, 3, "cpu", f32=torch.zeros(4, pool.layout.ld_f32)[:3])
    assert not part.whole_storage()
    with pytest.raises(ValueError):
        pool.swap_with(part)


def test_double_buffered_run_logic(monkeypatch):
    """RoundExecutor's double-buffered run on a CPU pool with the launch replaced by the torch
    restatement: aggregated rows hold the round, the other rows their old values (copied into
    the spare before the swap), two rounds alternate the memory, and each round reads the
    previous round's output (snapshot semantics per round)."""
    from topology_aware_learning_amd.round import RoundExecutor

    lay = StateLayout.from_layout([("w", (37,), "float32"), ("n", (), "int64")])
    pool = ModelPool(lay, 5, "cpu")
    pool.f32.normal_(generator=torch.Generator().manual_seed(1))
    pool.i64.random_(0, 1000, generator=torch.Generator().manual_seed(2))
    orders = [[1, 2, 0], [0, 1], [3, 4, 2]]
    ws = [[0.25, 0.25, 0.5], [0.5, 0.5], [0.2, 0.3, 0.5]]
    out_rows = [0, 1, 2]
    ex = RoundExecutor(pool, double_buffer=True)
    ex.spare = ModelPool(lay, 5, "cpu")  # (on a GPU: placed by timing candidates)

    def launch(plan, dst):
        assert dst is ex.spare
        for o, w, r in zip(orders, ws, out_rows):
            acc = torch.zeros(lay.ld_f32)
            for j, wj in zip(o, w):
                acc = acc + np.float32(wj) * pool.f32[j]
            dst.f32[r] = acc
            dst.i64[r] = sum(float(np.float32(wj)) * pool.i64[j].double() for j, wj in zip(o, w)).long()

    monkeypatch.setattr(ex, "_launch", launch)
    monkeypatch.setattr(ex, "plan", lambda o, w, r: _plan_with_rest(lay, 5, r))
    x0 = pool.f32.clone()
    view3 = pool.row_f32(3)
    ex.run(orders, ws, out_rows)
    assert ex.swaps == 1
    want0 = (x0[1] * np.float32(0.25) + x0[2] * np.float32(0.25)) + x0[0] * np.float32(0.5)
    assert torch.allclose(pool.f32[0], want0)
    assert torch.equal(pool.f32[3:], x0[3:]) and torch.equal(view3[:37], x0[3, :37])
    x1 = pool.f32.clone()
    ex.run(orders, ws, out_rows)
    assert ex.swaps == 2
    assert torch.allclose(pool.f32[1], x1[0] * np.float32(0.5) + x1[1] * np.float32(0.5))
    assert torch.equal(pool.f32[3:], x0[3:])


def _plan_with_rest(lay, rows, out_rows):
    class P:
        single_group = True

    p = P()
    rest = sorted(set(range(rows)) - set(out_rows))
    p.rest_rows = torch.as_tensor(rest, dtype=torch.long) if rest else None
    return p


def test_double_buffer_defaults():
    """On by default only for device pools whose segments are whole storages; off for host
    pools and with an explicit scratch pool."""
    from topology_aware_learning_amd.round import RoundExecutor

    lay = StateLayout.from_layout([("w", (5,), "float32")])
    assert not RoundExecutor(ModelPool(lay, 2, "cpu")).double_buffer
    assert not RoundExecutor(ModelPool(lay, 2, "cpu"), scratch=ModelPool(lay, 2, "cpu")).double_buffer
