"""Checkpoints from / into the model pool: same file structure as the
reference's save_checkpoint (reference utils.py:19-38), values bit-identical, round trip
through load_checkpoint.  CPU pool here; tests/test_gpu_interface.py repeats it on the GPU."""
import types

import pytest
import torch

from src import utils as U
from src.aggregation_scheduler import BaseScheduler
from topology_aware_learning_amd.aggregate import layout_of_module
from topology_aware_learning_amd.arena import ModelPool
from topology_aware_learning_amd.checkpoint import common_pool

from _models import TinyNet


def _clients(n, seed):
    torch.manual_seed(seed)
    out = []
    for i in range(n):
        m = TinyNet()
        with torch.no_grad():
            for b in m.buffers():
                if b.dtype == torch.int64:
                    b.fill_(1000 + i)
                else:
                    b.uniform_(0.5, 2.0)
        out.append(types.SimpleNamespace(idx=i, model=m))
    return out


def _check_same(a, b):
    assert list(a) == list(b)
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, k
        bits = (lambda t: t.view(torch.int32)) if a[k].dtype == torch.float32 else (lambda t: t)
        assert torch.equal(bits(a[k].cpu()), bits(b[k].cpu())), k


def _bound(rows, seed=0, device="cpu"):
    cl = _clients(len(rows), seed)
    pool = ModelPool(layout_of_module(cl[0].model), max(rows) + 1, device)
    for c, r in zip(cl, rows):
        c.model.to(device)
        pool.bind(c.model, r)
    return cl, pool


@pytest.mark.parametrize("rows", [[0, 1, 2], [2, 0, 1], [0, 3, 4]])
def test_pool_checkpoint_matches_reference_format(tmp_path, rows):
    cl, pool = _bound(rows)
    assert common_pool([c.model for c in cl]) is not None
    results = [{"client_idx": 0, "acc": 0.5}]
    U.save_checkpoint(3, cl, results, tmp_path / "pool.pth")
    # the reference's way: per-client state_dict() copies
    torch.save({"client_state_dicts": [c.model.state_dict() for c in cl], "round_idx": 3,
                "client_results": results}, tmp_path / "ref.pth")
    a = torch.load(tmp_path / "pool.pth", weights_only=False)
    b = torch.load(tmp_path / "ref.pth", weights_only=False)
    assert list(a) == list(b) and a["round_idx"] == 3 and a["client_results"] == results
    for sa, sb in zip(a["client_state_dicts"], b["client_state_dicts"]):
        _check_same(sa, sb)
    # the reference's loader: load_state_dict into unbound models
    fresh = _clients(len(rows), 99)
    r, fresh, res, _ = U.load_checkpoint(tmp_path / "pool.pth", fresh, BaseScheduler(1.0))
    assert r == 3 and res == results
    for c, f in zip(cl, fresh):
        _check_same(c.model.state_dict(), f.model.state_dict())


def test_load_checkpoint_into_bound_pool(tmp_path):
    cl, pool = _bound([0, 1, 2], seed=1)
    U.save_checkpoint(1, cl, [], tmp_path / "c.pth")
    cl2, pool2 = _bound([2, 1, 0], seed=5)
    U.load_checkpoint(tmp_path / "c.pth", cl2, BaseScheduler(1.0))
    for c, c2 in zip(cl, cl2):  # client k restored into its own (different) row
        _check_same(c.model.state_dict(), c2.model.state_dict())
        assert common_pool([c2.model]) is not None  # still bound: the pool rows were written


def test_bound_row_tracks_rebinding():
    """row_of: a bound module stays bound while every state entry is its row view; param.data
    assignment, a re-registered buffer or module.to() copies unbind it (checked per entry
    through the tables kept at bind time)."""
    from topology_aware_learning_amd.arena import bound_row

    cl, pool = _bound([0, 1])
    m = cl[0].model
    assert bound_row(m) == (pool, 0) and pool.row_of(cl[1].model) == 1
    m.fc.weight.data = m.fc.weight.data.clone()
    assert bound_row(m) is None
    pool.bind(m, 0)
    assert bound_row(m) == (pool, 0)
    m.bn.running_mean = m.bn.running_mean.clone()
    assert bound_row(m) is None
    pool.bind(m, 0)
    m.bn2.num_batches_tracked = m.bn2.num_batches_tracked.clone()
    assert bound_row(m) is None
    pool.bind(m, 0)
    m.to(torch.float64)
    assert bound_row(m) is None
    pool.bind(m.to(torch.float32), 0)
    assert bound_row(m) == (pool, 0)
    m.fc.bias = None  # an entry removed from its table
    assert bound_row(m) is None


def test_bound_row_generation_hooks():
    """The O(1) binding check (arena._GEN): every re-pointing path bumps the generation and is
    then caught by the full check - submodule replaced, parameter / buffer set to None or
    deleted, `.to()` of a submodule, parameter `.data` assignment, load_state_dict(assign=True);
    an in-place load_state_dict and unrelated module construction keep the binding."""
    import torch.nn as nn

    from topology_aware_learning_amd import arena
    from topology_aware_learning_amd.arena import ModelPool, StateLayout, bound_row

    def mk():
        m = nn.Sequential(nn.Linear(3, 4), nn.BatchNorm1d(4), nn.Linear(4, 2))
        pool = ModelPool(StateLayout.from_state_dict(m.state_dict()), 1, "cpu")
        pool.bind(m, 0)
        assert bound_row(m) == (pool, 0)
        return m, pool

    cases = [
        lambda m: m.__setitem__(0, nn.Linear(3, 4)),
        lambda m: setattr(m[1], "running_var", None),
        lambda m: delattr(m[2], "bias"),
        lambda m: m[2].to(torch.float64),
        lambda m: setattr(m[2].weight, "data", m[2].weight.data.clone()),
        lambda m: m.load_state_dict({k: v.clone() for k, v in m.state_dict().items()}, assign=True),
        lambda m: setattr(m[1], "running_mean", m[1].running_mean.clone()),
    ]
    for k, change in enumerate(cases):
        m, _ = mk()
        g = arena._GEN[0]
        change(m)
        assert arena._GEN[0] != g, k
        assert bound_row(m) is None, k
    m, pool = mk()
    m.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})  # copy_: still bound
    nn.Linear(2, 2)  # a hook event elsewhere: one full check, then O(1) again
    assert bound_row(m) == (pool, 0) and m._tal_gen == arena._GEN[0]
    assert bound_row(m) == (pool, 0)
