"""The reference's driver on several GPUs of its one process (multipool.MultiPool, TAL_GPUS).

The reference runs every aggregation in one coordinator process
(/root/reference/src/experiments/parsl_setup.py:75-78, /root/reference/src/decentralized_app.py:
605-641).  Here its clients are spread over N GPUs in contiguous blocks, each GPU's pool holding
its own clients and ghost rows of the neighbors other GPUs own.

CPU: the partition (own blocks, ghost rows from the topology, contiguous per-owner ghost blocks),
the copy transport's full halo and the per-call ghost refresh on CPU pools; the C-ABI refuses a
local communicator over repeated devices.  GPU (one GPU, `TAL_VIRTUAL_GPUS`: N pools on it, copy
transport): decentralized_main.py unchanged on a barbell graph cut to 20 clients, batched rounds
(every ghost row equal to its owner's row after the halo, every GPU's round bitwise the oracle's
snapshot round) and per-call rounds (every app call bitwise the oracle on the operands as their
owners hold them).  The RCCL leg (tal_comm_init_local / tal_halo_exchange_local) needs >= 2
GPUs: unmeasured until a multi-GPU box runs `test_rccl_local_halo`.
"""
from __future__ import annotations

import threading

import networkx as nx
import numpy as np
import pytest
import torch

from topology_aware_learning_amd import synth
from topology_aware_learning_amd.arena import ModelPool, StateLayout
from topology_aware_learning_amd.multipool import MultiPool

_LAY = [("w", (257,), "float32"), ("b", (5, 3), "float32"), ("n", (), "int64")]


def _fill_own(mp: MultiPool, seed: int = 0) -> None:
    rng = np.random.default_rng(seed)
    for g, p in enumerate(mp.pools):
        for gid in mp.own[g]:
            r = mp.local[g][gid]
            p.f32[r].copy_(torch.from_numpy(rng.standard_normal(p.f32.shape[1]).astype(np.float32)) + gid)
            p.i64[r].fill_(1000 + gid)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_partition_and_ghost_blocks(world):
    g = nx.barbell_graph(8, 4)
    adj = nx.to_numpy_array(g)
    n = adj.shape[0]
    mp = MultiPool(StateLayout.from_layout(_LAY), n, ["cpu"] * world, adjacency=adj)
    assert mp.transport == "copy"
    assert sorted(j for own in mp.own for j in own) == list(range(n))
    for q in range(world):
        own = set(mp.own[q])
        assert mp.own[q] == sorted(own) and max(own) - min(own) + 1 == len(own)  # contiguous block
        want = sorted({j for i in own for j in g.neighbors(i) if j not in own})
        assert sorted(mp.halo[q]) == want
        assert mp.pools[q].rows == len(own) + len(want)
        for h, (first, cnt) in mp.ghost_block[q].items():  # grouped by owner, ascending ids
            ids = [j for j in mp.halo[q] if mp.owner[j] == h]
            assert [mp.local[q][j] for j in ids] == list(range(first, first + cnt))
            assert ids == sorted(ids)
        for gid in mp.own[q]:
            assert mp.home(gid) == (q, mp.local[q][gid])


def test_full_mesh_without_adjacency():
    mp = MultiPool(StateLayout.from_layout(_LAY), 9, ["cpu"] * 3)
    for q in range(3):
        assert len(mp.halo[q]) == 6 and mp.pools[q].rows == 9


def test_copy_halo_and_per_call_refresh():
    adj = nx.to_numpy_array(nx.cycle_graph(12))
    mp = MultiPool(StateLayout.from_layout(_LAY), 12, ["cpu"] * 3, adjacency=adj)
    _fill_own(mp, 1)
    mp.exchange_halo()
    for q in range(3):
        for gid in mp.halo[q]:
            h, r = mp.home(gid)
            gr = mp.local[q][gid]
            assert torch.equal(mp.pools[q].f32[gr], mp.pools[h].f32[r])
            assert torch.equal(mp.pools[q].i64[gr], mp.pools[h].i64[r])
    # an owner row changes (a neighbor's per-call aggregation): the next read refreshes the ghost
    h, r = mp.home(4)
    mp.pools[h].f32[r].add_(1.0)
    q = int(mp.owner[3])
    assert q != h
    rows = mp.rows_for(q, [(mp.pools[h], r), (mp.pools[q], mp.local[q][3])])
    assert rows == [mp.local[q][4], mp.local[q][3]]
    assert torch.equal(mp.pools[q].f32[rows[0]], mp.pools[h].f32[r])
    with pytest.raises(ValueError):  # client 9 is no neighbor of GPU q's clients on a ring
        h9, r9 = mp.home(9)
        mp.rows_for(q, [(mp.pools[h9], r9)])


def test_halo_bytes():
    lay = StateLayout.from_layout(_LAY)
    mp = MultiPool(lay, 12, ["cpu"] * 3, adjacency=nx.to_numpy_array(nx.cycle_graph(12)))
    row = 4 * lay.ld_f32 + 8 * lay.ld_i64
    hb = mp.halo_bytes()
    assert hb["busiest_pair"] == row and hb["total"] == 6 * row  # a ring: one model per neighbor GPU and side


def test_local_comm_refuses_repeated_devices():
    import ctypes

    from topology_aware_learning_amd import _lib

    comms = (ctypes.c_void_p * 2)()
    dev = (ctypes.c_int32 * 2)(0, 0)
    assert _lib.load().tal_comm_init_local(comms, 2, dev) == _lib.TAL_ERR_INVALID
    with pytest.raises(ValueError):
        MultiPool(StateLayout.from_layout(_LAY), 4, ["cpu"] * 2, transport="rccl")


# ------------------------------------------------------------------------------------------
# GPU: the reference's driver over virtual GPUs (pools sharing cuda:0, copy transport)
# ------------------------------------------------------------------------------------------
def _barbell_file(tmp_path):
    topo = tmp_path / "barbell20.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.barbell_graph(8, 4)), fmt="%d")  # 8 + 4 + 8 clients
    return topo


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,world", [("degCent", 4), ("unweighted", 3)])
def test_driver_batched_round_virtual_gpus(cuda, tmp_path, monkeypatch, strategy, world):
    """TAL_VIRTUAL_GPUS + TAL_BATCHED_ROUND: decentralized_main.py unchanged over `world` pools;
    after every halo each ghost row equals its owner's row bitwise, and each GPU's share of the
    round (double-buffered, the ghost rows not carried into the spare) equals the oracle's
    snapshot round over that pool (own and ghost rows in) on the pool's own rows, so the whole
    round is the snapshot round of the models after training."""
    import oracle
    from oracle import reference_alg as ra
    from topology_aware_learning_amd.round import RoundExecutor

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_BATCHED_ROUND", "1")
    monkeypatch.setenv("TAL_VIRTUAL_GPUS", str(world))
    monkeypatch.setenv("TAL_POOL_PLACEMENT_TRIALS", "1")
    real_halo, real_run = MultiPool.exchange_halo, RoundExecutor.run
    seen = dict(halos=0, rows=[])

    def checked_halo(self):
        real_halo(self)
        for q in range(self.world):
            for gid in self.halo[q]:
                h, r = self.home(gid)
                gr = self.local[q][gid]
                assert torch.equal(self.pools[q].f32[gr], self.pools[h].f32[r]), (q, gid)
                assert torch.equal(self.pools[q].i64[gr], self.pools[h].i64[r]), (q, gid)
        seen["halos"] += 1

    def checked_run(self, orders, weights, out_rows=None, sequential=False, plan=None):
        lay = self.pool.layout
        f_in = self.pool.f32[:, : lay.n_f32].cpu().numpy().copy()
        i_in = self.pool.i64[:, : lay.n_i64].cpu().numpy().copy()
        real_run(self, orders, weights, out_rows, sequential, plan)
        rp, col, w = ra.round_csr(orders, weights)
        ref, iref = f_in.copy(), i_in.copy()
        oracle.round_f32(f_in, rp, col, w, np.asarray(out_rows), pool_out=ref)
        oracle.round_i64(i_in, rp, col, w, np.asarray(out_rows), pool_out=iref)
        k = self.carried_rows  # the pool's own rows (ghost rows: stale until the next halo)
        assert self.double_buffer and self.swaps >= 1 and k < self.pool.rows
        assert np.array_equal(self.pool.f32[:k, : lay.n_f32].cpu().numpy().view(np.uint32), ref[:k].view(np.uint32))
        assert np.array_equal(self.pool.i64[:k, : lay.n_i64].cpu().numpy(), iref[:k])
        seen["rows"].append(len(out_rows))

    monkeypatch.setattr(MultiPool, "exchange_halo", checked_halo)
    monkeypatch.setattr(RoundExecutor, "run", checked_run)
    from src.experiments import decentralized_main

    args = ["--dataset", "cifar10", "--aggregation_strategy", strategy, "--rounds", "2", "--epochs", "1",
            "--topology_file", str(_barbell_file(tmp_path)), "--out_dir", str(tmp_path / "logs"), "--batch_size", "32"]
    if strategy == "degCent":
        args.append("--softmax")
    assert decentralized_main.main(args) == 0
    assert seen["halos"] == 2 and sum(seen["rows"]) == 40 and len(seen["rows"]) == 2 * world


@pytest.mark.gpu
def test_driver_per_call_virtual_gpus(cuda, tmp_path, monkeypatch):
    """TAL_VIRTUAL_GPUS, the reference's per-call round: every app call (operands on other GPUs
    read through refreshed ghost rows) equals the oracle's aggregation of the operands as their
    owners hold them at that moment, bitwise; calls are made atomic with their check by a lock
    (the app pool runs two at once, as the reference's)."""
    import oracle
    from topology_aware_learning_amd import aggregate as agg_mod
    from topology_aware_learning_amd.arena import bound_row

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_VIRTUAL_GPUS", "4")
    monkeypatch.setenv("TAL_POOL_PLACEMENT_TRIALS", "1")
    real = agg_mod.aggregate_models
    lock = threading.Lock()
    calls = []

    def home_rows(m):
        pool, r = bound_row(m)
        return pool.f32[r, : pool.layout.n_f32].cpu().numpy().copy(), pool.i64[r, : pool.layout.n_i64].cpu().numpy().copy()

    def checked(operands, weights, target, mode=1):  # ops.MODE_EXACT, the apps' mode
        with lock:
            xs = [home_rows(m) for m in operands]
            out = real(operands, weights, target, mode)
            got_f, got_i = home_rows(target)
            ref_f = oracle.agg_f32([x[0] for x in xs], list(weights))
            ref_i = oracle.agg_i64([x[1] for x in xs], list(weights))
            assert np.array_equal(got_f.view(np.uint32), ref_f.view(np.uint32))
            assert np.array_equal(got_i, ref_i)
            calls.append(len(operands))
            return out

    import src.decentralized_client as dc

    monkeypatch.setattr(dc, "aggregate_models", checked)  # the apps' binding (decentralized_client.py)
    from src.experiments import decentralized_main

    args = ["--dataset", "cifar10", "--aggregation_strategy", "unweighted", "--rounds", "2", "--epochs", "1",
            "--topology_file", str(_barbell_file(tmp_path)), "--out_dir", str(tmp_path / "logs"), "--batch_size", "32"]
    assert decentralized_main.main(args) == 0
    assert len(calls) == 40


@pytest.mark.gpu
def test_rccl_local_halo(cuda):
    """The RCCL leg: tal_comm_init_local over this process's GPUs and one full halo through
    tal_halo_exchange_local, ghost rows bitwise their owners' rows.  Needs >= 2 GPUs."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("one GPU: the in-process RCCL halo needs >= 2 (unmeasured on this box)")
    lay = StateLayout.from_layout(synth.truncate_layout(synth.get_layout("resnet50"), 1 << 16))
    adj = nx.to_numpy_array(nx.random_regular_graph(4, 8 * n, seed=0))
    mp = MultiPool(lay, 8 * n, [torch.device("cuda", k) for k in range(n)], adjacency=adj)
    assert mp.transport == "rccl"
    _fill_own(mp, 3)
    mp.exchange_halo()
    for d in mp.devices:
        torch.cuda.synchronize(d)
    for q in range(n):
        for gid in mp.halo[q]:
            h, r = mp.home(gid)
            gr = mp.local[q][gid]
            assert torch.equal(mp.pools[q].f32[gr].cpu(), mp.pools[h].f32[r].cpu())
    mp.close()
