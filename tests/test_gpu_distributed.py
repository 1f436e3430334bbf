"""Sharded rounds on the GPU: K3 kernels over per-rank pools (interior + boundary plans,
double buffering) with the halo exchange replaced by in-process device copies — the same
ShardedRound the multi-GPU bench runs over RCCL — checked bit for bit against the oracle."""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import synth
from topology_aware_learning_amd.arena import StateLayout
from topology_aware_learning_amd.distributed import ShardedRound, partition_contiguous

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graph,world", [("regular", 4), ("barbell", 8), ("ring", 2)])
def test_virtual_ranks_two_rounds(cuda, graph, world):
    g = {"regular": nx.random_regular_graph(8, 48, seed=0), "barbell": nx.barbell_graph(20, 8),
         "ring": nx.cycle_graph(12)}[graph]
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    lay = [("w", (1001,), "float32"), ("b", (7,), "float32"), ("nbt", (), "int64")]
    layout = StateLayout.from_layout(lay)
    rng = np.random.default_rng(1)
    pool = rng.standard_normal((n, layout.n_f32)).astype(np.float32)
    ipool = rng.integers(0, 10 ** 6, size=(n, 1)).astype(np.int64)
    owner = partition_contiguous(n, world)
    srs = [ShardedRound(layout, orders, ws, r, world, cuda, exchange=lambda sr: []) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.spec.own):
            sr.pool_a.f32[k, : layout.n_f32] = torch.from_numpy(pool[gid]).to(cuda)
            sr.pool_a.i64[k, :1] = torch.from_numpy(ipool[gid]).to(cuda)

    def exchange_all():
        for sr in srs:
            base = len(sr.spec.own)
            for k, gid in enumerate(sr.spec.halo):
                src = srs[owner[gid]]
                sr.pool_a.f32[base + k].copy_(src.pool_a.f32[src.spec.local_of[gid]])
                sr.pool_a.i64[base + k].copy_(src.pool_a.i64[src.spec.local_of[gid]])

    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        exchange_all()
        for sr in srs:
            sr.step()
        ref = oracle.round_f32(ref, rp, col, w, np.arange(n))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    for sr in srs:
        got = sr.own_rows().f32[: len(sr.spec.own), : layout.n_f32].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref[sr.spec.own].view(np.uint32))
        assert np.array_equal(sr.own_rows().i64[: len(sr.spec.own), :1].cpu().numpy(), iref[sr.spec.own])


@pytest.mark.parametrize("graph,world", [("regular", 4), ("barbell", 8), ("ring", 3)])
def test_virtual_ranks_transposed_two_rounds(cuda, graph, world):
    """TransposedRound (column blocks by all-to-all) with the two all-to-alls done by in-process
    copies between virtual ranks: K3 on each rank's column block, bitwise the oracle round."""
    from topology_aware_learning_amd.transposed import TransposedRound

    g = {"regular": nx.random_regular_graph(8, 48, seed=0), "barbell": nx.barbell_graph(20, 8),
         "ring": nx.cycle_graph(13)}[graph]
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    lay = [("w", (1001,), "float32"), ("b", (7,), "float32"), ("nbt", (), "int64")]
    layout = StateLayout.from_layout(lay)
    rng = np.random.default_rng(2)
    pool = rng.standard_normal((n, layout.n_f32)).astype(np.float32)
    ipool = rng.integers(0, 10 ** 6, size=(n, 1)).astype(np.int64)
    owner = np.array([(5 * i) % world for i in range(n)], np.int32)  # interleaved owners
    srs = [TransposedRound(layout, orders, ws, r, world, cuda, owner=owner) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.own):
            sr.pool_a.f32[k, : layout.n_f32] = torch.from_numpy(pool[gid]).to(cuda)
            sr.pool_a.i64[k, :1] = torch.from_numpy(ipool[gid]).to(cuda)
    base = srs[0].base
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        for sr in srs:
            sr.pack()
        for r, sr in enumerate(srs):  # forward all-to-all: block r of every rank's models
            for key, s in sr.segs.items():
                for p, src in enumerate(srs):
                    s.work_in[base[p]: base[p + 1]].copy_(src.segs[key].send[r])
        for sr in srs:
            sr.compute()
        for r, sr in enumerate(srs):  # backward all-to-all: my rows of every rank's block
            for key, s in sr.segs.items():
                for p, src in enumerate(srs):
                    s.back[p].copy_(src.segs[key].work_out[base[r]: base[r + 1]])
        for sr in srs:
            sr.unpack()
        ref = oracle.round_f32(ref, rp, col, w, np.arange(n))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    for sr in srs:
        assert sr.spot_check()
        got = sr.own_rows().f32[: sr.local_rows, : layout.n_f32].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref[sr.own].view(np.uint32))
        assert np.array_equal(sr.own_rows().i64[: sr.local_rows, :1].cpu().numpy(), iref[sr.own])
