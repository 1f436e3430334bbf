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


def _seg_setup(dtype, n_dev, seed):
    """Layout + pool of one test: fp32 or bf16 weights (bf16 kept as uint16 bit patterns)."""
    dt = "float32" if dtype == "f32" else "bfloat16"
    layout = StateLayout.from_layout([("w", (1001,), dt), ("b", (7,), dt), ("nbt", (), "int64")])
    rng = np.random.default_rng(seed)
    pool = rng.standard_normal((n_dev, 1008)).astype(np.float32)
    if dtype == "bf16":
        pool = oracle.f32_to_bf16(pool)
    ipool = rng.integers(0, 10 ** 6, size=(n_dev, 1)).astype(np.int64)
    return layout, pool, ipool


def _put_row(pool_obj, k, dtype, row, irow, cuda):
    if dtype == "f32":
        pool_obj.f32[k, :1008] = torch.from_numpy(row).to(cuda)
    else:
        pool_obj.b16[k, :1008] = torch.from_numpy(row.view(np.int16)).to(cuda).view(torch.bfloat16)
    pool_obj.i64[k, :1] = torch.from_numpy(irow).to(cuda)


def _get_rows(pool_obj, rows, dtype):
    if dtype == "f32":
        return pool_obj.f32[:rows, :1008].cpu().numpy().view(np.uint32)
    return pool_obj.b16[:rows, :1008].cpu().view(torch.int16).numpy().view(np.uint16)


def _oracle_round(dtype, pool, rp, col, w, n):
    if dtype == "f32":
        return oracle.round_f32(pool, rp, col, w, np.arange(n))
    return oracle.round_bf16(pool, rp, col, w, np.arange(n), exact=True)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("graph,world", [("regular", 4), ("barbell", 8), ("ring", 2)])
def test_virtual_ranks_two_rounds(cuda, graph, world, dtype):
    g = {"regular": nx.random_regular_graph(8, 48, seed=0), "barbell": nx.barbell_graph(20, 8),
         "ring": nx.cycle_graph(12)}[graph]
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    layout, pool, ipool = _seg_setup(dtype, n, 1)
    owner = partition_contiguous(n, world)
    srs = [ShardedRound(layout, orders, ws, r, world, cuda, exchange=lambda sr: []) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.spec.own):
            _put_row(sr.pool_a, k, dtype, pool[gid], ipool[gid], cuda)

    def exchange_all():
        for sr in srs:
            base = len(sr.spec.own)
            for k, gid in enumerate(sr.spec.halo):
                src = srs[owner[gid]]
                for _, t, _ in sr.pool_a.segments():
                    st = {id(sr.pool_a.f32): src.pool_a.f32, id(sr.pool_a.b16): src.pool_a.b16,
                          id(sr.pool_a.i64): src.pool_a.i64}[id(t)]
                    t[base + k].copy_(st[src.spec.local_of[gid]])

    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        exchange_all()
        for sr in srs:
            sr.step()
        ref = _oracle_round(dtype, ref, rp, col, w, n)
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    for sr in srs:
        assert sr.spot_check()
        got = _get_rows(sr.own_rows(), len(sr.spec.own), dtype)
        assert np.array_equal(got, ref[sr.spec.own].view(got.dtype))
        assert np.array_equal(sr.own_rows().i64[: len(sr.spec.own), :1].cpu().numpy(), iref[sr.spec.own])


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("graph,world", [("regular", 4), ("barbell", 8), ("ring", 3)])
def test_virtual_ranks_transposed_two_rounds(cuda, graph, world, dtype, chunks):
    """TransposedRound (column blocks by all-to-all) with the two all-to-alls done by in-process
    copies between virtual ranks: K3 on each rank's column block, bitwise the oracle round."""
    from topology_aware_learning_amd.transposed import TransposedRound

    g = {"regular": nx.random_regular_graph(8, 48, seed=0), "barbell": nx.barbell_graph(20, 8),
         "ring": nx.cycle_graph(13)}[graph]
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    layout, pool, ipool = _seg_setup(dtype, n, 2)
    owner = np.array([(5 * i) % world for i in range(n)], np.int32)  # interleaved owners
    srs = [TransposedRound(layout, orders, ws, r, world, cuda, owner=owner, chunks=chunks) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.own):
            _put_row(sr.pool_a, k, dtype, pool[gid], ipool[gid], cuda)
    base = srs[0].base
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        for k in range(srs[0].chunks):
            for sr in srs:
                sr.pack(k)
            for r, sr in enumerate(srs):  # forward all-to-all: chunk k of block r of every model
                for key, s in sr._segs_at(k):
                    for p, src in enumerate(srs):
                        s.work_in[k][base[p]: base[p + 1]].copy_(src.segs[key].send[k][r])
            for sr in srs:
                sr.compute(k)
            for r, sr in enumerate(srs):  # backward all-to-all: my rows of every rank's chunk
                for key, s in sr._segs_at(k):
                    for p, src in enumerate(srs):
                        s.back[k][p].copy_(src.segs[key].work_out[k][base[r]: base[r + 1]])
            for sr in srs:
                sr.unpack(k)
        ref = _oracle_round(dtype, ref, rp, col, w, n)
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    for sr in srs:
        assert sr.spot_check()
        got = _get_rows(sr.own_rows(), sr.local_rows, dtype)
        assert np.array_equal(got, ref[sr.own].view(got.dtype))
        assert np.array_equal(sr.own_rows().i64[: sr.local_rows, :1].cpu().numpy(), iref[sr.own])


@pytest.mark.parametrize("exchange,world", [("halo", 2), ("transpose", 2), ("transpose", 3), ("halo", 3)])
def test_bench_multi_rank_rehearsal(cuda, tmp_path, exchange, world):
    """bench.py's N > 1 branch end to end (make_round, tuning, exchange, spot check, timing, JSON)
    with `world` ranks sharing this GPU over gloo (exchange staged through host memory): the
    same code the 8-GPU RCCL run executes, except the transport."""
    import json
    import os
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    port = 29500 + (os.getpid() % 400) + world * 7 + (0 if exchange == "halo" else 3)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), "--gpus", str(world),
           "--dist-backend", "gloo", "--exchange", exchange, "--model", "cifar10", "--devices-per-gpu", "16",
           "--degree", "4", "--steps", "2", "--warmup", "1", "--no-tune"]
    out = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == world and d["parity"] is True and d["exchange"] == exchange
    assert d["value"] > 0 and d["link_bytes_in_per_round"] > 0
