"""The C-ABI halo exchange (include/tal_agg.h, halo section) on one GPU: the gather kernel
against torch indexing, a world-1 RCCL communicator sending to itself, argument errors, and a
sharded round whose exchange goes through the library (transport "cabi") against the oracle.
Multi-rank transport needs one GPU per rank (the driver's 8-GPU run); the same per-peer
messages are rehearsed across ranks by tests/test_distributed_gloo.py."""
import numpy as np
import pytest
import torch

import oracle
from topology_aware_learning_amd import _lib
from topology_aware_learning_amd.comm import HaloComm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm1(cuda):
    c = HaloComm(1, 0, HaloComm.unique_id(), cuda)
    yield c
    c.close()


@pytest.mark.parametrize("dtype,ld", [(torch.float32, 1028), (torch.bfloat16, 1030), (torch.int64, 53),
                                      (torch.float32, 4096)])
def test_pack_gathers_rows(cuda, dtype, ld):
    """16-B lanes when rows and pitch allow it (fp32 1028 / 4096), 4-B lanes otherwise."""
    g = torch.Generator().manual_seed(ld)
    pool = (torch.randn(10, ld, generator=g) * 1e3).to(dtype).to(cuda)
    rows = torch.tensor([5, 2, 7, 2, 9], dtype=torch.int32, device=cuda)
    out = torch.empty((5, ld), dtype=dtype, device=cuda)
    HaloComm.pack(pool, rows, out)
    assert torch.equal(out, pool[rows.long()])


def test_pack_skips_rows_out_of_range(cuda):
    pool = torch.arange(40, dtype=torch.float32, device=cuda).view(4, 10)
    out = torch.full((2, 10), -7.0, device=cuda)
    HaloComm.pack(pool, torch.tensor([1, 99], dtype=torch.int32, device=cuda), out)
    assert torch.equal(out[0], pool[1]) and bool((out[1] == -7.0).all())


def test_exchange_to_self(cuda, comm1):
    g = torch.Generator().manual_seed(3)
    pool = torch.randn(12, 2048, generator=g).to(cuda)
    rows = torch.tensor([11, 0, 4], dtype=torch.int32, device=cuda)
    send = HaloComm.pack(pool, rows, torch.empty((3, 2048), device=cuda))
    recv = torch.zeros_like(send)
    comm1.exchange([send], [recv])
    torch.cuda.synchronize()
    assert torch.equal(recv, pool[rows.long()])
    comm1.exchange([None], [None])  # nothing to move: an empty group
    torch.cuda.synchronize()


def test_exchange_rejects_wrong_world(cuda, comm1):
    x = torch.zeros(4, device=cuda)
    with pytest.raises(ValueError):
        comm1.exchange([x, x], [x, x])
    L = _lib.load()
    import ctypes

    sb = (ctypes.c_void_p * 2)()
    n = (ctypes.c_int64 * 2)(0, 0)
    assert L.tal_halo_exchange(comm1._comm, 2, sb, n, sb, n, None) == _lib.TAL_ERR_INVALID
    assert b"communicator's size" in L.tal_last_error()


def test_sharded_round_through_cabi_transport(cuda, tmp_path):
    """A world-1 torch.distributed group (gloo, for the unique-id broadcast) and a ShardedRound
    whose exchange is the library's: the round equals the oracle bit for bit."""
    import networkx as nx
    import torch.distributed as dist

    from topology_aware_learning_amd.arena import StateLayout
    from topology_aware_learning_amd.distributed import ShardedRound

    init = f"file://{tmp_path}/pg"
    dist.init_process_group("gloo", init_method=init, rank=0, world_size=1)
    try:
        g = nx.random_regular_graph(4, 12, seed=1)
        orders = [sorted(g.neighbors(i)) + [i] for i in range(12)]
        weights = [[1 / len(o)] * len(o) for o in orders]
        lay = StateLayout.from_layout([("w", (70001,), "float32"), ("b", (13,), "float32"), ("nbt", (), "int64")])
        sr = ShardedRound(lay, orders, weights, 0, 1, cuda, transport="cabi")
        gen = torch.Generator(device=cuda).manual_seed(7)
        sr.pool_a.f32.normal_(generator=gen)
        sr.pool_a.i64.random_(0, 1000, generator=gen)
        before = sr.pool_a.f32[:, : lay.n_f32].cpu().numpy().copy()
        sr.step()
        torch.cuda.synchronize()
        row_ptr = np.cumsum([0] + [len(o) for o in orders]).astype(np.int32)
        col = np.concatenate(orders).astype(np.int32)
        w = np.concatenate(weights)
        ref = oracle.round_f32(before, row_ptr, col, w, np.arange(12, dtype=np.int32))
        got = sr.pool_a.f32[:, : lay.n_f32].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        sr.comm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("graph,world,dtype", [("regular", 4, "f32"), ("sbm256", 8, "f32"), ("sbm256", 8, "bf16"),
                                               ("barbell60", 8, "bf16"), ("ring", 2, "bf16")])
def test_virtual_ranks_messages_from_cabi_pack(cuda, graph, world, dtype):
    """The multi-rank 'cabi' transport's messages without a second GPU: `world` ShardedRounds
    in one process, each peer's message built exactly as post_exchange_cabi builds it (the
    library's gather kernel into the HaloPacker buffers, or the consecutive-row view) and copied
    into the receiver's halo block, two rounds, bitwise the oracle.  (RCCL refuses two ranks on
    one GPU, so the exchange itself runs across ranks only on the driver's node.)"""
    from test_gpu_distributed import _get_rows, _graph, _put_row, _seg_setup

    from oracle import reference_alg as ra
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.distributed import ShardedRound, recv_range

    g = _graph(graph)
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    layout, pool, ipool = _seg_setup(dtype, n, 2)
    srs = [ShardedRound(layout, orders, ws, r, world, cuda, exchange=lambda sr: []) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.spec.own):
            _put_row(sr.pool_a, k, dtype, pool[gid], ipool[gid], cuda)
    packed = 0
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        for sr in srs:  # post_exchange_cabi's message construction, peer by peer
            for peer in sr.spec.recv:
                r0, r1 = recv_range(sr.spec, peer)
                src = srs[peer]
                for si, (_, t, _) in enumerate(sr.pool_a.segments()):
                    ts = src.pool_a.segments()[si][1]
                    pk = src.packers[si]
                    if sr.spec.rank in pk.idx32:
                        msg = HaloComm.pack(ts, pk.idx32[sr.spec.rank], pk.bufs[sr.spec.rank])
                        packed += 1
                    else:
                        rows = src.spec.send[sr.spec.rank]
                        msg = ts[rows[0]: rows[0] + len(rows)]
                    t[r0:r1].copy_(msg)
        for sr in srs:
            sr.step()
        ref = (oracle.round_f32(ref, rp, col, w, np.arange(n)) if dtype == "f32"
               else oracle.round_bf16(ref, rp, col, w, np.arange(n)))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    # the gather kernel ran (regular at world 2 or 3, barbell60 at 8 and rings send consecutive
    # rows: views only)
    assert packed > 0 or graph in ("ring", "barbell60")
    for sr in srs:
        got = _get_rows(sr.own_rows(), len(sr.spec.own), dtype)
        assert np.array_equal(got, ref[sr.spec.own].view(got.dtype))
        assert np.array_equal(sr.own_rows().i64[: len(sr.spec.own), :1].cpu().numpy(), iref[sr.spec.own])


@pytest.mark.parametrize("graph,world,dtype,chunks", [("regular", 4, "f32", 1), ("sbm256", 8, "f32", 2),
                                                      ("barbell60", 8, "bf16", 3), ("ring", 3, "bf16", 1)])
def test_virtual_ranks_transposed_through_cabi_exchange(cuda, comm1, graph, world, dtype, chunks):
    """The transposed exchange's C-ABI transport without a second GPU: `world` TransposedRounds
    in one process; every per-peer message of both all-to-alls (forward_messages /
    backward_messages, exactly the tensors _exchange_cabi hands to tal_halo_exchange) moves
    through the library's RCCL communicator - a world-1 communicator sending rank p's message
    to itself into rank r's receive buffer - two rounds, bitwise the oracle."""
    from test_gpu_distributed import _get_rows, _graph, _put_row, _seg_setup

    from oracle import reference_alg as ra
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.distributed import partition_contiguous
    from topology_aware_learning_amd.transposed import TransposedRound

    import networkx as nx

    g = nx.cycle_graph(13) if graph == "ring" else _graph(graph)
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    layout, pool, ipool = _seg_setup(dtype, n, 3)
    owner = partition_contiguous(n, world)
    srs = [TransposedRound(layout, orders, ws, r, world, cuda, owner=owner, chunks=chunks) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.own):
            _put_row(sr.pool_a, k, dtype, pool[gid], ipool[gid], cuda)
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    moved = 0

    def through_comm(messages, k):
        nonlocal moved
        for r, sr in enumerate(srs):
            for key, _ in sr._segs_at(k):
                recvs = messages(sr, k, key)[1]
                for p in sr.peers():
                    send = messages(srs[p], k, key)[0][r]
                    assert send.shape == recvs[p].shape and send.is_contiguous() and recvs[p].is_contiguous()
                    if send.numel():
                        comm1.exchange([send], [recvs[p]])
                        moved += 1

    for _ in range(2):
        for k in range(srs[0].chunks):
            for sr in srs:
                sr.pack(k)
            through_comm(lambda sr, k, key: sr.forward_messages(k, key), k)
            for sr in srs:
                sr.compute(k)
            through_comm(lambda sr, k, key: sr.backward_messages(k, key), k)
            for sr in srs:
                sr.unpack(k)
        ref = (oracle.round_f32(ref, rp, col, w, np.arange(n)) if dtype == "f32"
               else oracle.round_bf16(ref, rp, col, w, np.arange(n)))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    assert moved > 0
    for sr in srs:
        got = _get_rows(sr.own_rows(), sr.local_rows, dtype)
        assert np.array_equal(got, ref[sr.own].view(got.dtype))
        assert np.array_equal(sr.own_rows().i64[: sr.local_rows, :1].cpu().numpy(), iref[sr.own])


def test_transposed_round_cabi_transport_world1(cuda, tmp_path):
    """TransposedRound(transport="cabi") at world 1: the communicator is made through the
    library (unique id broadcast over the torch.distributed group), the own block never enters
    RCCL, the round equals the oracle bit for bit."""
    import networkx as nx
    import torch.distributed as dist

    from topology_aware_learning_amd.arena import StateLayout
    from topology_aware_learning_amd.transposed import make_round

    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        g = nx.random_regular_graph(4, 12, seed=1)
        orders = [sorted(g.neighbors(i)) + [i] for i in range(12)]
        weights = [[1 / len(o)] * len(o) for o in orders]
        lay = StateLayout.from_layout([("w", (70001,), "float32"), ("b", (13,), "float32"), ("nbt", (), "int64")])
        sr = make_round(lay, orders, weights, 0, 1, cuda, exchange="transpose", transport="cabi")
        assert sr.transport == "cabi" and sr.exchange_kind == "transpose"
        gen = torch.Generator(device=cuda).manual_seed(7)
        sr.pool_a.f32.normal_(generator=gen)
        before = sr.pool_a.f32[:, : lay.n_f32].cpu().numpy().copy()
        sr.step()
        torch.cuda.synchronize()
        rp = np.cumsum([0] + [len(o) for o in orders]).astype(np.int32)
        ref = oracle.round_f32(before, rp, np.concatenate(orders).astype(np.int32), np.concatenate(weights),
                               np.arange(12, dtype=np.int32))
        got = sr.pool_a.f32[:, : lay.n_f32].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        sr.comm.close()
    finally:
        dist.destroy_process_group()
