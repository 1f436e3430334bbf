"""Sharded rounds: halo plans and the P2P exchange on world_size 2 (gloo, CPU), checked
against the single-process oracle round.  The GPU form of the same path (K3 kernels + the
exchange) is in tests/test_gpu_distributed.py."""
import os
import socket

import networkx as nx
import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd.distributed import (HaloPacker, build_shard, partition_contiguous, post_exchange,
                                                    recv_range)


def problem(n=14, k=4, seed=3, width=203, kind="regular"):
    if kind == "regular":
        g = nx.random_regular_graph(k, n, seed=seed)
    else:  # BASELINE config 4 / 5 topologies (bench.make_graph), at reduced width
        import bench

        g = bench.make_graph({"barbell60": "barbell", "sbm256": "sbm"}[kind], 256, 0)
        n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.centrality_weights(o, nx.degree_centrality(g), True, 3.0) for o in orders]
    rng = np.random.default_rng(seed)
    pool = rng.standard_normal((n, width)).astype(np.float32)
    ipool = rng.integers(0, 10 ** 6, size=(n, 5)).astype(np.int64)
    return orders, ws, pool, ipool


def test_shard_specs_cover_the_round():
    orders, ws, _, _ = problem()
    owner = partition_contiguous(len(orders), 3)
    specs = [build_shard(orders, ws, owner, r, 3) for r in range(3)]
    assert sorted(sum((s.own for s in specs), [])) == list(range(len(orders)))
    for s in specs:
        for k, i in enumerate(s.own):
            glob = [([*s.own, *s.halo])[j] for j in s.orders_local[k]]
            assert glob == orders[i]
            assert (k in s.interior) != (k in s.boundary)
        for p, rows in s.recv.items():  # what I receive from p is exactly what p sends me
            mine = [([*s.own, *s.halo])[r] for r in rows]
            theirs = [specs[p].own[r] for r in specs[p].send[s.rank]]
            assert mine == theirs


@pytest.mark.parametrize("kind", ["barbell60", "sbm256"])
def test_halo_messages_one_per_peer(kind):
    """Per rank and segment: one send per peer (its rows gathered in the receiver's order) and
    one receive per peer into a contiguous halo block."""
    orders, ws, pool, _ = problem(kind=kind)
    owner = partition_contiguous(len(orders), 8)
    specs = [build_shard(orders, ws, owner, r, 8) for r in range(8)]
    tens = []
    for s in specs:
        t = torch.zeros(s.rows, pool.shape[1])
        for k, g in enumerate(s.own):
            t[k] = torch.from_numpy(pool[g])
        tens.append(t)
    for s, t in zip(specs, tens):
        for p in s.recv:
            r0, r1 = recv_range(s, p)
            msg = HaloPacker(specs[p], tens[p]).send_tensor(tens[p], s.rank)
            t[r0:r1] = msg
        glob = s.own + s.halo
        assert np.array_equal(t.numpy(), pool[glob])


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, world, port, out_dir, kind="regular"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orders, ws, pool, ipool = problem(kind=kind)
    owner = partition_contiguous(len(orders), world)
    spec = build_shard(orders, ws, owner, rank, world)
    glob_ids = spec.own + spec.halo
    f = torch.zeros(spec.rows, pool.shape[1])
    i = torch.zeros(spec.rows, ipool.shape[1], dtype=torch.int64)
    for k, g in enumerate(spec.own):
        f[k] = torch.from_numpy(pool[g])
        i[k] = torch.from_numpy(ipool[g])
    for r in post_exchange(spec, [f, i]):
        r.wait()
    assert np.array_equal(f.numpy(), pool[glob_ids]) and np.array_equal(i.numpy(), ipool[glob_ids])
    # the reduction itself: the oracle on the local pool (the GPU test runs the K3 kernel here)
    rp, col, w = ra.round_csr(spec.orders_local, spec.weights)
    out = oracle.round_f32(f.numpy(), rp, col, w, np.arange(len(spec.own)))
    iout = oracle.round_i64(i.numpy(), rp, col, w, np.arange(len(spec.own)))
    np.save(os.path.join(out_dir, f"r{rank}.npy"), out[: len(spec.own)])
    np.save(os.path.join(out_dir, f"i{rank}.npy"), iout[: len(spec.own)])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "regular"), (3, "regular"), (8, "barbell60"), (8, "sbm256")])
def test_gloo_exchange_matches_global_round(tmp_path, world, kind):
    """Halo exchange (one packed message per peer per segment) + local round on `world` gloo
    ranks == the single-process oracle round; barbell60 / sbm256 are BASELINE configs 4 / 5
    sharded 8 ways as bench.py --gpus 8 does (contiguous blocks)."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), kind), nprocs=world, join=True)
    orders, ws, pool, ipool = problem(kind=kind)
    rp, col, w = ra.round_csr(orders, ws)
    ref = oracle.round_f32(pool, rp, col, w, np.arange(len(orders)))
    iref = oracle.round_i64(ipool, rp, col, w, np.arange(len(orders)))
    got = np.concatenate([np.load(tmp_path / f"r{r}.npy") for r in range(world)])
    igot = np.concatenate([np.load(tmp_path / f"i{r}.npy") for r in range(world)])
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(igot, iref)


# ------------------------------------------------------------------------------------------
# transposed exchange (transposed.py): column blocks by all-to-all instead of halo rows

from topology_aware_learning_amd.transposed import (choose_exchange, column_blocks, exchange_bytes,  # noqa: E402
                                                    pack_columns, positions, unpack_columns)


@pytest.mark.parametrize("n,world", [(203, 1), (203, 2), (203, 3), (5, 4), (1, 3), (4096, 8)])
def test_column_blocks_pack_round_trip(n, world):
    b, blocks = column_blocks(n, world)
    assert b % 4 == 0 and sum(w for _, w in blocks) == n
    assert all(c0 == p * b and w <= b for p, (c0, w) in enumerate(blocks))
    rows, ld = 5, n + 7
    pool = torch.randn(rows, ld)
    send = torch.zeros(world * rows * b)
    pack_columns(pool, rows, blocks, b, send)
    back = torch.zeros(rows, ld)
    unpack_columns(send, rows, blocks, b, back)
    assert torch.equal(back[:, :n], pool[:, :n]) and not back[:, n:].any()


def test_exchange_choice_follows_link_bytes():
    import networkx as nx

    def orders_of(g):
        return [sorted(g.neighbors(i)) + [i] for i in range(g.number_of_nodes())]

    n_f, n_i = 23_573_962, 53
    reg = orders_of(nx.random_regular_graph(8, 512, seed=0))
    own8 = partition_contiguous(512, 8)
    b = exchange_bytes(reg, own8, 8, n_f, n_i)
    assert b["transpose"] == 2 * 64 * (4 * n_f + 8 * n_i) * 7 // 8
    assert b["halo"] > 2.5 * b["transpose"]  # ~280 of 448 remote models per rank
    assert choose_exchange(reg, own8, 8, n_f, n_i) == "transpose"
    reg2 = orders_of(nx.random_regular_graph(8, 128, seed=0))
    assert choose_exchange(reg2, partition_contiguous(128, 2), 2, n_f, n_i) == "halo"  # equal bytes
    ring = orders_of(nx.cycle_graph(64))
    assert choose_exchange(ring, partition_contiguous(64, 8), 8, n_f, n_i) == "halo"
    assert choose_exchange(ring, partition_contiguous(64, 1), 1, n_f, n_i) == "halo"


def _worker_transposed(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orders, ws, pool, ipool = problem()
    n_dev = len(orders)
    owner = np.array([(i * 7) % world for i in range(n_dev)], np.int32)  # not contiguous
    own_by_rank, base, pos = positions(owner, world)
    own = own_by_rank[rank]
    inv = np.empty(n_dev, np.int64)
    inv[pos] = np.arange(n_dev)
    outs = {}
    for name, data, dt in (("f", pool, torch.float32), ("i", ipool, torch.int64)):
        n = data.shape[1]
        b, blocks = column_blocks(n, world)
        mine = torch.zeros(len(own), n + 3, dtype=dt)
        mine[:, :n] = torch.from_numpy(data[own])
        send = torch.zeros(world * len(own) * b, dtype=dt)
        pack_columns(mine, len(own), blocks, b, send)
        work_in = torch.zeros(n_dev, b, dtype=dt)
        dist.all_to_all_single(work_in.view(-1), send, [len(o) * b for o in own_by_rank], [len(own) * b] * world)
        assert np.array_equal(work_in[:, : blocks[rank][1]].numpy(),
                              data[inv][:, blocks[rank][0]: blocks[rank][0] + blocks[rank][1]])
        # the round on this rank's column block, rows in rank-major order (the GPU test runs K3)
        rp, col, w = ra.round_csr([[int(pos[j]) for j in orders[int(inv[q])]] for q in range(n_dev)],
                                  [ws[int(inv[q])] for q in range(n_dev)])
        fn = oracle.round_f32 if dt == torch.float32 else oracle.round_i64
        work_out = torch.from_numpy(np.ascontiguousarray(fn(work_in.numpy(), rp, col, w, np.arange(n_dev))))
        back = torch.zeros(world * len(own) * b, dtype=dt)
        dist.all_to_all_single(back, work_out.view(-1), [len(own) * b] * world, [len(o) * b for o in own_by_rank])
        unpack_columns(back, len(own), blocks, b, mine)
        outs[name] = mine[:, :n].numpy()
    np.save(os.path.join(out_dir, f"tr{rank}.npy"), outs["f"])
    np.save(os.path.join(out_dir, f"ti{rank}.npy"), outs["i"])
    np.save(os.path.join(out_dir, f"town{rank}.npy"), np.asarray(own))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_transposed_exchange_matches_global_round(tmp_path, world):
    mp.spawn(_worker_transposed, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    orders, ws, pool, ipool = problem()
    rp, col, w = ra.round_csr(orders, ws)
    ref = oracle.round_f32(pool, rp, col, w, np.arange(len(orders)))
    iref = oracle.round_i64(ipool, rp, col, w, np.arange(len(orders)))
    for r in range(world):
        own = np.load(tmp_path / f"town{r}.npy")
        assert np.array_equal(np.load(tmp_path / f"tr{r}.npy").view(np.uint32), ref[own].view(np.uint32))
        assert np.array_equal(np.load(tmp_path / f"ti{r}.npy"), iref[own])


def _worker_transposed_class(rank, world, port, out_dir, chunks):
    """transposed.TransposedRound itself on CPU tensors over gloo (its own rank's column block
    packed and unpacked locally, the others by all-to-all with a zero split for itself); the
    K3 launch is replaced by the oracle round on the same work buffers - test infrastructure
    for a host without a GPU (tests/test_gpu_distributed.py runs the kernels)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from topology_aware_learning_amd import transposed as tr
    from topology_aware_learning_amd.arena import StateLayout

    orders, ws, pool, ipool = problem()
    n_dev = len(orders)
    owner = np.array([(i * 7) % world for i in range(n_dev)], np.int32)  # not contiguous
    layout = StateLayout.from_layout([("w", (pool.shape[1],), "float32"), ("c", (ipool.shape[1],), "int64")])
    sr = tr.TransposedRound(layout, orders, ws, rank, world, "cpu", owner=owner, chunks=chunks)
    rp, col, w = ra.round_csr(sr.orders_pos, sr.weights_pos)

    def oracle_segments(layout_, seg_in, seg_out, plan, mode, n_of=None):
        for g, fn in (("f32", oracle.round_f32), ("i64", oracle.round_i64)):
            n = n_of.get(g, 0)
            if n:
                x = np.ascontiguousarray(seg_in[g][:, :n].numpy())
                seg_out[g][:, :n] = torch.from_numpy(np.ascontiguousarray(fn(x, rp, col, w, np.arange(n_dev))))

    tr.run_round_segments = oracle_segments
    sr.pool_a.f32[:, : pool.shape[1]] = torch.from_numpy(pool[sr.own])
    sr.pool_a.i64[:, : ipool.shape[1]] = torch.from_numpy(ipool[sr.own])
    for _ in range(2):
        sr.step()
    np.save(os.path.join(out_dir, f"cr{rank}.npy"), sr.pool_a.f32[:, : pool.shape[1]].numpy())
    np.save(os.path.join(out_dir, f"ci{rank}.npy"), sr.pool_a.i64[:, : ipool.shape[1]].numpy())
    np.save(os.path.join(out_dir, f"cown{rank}.npy"), np.asarray(sr.own))
    np.save(os.path.join(out_dir, f"clink{rank}.npy"), np.asarray([sr.link_bytes]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(1, 1), (2, 1), (3, 2), (4, 3)])
def test_gloo_transposed_round_class_two_rounds(tmp_path, world, chunks):
    """TransposedRound.step on `world` CPU ranks: two rounds bitwise the oracle's two snapshot
    rounds; each rank's link bytes count only the other ranks' blocks."""
    mp.spawn(_worker_transposed_class, args=(world, _free_port(), str(tmp_path), chunks), nprocs=world, join=True)
    orders, ws, pool, ipool = problem()
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        ref = oracle.round_f32(ref, rp, col, w, np.arange(len(orders)))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(len(orders)))
    for r in range(world):
        own = np.load(tmp_path / f"cown{r}.npy")
        assert np.array_equal(np.load(tmp_path / f"cr{r}.npy").view(np.uint32), ref[own].view(np.uint32))
        assert np.array_equal(np.load(tmp_path / f"ci{r}.npy"), iref[own])
        if world == 1:
            assert int(np.load(tmp_path / f"clink{r}.npy")[0]) == 0


# ------------------------------------------------------------------------------------------
# the sharded bench's parity check (rowcheck): every owned output row against K1 on operands
# regenerated from their seeds, so a corrupted exchange fails it where spot_check passes

_RC_LAYOUT = [("w", (203,), "float32"), ("bn.running_var", (9,), "float32"),
              ("bn.num_batches_tracked", (), "int64"), ("b", (5,), "float32")]


def _patch_oracle_kernels(set_=setattr):
    """Test infrastructure for a host without a GPU: the oracle in place of the kernels (K1 for
    rowcheck / spot_check, the K3 round for the round classes); plans remember their CSR.
    set_: setattr in a spawned worker, monkeypatch.setattr in the test process."""
    from topology_aware_learning_amd import distributed as dd
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd import transposed as tr

    def agg_f32(xs, w, out, mode=0, **kw):
        out.copy_(torch.from_numpy(oracle.agg_f32([x.contiguous().numpy() for x in xs], w)))

    def agg_i64(xs, w, out, **kw):
        out.copy_(torch.from_numpy(oracle.agg_i64([x.contiguous().numpy() for x in xs], w)))

    orig = ops.default_plan

    def default_plan(rp, col, w, out, **kw):
        p = orig(rp, col, w, out, **kw)
        p._csr = (rp, col, w, out)
        return p

    def oracle_segments(layout_, seg_in, seg_out, plan, mode, n_of=None):
        rp, col, w, out = plan._csr
        for g, fn in (("f32", oracle.round_f32), ("i64", oracle.round_i64)):
            n = getattr(layout_, "n_" + g) if n_of is None else n_of.get(g, 0)
            if n:
                x = np.ascontiguousarray(seg_in[g][:, :n].numpy())
                res = fn(x, rp, col, w, out)
                seg_out[g][np.asarray(out), :n] = torch.from_numpy(np.ascontiguousarray(res[np.asarray(out)]))

    for mod, name, fn in ((ops, "agg_f32", agg_f32), (ops, "agg_i64", agg_i64), (ops, "default_plan", default_plan),
                          (dd, "run_round_segments", oracle_segments), (tr, "run_round_segments", oracle_segments)):
        set_(mod, name, fn)


def _worker_rowcheck(rank, world, port, out_dir, exchange, corrupt):
    import json

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch_oracle_kernels()
    from topology_aware_learning_amd import distributed as dd
    from topology_aware_learning_amd import ops, rowcheck
    from topology_aware_learning_amd import transposed as tr
    from topology_aware_learning_amd.arena import StateLayout

    orders, ws, _, _ = problem()
    layout = StateLayout.from_layout(_RC_LAYOUT)
    if exchange == "halo":
        def exch(sr):
            for r in dd.post_exchange(sr.spec, [t for _, t, _ in sr.pool_a.segments()], None, sr.packers):
                r.wait()
            if corrupt and rank == 0:  # one value of the first received halo row
                sr.pool_a.f32[len(sr.spec.own), 0] += 1.0
            return []

        sr = dd.ShardedRound(layout, orders, ws, rank, world, "cpu", exchange=exch)
        assert sr.spec.halo
    else:
        sr = tr.TransposedRound(layout, orders, ws, rank, world, "cpu", chunks=1)
        fwd = sr.forward_exchange

        def forward(k=0):
            for w in fwd(k):
                w.wait()
            if corrupt and rank == 0:  # one value of the first received column chunk
                sr.segs["f32"].work_in[k][sr.local_rows, 0] += 1.0
            return []

        sr.forward_exchange = forward
    rowcheck.fill_owned(sr.pool_a, _RC_LAYOUT, sr.own_ids, 500)
    sr.step()
    chk = rowcheck.check_round(sr.own_rows(), sr.own_ids, _RC_LAYOUT, orders, ws, 500, ops.MODE_EXACT)
    with open(os.path.join(out_dir, f"rc{rank}.json"), "w") as f:
        json.dump(dict(chk, spot=bool(sr.spot_check())), f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["halo", "transpose"])
@pytest.mark.parametrize("corrupt", [False, True])
def test_gloo_rowcheck_catches_a_corrupted_exchange(tmp_path, exchange, corrupt):
    """Two gloo ranks, one round of ShardedRound / TransposedRound, rowcheck on every owned
    row: clean exchange -> every row checked, none differs; one received halo value (or one
    all-to-all chunk value) changed -> rows differ, while spot_check - K1 on the operands as
    received, the bench's round-4 check - still passes on every rank."""
    import json

    mp.spawn(_worker_rowcheck, args=(2, _free_port(), str(tmp_path), exchange, corrupt), nprocs=2, join=True)
    res = [json.loads((tmp_path / f"rc{r}.json").read_text()) for r in range(2)]
    assert sum(r["rows_checked"] for r in res) == len(problem()[0])
    assert all(r["spot"] for r in res)
    assert all(r["reference"].startswith("K1") for r in res)
    differing = sum(r["rows_differing"] for r in res)
    assert (differing > 0) == corrupt, res


def test_rowcheck_batches_regenerated_operands(monkeypatch):
    """check_against_k1 in batches smaller than the round (a tight budget): same verdict."""
    _patch_oracle_kernels(monkeypatch.setattr)
    from topology_aware_learning_amd import ops, rowcheck
    from topology_aware_learning_amd.arena import ModelPool, StateLayout

    orders, ws, _, _ = problem()
    layout = StateLayout.from_layout(_RC_LAYOUT)
    n = len(orders)
    pin, pout = ModelPool(layout, n, "cpu"), ModelPool(layout, n, "cpu")
    rowcheck.fill_owned(pin, _RC_LAYOUT, range(n), 7)
    rp, col, w = ra.round_csr(orders, ws)
    pout.f32[:, :layout.n_f32] = torch.from_numpy(oracle.round_f32(pin.f32[:, :layout.n_f32].numpy().copy(), rp, col, w,
                                                                   np.arange(n)))
    pout.i64[:, :1] = torch.from_numpy(oracle.round_i64(pin.i64[:, :1].numpy().copy(), rp, col, w, np.arange(n)))
    for budget in (1, 6 * 4 * layout.ld_f32, 1 << 30):
        assert rowcheck.check_against_k1(pout, range(n), _RC_LAYOUT, orders, ws, 7, ops.MODE_EXACT,
                                         budget_bytes=budget) == []
    pout.f32[3, 100] += 1.0
    pout.i64[9, 0] += 1
    assert rowcheck.check_against_k1(pout, range(n), _RC_LAYOUT, orders, ws, 7, ops.MODE_EXACT, budget_bytes=1) == [3, 9]
