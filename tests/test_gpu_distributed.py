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
from topology_aware_learning_amd import ops
from topology_aware_learning_amd.distributed import ShardedRound, partition_contiguous, recv_range

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


def _virtual_halo_exchange(srs):
    """The halo exchange between virtual ranks through the same per-peer messages the RCCL path
    sends (HaloPacker.send_tensor -> the receiver's contiguous halo block, recv_range)."""
    for sr in srs:
        for peer in sr.spec.recv:
            r0, r1 = recv_range(sr.spec, peer)
            src = srs[peer]
            for si, (_, t, _) in enumerate(sr.pool_a.segments()):
                ts = src.pool_a.segments()[si][1]
                msg = src.packers[si].send_tensor(ts, sr.spec.rank)
                assert msg.shape[0] == r1 - r0
                t[r0:r1].copy_(msg)


def _graph(name):
    import bench

    return {"regular": lambda: nx.random_regular_graph(8, 48, seed=0), "barbell": lambda: nx.barbell_graph(20, 8),
            "ring": lambda: nx.cycle_graph(12),
            # BASELINE config 4 / 5 topologies at their own size (reduced columns)
            "barbell60": lambda: bench.make_graph("barbell", 128, 0),
            "sbm256": lambda: bench.make_graph("sbm", 256, 0)}[name]()


@pytest.mark.parametrize("dtype,mode", [("f32", ops.MODE_EXACT), ("bf16", ops.MODE_EXACT), ("bf16", ops.MODE_FMA)])
@pytest.mark.parametrize("graph,world", [("regular", 4), ("barbell", 8), ("ring", 2), ("barbell60", 8), ("sbm256", 8)])
def test_virtual_ranks_two_rounds(cuda, graph, world, dtype, mode):
    """ShardedRound on `world` virtual ranks (halo exchange by in-process copies of the packed
    per-peer messages), two rounds, bitwise the oracle's snapshot rounds.  barbell60 / sbm256 are
    BASELINE configs 4 / 5 sharded 8 ways (16 / 32 devices per rank)."""
    if dtype == "f32" and mode == ops.MODE_FMA:
        pytest.skip("fp32 FMA rounds are checked against K1-FMA elsewhere")
    g = _graph(graph)
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    layout, pool, ipool = _seg_setup(dtype, n, 1)
    owner = partition_contiguous(n, world)
    srs = [ShardedRound(layout, orders, ws, r, world, cuda, mode=mode, exchange=lambda sr: []) for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.spec.own):
            _put_row(sr.pool_a, k, dtype, pool[gid], ipool[gid], cuda)
    if graph in ("barbell60", "sbm256"):  # one message per peer per segment, each way
        assert all(len(sr.spec.send) <= world - 1 and len(sr.spec.recv) <= world - 1 for sr in srs)
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        _virtual_halo_exchange(srs)
        for sr in srs:
            sr.step()
        if dtype == "f32":
            ref = oracle.round_f32(ref, rp, col, w, np.arange(n))
        else:
            ref = oracle.round_bf16(ref, rp, col, w, np.arange(n), exact=(mode == ops.MODE_EXACT))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    for sr in srs:
        assert sr.spot_check()
        got = _get_rows(sr.own_rows(), len(sr.spec.own), dtype)
        assert np.array_equal(got, ref[sr.spec.own].view(got.dtype))
        assert np.array_equal(sr.own_rows().i64[: len(sr.spec.own), :1].cpu().numpy(), iref[sr.spec.own])


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("dtype,mode", [("f32", ops.MODE_EXACT), ("bf16", ops.MODE_EXACT), ("bf16", ops.MODE_FMA)])
@pytest.mark.parametrize("graph,world", [("regular", 4), ("barbell", 8), ("ring", 3), ("barbell60", 8), ("sbm256", 8)])
def test_virtual_ranks_transposed_two_rounds(cuda, graph, world, dtype, mode, chunks):
    """TransposedRound (column blocks by all-to-all) with the two all-to-alls done by in-process
    copies between virtual ranks: K3 on each rank's column block, bitwise the oracle round."""
    from topology_aware_learning_amd.transposed import TransposedRound

    g = nx.cycle_graph(13) if graph == "ring" else _graph(graph)
    n = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    layout, pool, ipool = _seg_setup(dtype, n, 2)
    # interleaved owners for the small graphs; BASELINE configs 4 / 5 in contiguous blocks (bench)
    owner = (partition_contiguous(n, world) if graph in ("barbell60", "sbm256")
             else np.array([(5 * i) % world for i in range(n)], np.int32))
    srs = [TransposedRound(layout, orders, ws, r, world, cuda, owner=owner, chunks=chunks, mode=mode)
           for r in range(world)]
    for sr in srs:
        for k, gid in enumerate(sr.own):
            _put_row(sr.pool_a, k, dtype, pool[gid], ipool[gid], cuda)
    rp, col, w = ra.round_csr(orders, ws)
    ref, iref = pool, ipool
    for _ in range(2):
        for k in range(srs[0].chunks):
            for sr in srs:
                sr.pack(k)  # the own block straight into the head rows of work_in
            for r, sr in enumerate(srs):  # forward all-to-all: chunk k of block r of every other model
                for key, s in sr._segs_at(k):
                    for p in sr.peers():
                        s.work_in[k][sr.rows_of(p)].copy_(srs[p].segs[key].send[k][srs[p].peer_slot(r)])
            for sr in srs:
                sr.compute(k)
            for r, sr in enumerate(srs):  # backward all-to-all: my rows of every other rank's chunk
                for key, s in sr._segs_at(k):
                    for p in sr.peers():
                        s.back[k][sr.peer_slot(p)].copy_(srs[p].segs[key].work_out[k][srs[p].rows_of(r)])
            for sr in srs:
                sr.unpack(k)  # the own block straight from the head rows of work_out
        if dtype == "f32":
            ref = oracle.round_f32(ref, rp, col, w, np.arange(n))
        else:
            ref = oracle.round_bf16(ref, rp, col, w, np.arange(n), exact=(mode == ops.MODE_EXACT))
        iref = oracle.round_i64(iref, rp, col, w, np.arange(n))
    torch.cuda.synchronize()
    for sr in srs:
        assert sr.spot_check()
        got = _get_rows(sr.own_rows(), sr.local_rows, dtype)
        assert np.array_equal(got, ref[sr.own].view(got.dtype))
        assert np.array_equal(sr.own_rows().i64[: sr.local_rows, :1].cpu().numpy(), iref[sr.own])


@pytest.mark.parametrize("exchange,world,tune", [("halo", 2, False), ("transpose", 2, False), ("transpose", 3, False),
                                                ("halo", 3, False), ("halo", 2, True), ("transpose", 2, True)])
def test_bench_multi_rank_rehearsal(cuda, tmp_path, exchange, world, tune):
    """bench.py's N > 1 branch end to end (make_round, exchange, spot check, timing, JSON) with
    `world` ranks sharing this GPU over gloo (exchange staged through host memory): the same
    code the 8-GPU RCCL run executes, except the transport; tune=True is the driver's default
    command (every rank tunes its plans on its own buffers)."""
    import json
    import os
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    port = 29500 + (os.getpid() % 400) + world * 7 + (0 if exchange == "halo" else 3) + (50 if tune else 0)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), "--gpus", str(world),
           "--dist-backend", "gloo", "--exchange", exchange, "--model", "cifar10", "--devices-per-gpu", "16",
           "--degree", "4", "--steps", "2", "--warmup", "1"] + ([] if tune else ["--no-tune"])
    out = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == world and d["parity"] is True and d["exchange"] == exchange
    assert d["value"] > 0 and d["link_bytes_in_per_round"] > 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("graph,model,dtype,exchange", [("barbell", "resnet50", "f32", "auto"),
                                                        ("sbm", "vit_b16", "bf16", "auto"),
                                                        ("sbm", "vit_b16", "bf16", "transpose"),
                                                        ("random", "resnet50", "f32", "auto")])
def test_bench_world8_rehearsal(cuda, tmp_path, graph, model, dtype, exchange):
    """bench.py --gpus 8 on BASELINE config 4 (barbell(60, 8), ResNet-50 layout), config 5
    (SBM 8 x 32, ViT-B/16 layout, bf16) and the weak-scaling default (random 8-regular graph over
    64 x 8 devices, ResNet-50 layout, plans tuned per rank: the driver's SCALE command) with 8
    gloo ranks sharing this GPU: the exchange staged through host memory and the layouts cut to
    their first 131,072 float params (--max-params)."""
    import json
    import os
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    port = 29900 + (os.getpid() % 300) + {"barbell": 0, "sbm": 11, "random": 23}[graph] + (0 if exchange == "auto" else 5)
    devices = {"sbm": ["--devices", "256"], "barbell": ["--devices", "128"], "random": []}[graph]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), "--gpus", "8",
           "--dist-backend", "gloo", "--graph", graph, "--model", model, "--dtype", dtype, *devices,
           "--exchange", exchange, "--max-params", "131072", "--steps", "2", "--warmup", "1"] + \
        ([] if graph == "random" else ["--no-tune"])
    out = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 8 and d["parity"] is True
    assert d["config"]["devices"] == {"sbm": 256, "barbell": 128, "random": 512}[graph]
    pr = d["parity_rows"]  # every owned output row of every rank, vs K1 on regenerated operands
    assert pr["rows_checked"] == pr["devices"] == d["config"]["devices"] and pr["rows_differing"] == 0
    assert pr["reference"].startswith("K1")  # --max-params: no reference fixture for the cut layout
    assert d["value"] > 0 and d["link_bytes_in_per_round"] > 0
    # the link probe ran before the round was built and fed the bound model and the choice
    assert d["link_probe_GBps"] > 0 and d["link_probe"]["bytes_per_pair"] == 8 << 20
    if exchange != "auto":
        assert d["exchange"] == exchange


@pytest.mark.parametrize("exchange,tune,model,transport", [
    ("halo", False, "cifar10", "device"), ("transpose", False, "cifar10", "device"),
    ("transpose", True, "cifar10", "device"), ("halo", False, "resnet50", "device"),
    ("transpose", False, "resnet50", "device"), ("halo", False, "cifar10", "cabi"),
    ("transpose", False, "cifar10", "cabi")])
def test_bench_sharded_one_rank_rccl(cuda, tmp_path, exchange, tune, model, transport):
    """bench.py's sharded branch on a one-rank RCCL (backend "nccl") process group: the
    exchange's collectives (batched P2P group / all_to_all_single on device tensors, the
    spot-check all-reduce, barriers) on the real transport with nothing to move — the RCCL
    calls of the 8-GPU run, on one GPU (RCCL refuses two ranks on one device)."""
    import json
    import os
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    port = 28700 + (os.getpid() % 400) + (0 if exchange == "halo" else 3) + (20 if tune else 0) + (40 if model == "resnet50" else 0) + (60 if transport == "cabi" else 0)
    # cifar10: a 16-device 4-regular graph (rowcheck: K1 on regenerated operands); resnet50: BASELINE
    # config 3 itself (rowcheck: the reference's sha256 of all 64 output models)
    shape = ["--devices-per-gpu", "16", "--degree", "4"] if model == "cifar10" else []
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), "--gpus", "1",
           "--sharded", "--dist-backend", "nccl", "--exchange", exchange, "--model", model, *shape,
           "--transport", transport, "--steps", "2", "--warmup", "1"] + ([] if tune else ["--no-tune"])
    out = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, out.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 1 and d["parity"] is True and d["exchange"] == exchange
    assert d["config"]["parallelism"] == f"{exchange}-sharded x1" and d["transport"] == transport
    pr = d["parity_rows"]
    assert pr["rows_checked"] == d["config"]["devices"] and pr["rows_differing"] == 0
    assert pr["reference"].startswith("K1" if model == "cifar10" else "reference sha256")


def _rc_round(cuda, exchange, corrupt):
    """One round of 4 virtual ranks on a 48-device 8-regular graph with seeded models
    (rowcheck.fill_owned), the exchange done by in-process copies; with corrupt=True one value of
    rank 0's first received halo row (halo) or first received column-chunk row (transpose) is
    changed after it arrives.  Returns (rows checked, rows differing, every spot_check passed)."""
    from topology_aware_learning_amd import rowcheck
    from topology_aware_learning_amd.transposed import TransposedRound

    lay = [("w", (1001,), "float32"), ("bn.running_var", (7,), "float32"), ("bn.num_batches_tracked", (), "int64"),
           ("b", (13,), "float32")]
    layout = StateLayout.from_layout(lay)
    world = 4
    g = nx.random_regular_graph(8, 48, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(48)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    if exchange == "halo":
        srs = [ShardedRound(layout, orders, ws, r, world, cuda, exchange=lambda sr: []) for r in range(world)]
    else:
        srs = [TransposedRound(layout, orders, ws, r, world, cuda, chunks=1) for r in range(world)]
    for sr in srs:
        rowcheck.fill_owned(sr.pool_a, lay, sr.own_ids, 300)
    if exchange == "halo":
        _virtual_halo_exchange(srs)
        if corrupt:
            srs[0].pool_a.f32[len(srs[0].spec.own), 0] += 1.0
        for sr in srs:
            sr.step()
    else:
        for sr in srs:
            sr.pack(0)
        for r, sr in enumerate(srs):
            for key, s in sr._segs_at(0):
                for p in sr.peers():
                    s.work_in[0][sr.rows_of(p)].copy_(srs[p].segs[key].send[0][srs[p].peer_slot(r)])
        if corrupt:
            srs[0].segs["f32"].work_in[0][srs[0].local_rows, 0] += 1.0
        for sr in srs:
            sr.compute(0)
        for r, sr in enumerate(srs):
            for key, s in sr._segs_at(0):
                for p in sr.peers():
                    s.back[0][sr.peer_slot(p)].copy_(srs[p].segs[key].work_out[0][srs[p].rows_of(r)])
        for sr in srs:
            sr.unpack(0)
    torch.cuda.synchronize()
    res = [rowcheck.check_round(sr.own_rows(), sr.own_ids, lay, orders, ws, 300, ops.MODE_EXACT) for sr in srs]
    return (sum(r["rows_checked"] for r in res), sum(r["rows_differing"] for r in res),
            all(sr.spot_check() for sr in srs))


@pytest.mark.parametrize("exchange", ["halo", "transpose"])
@pytest.mark.parametrize("corrupt", [False, True])
def test_rowcheck_catches_a_corrupted_exchange(cuda, exchange, corrupt):
    """The sharded bench's parity check on the GPU (K3 rounds, K1 on operands regenerated from
    their seeds): a clean exchange passes with all 48 rows checked; one corrupted received halo
    value or all-to-all chunk value fails it, while spot_check (K1 on the operands as received)
    passes on every rank either way."""
    checked, differing, spots = _rc_round(cuda, exchange, corrupt)
    assert checked == 48 and spots
    assert (differing > 0) == corrupt
