"""The reference interface (src/decentralized_client.py apps, cosine_similarity, the round
driver) running on the HIP library, bit-compared with the reference's own outputs
(tests/golden/tiny_cases.*) for every app and every model placement."""
import json

import networkx as nx
import numpy as np
import pytest
import torch
from torch.utils.data import Subset, TensorDataset

from oracle import reference_alg as ra
from oracle import torch_path
from topology_aware_learning_amd.arena import ModelPool, StateLayout
from topology_aware_learning_amd.round import RoundExecutor

from _models import TinyNet
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

TINY = json.loads((GOLDEN / "tiny_cases.json").read_text())
TINYZ = np.load(GOLDEN / "tiny_cases.npz")
CENT = {k: {int(i): v for i, v in d.items()} for k, d in TINY["centrality"].items()}
LAYOUT = [(n, tuple(s), d) for n, s, d in TINY["layout"]]
DUMMY = TensorDataset(torch.zeros(4, 1), torch.zeros(4, dtype=torch.long))


def make_client(idx, model, n_train):
    from src.decentralized_client import DecentralClient

    data = TensorDataset(torch.zeros(n_train, 1), torch.zeros(n_train, dtype=torch.long))
    return DecentralClient(idx=idx, prox_coeff=0.0, model=model, train_data=Subset(data, list(range(n_train))),
                           test_data=None, valid_data=None, global_test_data=DUMMY,
                           global_backdoor_test_data=None, neighbors=[], neighbor_probs=[])


def bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype == np.float32:
        return np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
            a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))
    return np.array_equal(a, b)


def build_clients(case, placement, cuda):
    ci, M = case["case"], case["M"]
    layout = StateLayout.from_layout(LAYOUT)
    pool = ModelPool(layout, M, cuda) if placement == "pool" else None
    clients = []
    for oi, idx in enumerate(case["order"]):
        m = TinyNet()
        m.load_state_dict({n: torch.from_numpy(TINYZ[f"c{ci}_in{oi}_{n}"].copy()) for n, _, _ in LAYOUT})
        if placement == "gpu":
            m = m.to(cuda)
        elif placement == "pool":
            m = m.to(cuda)
            pool.bind(m, oi)
        clients.append((["r"], make_client(idx, m, case["data_lens"][oi])))
    return clients, pool


@pytest.mark.parametrize("placement", ["cpu", "gpu", "pool"])
def test_every_app_bit_exact(cuda, placement):
    import src.decentralized_client as dc

    for case in TINY["cases"]:
        clients, pool = build_clients(case, placement, cuda)
        fn = getattr(dc, case["fn"])
        res = fn(clients[-1], 0, *clients, centrality_metric=case["centrality_metric"], centrality_dict=CENT,
                 softmax=case["softmax"], softmax_coeff=case["softmax_coeff"]).result()
        assert res is clients[-1]
        sd = res[1].model.state_dict()
        if placement == "pool":
            assert pool.row_of(res[1].model) == case["M"] - 1  # written in place, still bound
        for name, _, _ in LAYOUT:
            assert bits_equal(sd[name].detach().cpu().numpy(), TINYZ[f"c{case['case']}_out_{name}"]), \
                (case["case"], case["fn"], name)


def test_cosine_similarity_matches_reference(cuda):
    """K2 through the reference interface returns the reference's fp32 similarity bit for bit."""
    import src.decentralized_client as dc

    for case in [c for c in TINY["cases"] if c["fn"] == "sim_centrality_module_avg"]:
        for placement in ("cpu", "pool"):
            clients, _ = build_clients(case, placement, cuda)
            for j, ref in enumerate(case["cosine"]):
                got = dc.cosine_similarity(clients[-1][1].model, clients[j][1].model)
                assert got.dtype == torch.float32
                assert np.float32(got.item()).view(np.uint32) == np.float32(ref).view(np.uint32), \
                    (case["case"], j, float(got), ref)


NEAR = json.loads((GOLDEN / "near_ties.json").read_text())
NEARZ = np.load(GOLDEN / "near_ties.npz")


@pytest.mark.parametrize("placement", ["cpu", "pool"])
def test_sim_centrality_near_ties_bit_exact(cuda, placement):
    """sim_centrality_module_avg where two neighbors' similarities tie in fp32, are 1-4 ulp
    apart, or are ordered differently in fp32 than in exact arithmetic (make_golden.py
    near_ties): the least-similar pick - and so the softmax sign and every output bit - is the
    reference's."""
    import src.decentralized_client as dc

    layout = StateLayout.from_layout([(n, tuple(s), d) for n, s, d in NEAR["layout"]])
    cent = {k: {int(i): v for i, v in d.items()} for k, d in NEAR["centrality"].items()}
    kinds = set()
    for case in NEAR["cases"]:
        ci = case["case"]
        pool = ModelPool(layout, len(case["order"]), cuda) if placement == "pool" else None
        clients = []
        for oi, idx in enumerate(case["order"]):
            m = TinyNet()
            m.load_state_dict({n: torch.from_numpy(NEARZ[f"c{ci}_in{oi}_{n}"].copy()) for n, _, _ in NEAR["layout"]})
            if pool is not None:
                m = m.to(cuda)
                pool.bind(m, oi)
            clients.append((["r"], make_client(idx, m, 10)))
        for j, ref in enumerate(case["cosine"]):
            got = dc.cosine_similarity(clients[-1][1].model, clients[j][1].model)
            assert np.float32(got.item()).view(np.uint32) == np.float32(ref).view(np.uint32), (ci, j)
        res = dc.sim_centrality_module_avg(clients[-1], 0, *clients, centrality_metric=NEAR["centrality_metric"],
                                           centrality_dict=cent, softmax=NEAR["softmax"],
                                           softmax_coeff=NEAR["softmax_coeff"]).result()
        sd = res[1].model.state_dict()
        for name, _, _ in NEAR["layout"]:
            assert bits_equal(sd[name].detach().cpu().numpy(), NEARZ[f"c{ci}_out_{name}"]), (ci, case["kind"], name)
        kinds.add(case["kind"])
    assert kinds == {"tie", "flip", "close"}


def test_round_executor_snapshot_and_sequential(cuda):
    """K3 over a pool == per-call oracle on the pre-round snapshot; sequential mode == the
    reference driven in client order (tests/golden/round_4ring)."""
    meta = json.loads((GOLDEN / "round_4ring.json").read_text())
    z = np.load(GOLDEN / "round_4ring.npz")
    layout = StateLayout.from_layout([(n, tuple(s), d) for n, s, d in meta["layout"]])
    orders = meta["orders"]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    pool = ModelPool(layout, 4, cuda)
    for i in range(4):
        pool.load_row(i, {n: torch.from_numpy(z[f"in{i}_{n}"]) for n, _, _ in meta["layout"]})
    before = [{k: v.cpu().clone() for k, v in pool.state_dict(i).items()} for i in range(4)]
    RoundExecutor(pool).run(orders, ws)
    for i in range(4):
        target = {k: v.clone() for k, v in before[i].items()}
        torch_path.aggregate_call([before[j] for j in orders[i]], ws[i], target)
        got = pool.state_dict(i)
        for k in target:
            assert bits_equal(got[k].cpu().numpy(), target[k].numpy()), (i, k)


def test_driver_config1_on_gpu(cuda, tmp_path, monkeypatch):
    """decentralized_main.py, 8-ring CIFAR CNN, one round, device-resident pool: every
    aggregation the driver issues goes through the HIP library and equals the reference loop
    applied to the same operands."""
    import src.decentralized_client as dc
    from topology_aware_learning_amd.aggregate import aggregate_models as real

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    checked = []

    def checked_aggregate(operands, weights, target, mode=0):
        sds = [{k: v.detach().cpu().clone() for k, v in m.state_dict().items()} for m in operands]
        ref = {k: v.clone() for k, v in sds[-1].items()}
        torch_path.aggregate_call(sds, weights, ref)
        out = real(operands, weights, target)
        assert getattr(target, "_tal_pool", None) is not None  # device-resident path
        for k, v in target.state_dict().items():
            assert bits_equal(v.detach().cpu().numpy(), ref[k].numpy()), k
        checked.append(len(operands))
        return out

    monkeypatch.setattr(dc, "aggregate_models", checked_aggregate)
    from src import _parsl_compat

    _parsl_compat.shutdown()
    _parsl_compat.configure({"threadpool_executor": 1})  # no in-place race between snapshot and kernel
    topo = tmp_path / "ring8.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.cycle_graph(8)), fmt="%d")
    from src.experiments import decentralized_main

    rc = decentralized_main.main(["--dataset", "cifar10", "--aggregation_strategy", "degCent", "--softmax",
                                  "--rounds", "2", "--epochs", "1", "--topology_file", str(topo), "--out_dir",
                                  str(tmp_path / "logs"), "--batch_size", "32"])
    _parsl_compat.configure({"threadpool_executor": 2})
    assert rc == 0 and checked == [3] * 16


def test_driver_batched_round(cuda, tmp_path, monkeypatch):
    """TAL_BATCHED_ROUND=1: decentralized_main.py issues each round's aggregations as ONE
    RoundExecutor.run (K3) with snapshot semantics; the pool after every round equals the
    oracle's snapshot round over the pool as it was after training, bit for bit."""
    import oracle

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_BATCHED_ROUND", "1")
    real_run = RoundExecutor.run
    runs = []

    def checked_run(self, orders, weights, out_rows=None, sequential=False, plan=None):
        lay = self.pool.layout
        f_in = self.pool.f32[:, : lay.n_f32].cpu().numpy().copy()
        i_in = self.pool.i64[:, : lay.n_i64].cpu().numpy().copy()
        real_run(self, orders, weights, out_rows, sequential, plan)
        rp, col, w = ra.round_csr(orders, weights)
        ref = oracle.round_f32(f_in, rp, col, w, np.asarray(out_rows))
        iref = oracle.round_i64(i_in, rp, col, w, np.asarray(out_rows))
        assert np.array_equal(self.pool.f32[:, : lay.n_f32].cpu().numpy().view(np.uint32), ref.view(np.uint32))
        assert np.array_equal(self.pool.i64[:, : lay.n_i64].cpu().numpy(), iref)
        runs.append(len(orders))

    monkeypatch.setattr(RoundExecutor, "run", checked_run)
    import src.decentralized_app as da

    apps = []
    real_batched = da.DecentrallearnApp._batched_aggregation

    def spy(self, batch, nxt):
        apps.append(self)
        return real_batched(self, batch, nxt)

    monkeypatch.setattr(da.DecentrallearnApp, "_batched_aggregation", spy)
    topo = tmp_path / "ring8.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.cycle_graph(8)), fmt="%d")
    from src.experiments import decentralized_main

    rc = decentralized_main.main(["--dataset", "cifar10", "--aggregation_strategy", "degCent", "--softmax",
                                  "--rounds", "3", "--epochs", "1", "--topology_file", str(topo), "--out_dir",
                                  str(tmp_path / "logs"), "--batch_size", "32"])
    assert rc == 0 and runs == [8, 8, 8]
    # rounds 2 and 3 drew the same neighbor sets (a %d topology: every link probability 1), so
    # they reused round 1's operand rows and weights (DecentrallearnApp._round_key), still
    # bitwise the oracle's snapshot round (checked_run above)
    assert apps[-1].round_cache_hits == 2


@pytest.mark.parametrize("strategy,participation", [("weighted", 0.5), ("unweighted", 0.75), ("test_agg", 1.0)])
def test_driver_batched_round_partial(cuda, tmp_path, monkeypatch, strategy, participation):
    """TAL_BATCHED_ROUND=1 with part of the clients selected (the others keep their trained
    model, decentralized_app.py:599-604), data-size weights, and test_agg (no aggregation): each
    round's launch covers exactly the selected clients with surviving neighbors, and the pool
    after it equals the oracle's snapshot round over those rows, the other rows untouched."""
    import oracle

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_BATCHED_ROUND", "1")
    real_run = RoundExecutor.run
    runs = []

    def checked_run(self, orders, weights, out_rows=None, sequential=False, plan=None):
        lay = self.pool.layout
        f_in = self.pool.f32[:, : lay.n_f32].cpu().numpy().copy()
        i_in = self.pool.i64[:, : lay.n_i64].cpu().numpy().copy()
        real_run(self, orders, weights, out_rows, sequential, plan)
        rp, col, w = ra.round_csr(orders, weights)
        ref = f_in.copy()
        iref = i_in.copy()
        oracle.round_f32(f_in, rp, col, w, np.asarray(out_rows), pool_out=ref)
        oracle.round_i64(i_in, rp, col, w, np.asarray(out_rows), pool_out=iref)
        assert np.array_equal(self.pool.f32[:, : lay.n_f32].cpu().numpy().view(np.uint32), ref.view(np.uint32))
        assert np.array_equal(self.pool.i64[:, : lay.n_i64].cpu().numpy(), iref)
        runs.append(sorted(out_rows))

    monkeypatch.setattr(RoundExecutor, "run", checked_run)
    topo = tmp_path / "rr12.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.random_regular_graph(3, 12, seed=1)), fmt="%d")
    from src.experiments import decentralized_main

    rc = decentralized_main.main(["--dataset", "cifar10", "--aggregation_strategy", strategy, "--rounds", "2",
                                  "--epochs", "1", "--topology_file", str(topo), "--out_dir", str(tmp_path / "logs"),
                                  "--batch_size", "32", "--participation", str(participation)])
    assert rc == 0
    if strategy == "test_agg":
        assert runs == []  # nothing to aggregate: no launch
    else:
        assert len(runs) == 2 and all(len(r) == int(12 * participation) for r in runs)


def test_checkpoint_from_device_pool(cuda, tmp_path):
    """SURVEY §8(f) row 2 on the GPU: the checkpoint is written from the pool rows and reads
    back (reference loader and pool loader) bit-identically."""
    import test_checkpoint as tc
    from src import utils as U
    from src.aggregation_scheduler import BaseScheduler

    cl, pool = tc._bound([1, 0, 2], seed=3, device=cuda)
    U.save_checkpoint(2, cl, [], tmp_path / "g.pth")
    ref = [{k: v.cpu() for k, v in c.model.state_dict().items()} for c in cl]
    got = torch.load(tmp_path / "g.pth", weights_only=False)["client_state_dicts"]
    for a, b in zip(got, ref):
        tc._check_same(a, b)
    cl2, pool2 = tc._bound([0, 1, 2], seed=8, device=cuda)
    U.load_checkpoint(tmp_path / "g.pth", cl2, BaseScheduler(1.0))
    for a, c2 in zip(ref, cl2):
        tc._check_same(a, c2.model.state_dict())


@pytest.mark.parametrize("k", [1, 3, 70])
def test_prox_term_matches_torch_loop(cuda, k):
    """fused proximal term over pool rows vs the reference's loop
    (tasks.py:277-286): value and gradients (client and neighbor parameters)."""
    import test_checkpoint as tc
    from topology_aware_learning_amd.prox import prox_term

    cl, pool = tc._bound(list(range(k + 1)), seed=k, device=cuda)
    with torch.no_grad():
        for c in cl:
            for p in c.model.parameters():
                p.add_(torch.randn_like(p) * 0.1)
        ref_params = dict(cl[0].model.named_parameters())
        for n, p in cl[1].model.named_parameters():  # an identical pair: norm 0, zero gradient
            p.copy_(ref_params[n])
    client, nbs = cl[0].model, [c.model for c in cl[1:]]
    fused = prox_term(client, nbs)
    assert fused is not None
    fused.backward()
    g_fused = [p.grad.clone() for c in cl for p in c.model.parameters()]
    for c in cl:
        c.model.zero_grad()
    ref = 0.0
    for m in nbs:
        for w, wt in zip(client.parameters(), m.parameters()):
            ref = ref + (w - wt).norm(2)
    ref.backward()
    g_ref = [p.grad.clone() for c in cl for p in c.model.parameters()]
    fused_v, ref_v = float(fused.detach()), float(ref.detach())
    assert abs(fused_v - ref_v) <= 1e-5 * abs(ref_v) + 1e-6
    for a, b in zip(g_fused, g_ref):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-6)


def test_round_executor_scratch_placement(cuda):
    """A multi-group round through RoundExecutor with scratch placement trials: the fastest of
    three scratch candidates is kept and the round is still bitwise the oracle's."""
    import networkx as nx

    import oracle

    g = nx.random_regular_graph(8, 1000, seed=4)  # 1000 sources: more than one LDS group
    orders = [sorted(g.neighbors(i)) + [i] for i in range(1000)]
    ws = [ra.unweighted_weights(9)] * 1000
    layout = StateLayout.from_layout([("w", (4093,), "float32"), ("nbt", (), "int64")])
    pool = ModelPool(layout, 1000, cuda)
    x = np.random.default_rng(9).standard_normal((1000, 4093)).astype(np.float32)
    pool.f32[:, :4093] = torch.from_numpy(x).to(cuda)
    ex = RoundExecutor(pool, placement_trials=3)
    ex.run(orders, ws)
    assert ex.placement is not None and len(ex.placement["scratch_ms"]) == 3
    rp, col, w = ra.round_csr(orders, ws)
    ref = oracle.round_f32(x, rp, col, w, np.arange(1000))
    assert bits_equal(pool.f32[:, :4093].cpu().numpy(), ref)


def test_host_reduction_unused_with_a_gpu(cuda, monkeypatch):
    """With a GPU visible the package never runs the host reduction (tal_host_agg_*, the
    no-GPU path of BASELINE config 1): CPU-resident models go through the HIP kernels."""
    import src.decentralized_client as dc
    from topology_aware_learning_amd import ops

    def refuse(*a, **k):
        raise AssertionError("host reduction called with a GPU visible")

    monkeypatch.setattr(ops, "host_agg", refuse)
    monkeypatch.setattr(ops, "host_cosine", refuse)
    for fn in ("unweighted_module_avg", "sim_centrality_module_avg"):
        case = next(c for c in TINY["cases"] if c["fn"] == fn)
        clients, _ = build_clients(case, "cpu", cuda)
        res = getattr(dc, fn)(clients[-1], 0, *clients, centrality_metric=case["centrality_metric"],
                              centrality_dict=CENT, softmax=case["softmax"],
                              softmax_coeff=case["softmax_coeff"]).result()
        sd = res[1].model.state_dict()
        for name, _, _ in LAYOUT:
            assert sd[name].device.type == "cpu"
            assert bits_equal(sd[name].detach().numpy(), TINYZ[f"c{case['case']}_out_{name}"]), (fn, name)
