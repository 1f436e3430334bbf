"""The library's host reduction (tal_host_agg_*), which a process that sees no GPU runs
(BASELINE config 1: the reference's driver on CPU models, no GPU).  This container has no GPU,
so everything here goes through that path, unpatched, and is bit-compared with the reference's
own outputs: every aggregation app on fp32 and bf16 models (tests/golden/tiny_cases.*,
bf16_cases.*), the sequential in-place 4-ring round (round_4ring.*), and the whole config-1
driver run against the same run with the reference's CPU loop.  On a GPU box the package never
takes this path (tests/test_gpu_interface.py::test_host_reduction_unused_with_a_gpu)."""
import json

import networkx as nx
import numpy as np
import pytest
import torch
from torch.utils.data import Subset, TensorDataset

from topology_aware_learning_amd import ops

from _models import TinyNet
from conftest import GOLDEN

pytestmark = pytest.mark.skipif(torch.cuda.is_available(), reason="the host reduction runs only without a GPU")

TINY = json.loads((GOLDEN / "tiny_cases.json").read_text())
TINYZ = np.load(GOLDEN / "tiny_cases.npz")
CENT = {k: {int(i): v for i, v in d.items()} for k, d in TINY["centrality"].items()}
LAYOUT = [(n, tuple(s), d) for n, s, d in TINY["layout"]]
BF16 = json.loads((GOLDEN / "bf16_cases.json").read_text())
BF16Z = np.load(GOLDEN / "bf16_cases.npz")
BF16_CENT = {k: {int(i): v for i, v in d.items()} for k, d in BF16["centrality"].items()}
DUMMY = TensorDataset(torch.zeros(4, 1), torch.zeros(4, dtype=torch.long))


def _client(idx, model, n_train):
    from src.decentralized_client import DecentralClient

    data = TensorDataset(torch.zeros(n_train, 1), torch.zeros(n_train, dtype=torch.long))
    return DecentralClient(idx=idx, prox_coeff=0.0, model=model, train_data=Subset(data, list(range(n_train))),
                           test_data=None, valid_data=None, global_test_data=DUMMY,
                           global_backdoor_test_data=None, neighbors=[], neighbor_probs=[])


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype == np.float32:
        return np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
            a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))
    return np.array_equal(a, b)


def test_every_app_bit_exact_on_host():
    """Every app of the reference interface on CPU models, sim_centrality_module_avg included
    (its cosine similarities through the library's host K2, tal_host_cosine): bitwise the
    reference's outputs, special values and int64 truncation included."""
    import src.decentralized_client as dc

    done = 0
    for case in TINY["cases"]:
        ci = case["case"]
        clients = []
        for oi, idx in enumerate(case["order"]):
            m = TinyNet()
            m.load_state_dict({n: torch.from_numpy(TINYZ[f"c{ci}_in{oi}_{n}"].copy()) for n, _, _ in LAYOUT})
            clients.append((["r"], _client(idx, m, case["data_lens"][oi])))
        res = getattr(dc, case["fn"])(clients[-1], 0, *clients, centrality_metric=case["centrality_metric"],
                                      centrality_dict=CENT, softmax=case["softmax"],
                                      softmax_coeff=case["softmax_coeff"]).result()
        sd = res[1].model.state_dict()
        for name, _, _ in LAYOUT:
            assert _bits_equal(sd[name].detach().numpy(), TINYZ[f"c{ci}_out_{name}"]), (ci, case["fn"], name)
        done += 1
    assert done == len(TINY["cases"])
    assert sum(c["fn"] == "sim_centrality_module_avg" for c in TINY["cases"]) == 24


def test_cosine_similarity_tiny_cases_on_host():
    """The reference's cosine_similarity values of the tiny cases (self vs every operand), from
    the host K2, bit for bit."""
    import src.decentralized_client as dc

    checked = 0
    for case in TINY["cases"]:
        if "cosine" not in case:
            continue
        ci = case["case"]
        ms = []
        for oi in range(len(case["order"])):
            m = TinyNet()
            m.load_state_dict({n: torch.from_numpy(TINYZ[f"c{ci}_in{oi}_{n}"].copy()) for n, _, _ in LAYOUT})
            ms.append(m)
        for j, ref in enumerate(case["cosine"]):
            got = dc.cosine_similarity(ms[-1], ms[j])
            assert _bits_equal(np.float32(got.item()), np.float32(ref)), (ci, j, float(got), ref)
            checked += 1
    assert checked > 0


NEAR = json.loads((GOLDEN / "near_ties.json").read_text())
NEARZ = np.load(GOLDEN / "near_ties.npz")


def test_sim_centrality_near_ties_on_host():
    """sim_centrality_module_avg on the near-tie fixtures (fp32 ties, 1-4 ulp gaps, fp32-vs-exact
    order flips) with no GPU: the reference's similarities, least-similar pick and output bits."""
    import src.decentralized_client as dc

    cent = {k: {int(i): v for i, v in d.items()} for k, d in NEAR["centrality"].items()}
    kinds = set()
    for case in NEAR["cases"]:
        ci = case["case"]
        clients = []
        for oi, idx in enumerate(case["order"]):
            m = TinyNet()
            m.load_state_dict({n: torch.from_numpy(NEARZ[f"c{ci}_in{oi}_{n}"].copy()) for n, _, _ in NEAR["layout"]})
            clients.append((["r"], _client(idx, m, 10)))
        for j, ref in enumerate(case["cosine"]):
            got = dc.cosine_similarity(clients[-1][1].model, clients[j][1].model)
            assert _bits_equal(np.float32(got.item()), np.float32(ref)), (ci, j)
        res = dc.sim_centrality_module_avg(clients[-1], 0, *clients, centrality_metric=NEAR["centrality_metric"],
                                           centrality_dict=cent, softmax=NEAR["softmax"],
                                           softmax_coeff=NEAR["softmax_coeff"]).result()
        sd = res[1].model.state_dict()
        for name, _, _ in NEAR["layout"]:
            assert _bits_equal(sd[name].detach().numpy(), NEARZ[f"c{ci}_out_{name}"]), (ci, case["kind"], name)
        kinds.add(case["kind"])
    assert kinds == {"tie", "flip", "close"}


def test_every_app_bit_exact_bf16_models_on_host():
    """bf16 models (model.to(torch.bfloat16)) through every app: the reference's own bf16
    arithmetic (every product and partial sum rounded to bf16), bit for bit."""
    import src.decentralized_client as dc

    for case in BF16["cases"]:
        ci = case["case"]
        clients = []
        for oi, idx in enumerate(case["order"]):
            m = TinyNet().to(torch.bfloat16)
            sd = {}
            for name, _, dt in BF16["layout"]:
                a = BF16Z[f"c{ci}_in{oi}_{name}"]
                sd[name] = (torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16) if dt == "bfloat16"
                            else torch.from_numpy(a.copy()))
            m.load_state_dict(sd)
            clients.append((["r"], _client(idx, m, case["data_lens"][oi])))
        res = getattr(dc, case["fn"])(clients[-1], 0, *clients, centrality_metric=case["centrality_metric"],
                                      centrality_dict=BF16_CENT, softmax=case["softmax"],
                                      softmax_coeff=case["softmax_coeff"]).result()
        out = res[1].model.state_dict()
        for name, _, dt in BF16["layout"]:
            t = out[name].detach()
            got = t.view(torch.int16).numpy().view(np.uint16) if dt == "bfloat16" else t.numpy()
            assert np.array_equal(got, BF16Z[f"c{ci}_out_{name}"]), (ci, case["fn"], name)


def test_sequential_4ring_round_on_host():
    """The reference's sequential in-place 4-ring round (each client aggregates, in client order,
    neighbors an earlier call may already have overwritten) through the unweighted app."""
    import src.decentralized_client as dc

    meta = json.loads((GOLDEN / "round_4ring.json").read_text())
    z = np.load(GOLDEN / "round_4ring.npz")
    clients = []
    for i in range(4):
        m = TinyNet()
        m.load_state_dict({n: torch.from_numpy(z[f"in{i}_{n}"].copy()) for n, _, _ in meta["layout"]})
        clients.append((["r"], _client(i, m, 10)))
    for i, order in enumerate(meta["orders"]):
        assert order[-1] == i
        dc.unweighted_module_avg(clients[i], 0, *[clients[j] for j in order]).result()
    for i in range(4):
        sd = clients[i][1].model.state_dict()
        for n, _, _ in meta["layout"]:
            assert _bits_equal(sd[n].detach().numpy(), z[f"seq{i}_{n}"]), (i, n)


def test_host_agg_fma_and_aliasing():
    """FMA mode is one fused chain per element: against a float64 emulation (w * x is exact in
    float64; the float64 sum with acc is then rounded to float32 - the fma's single rounding
    unless that sum itself was inexact, which these inputs never hit); out may alias an
    operand."""
    rng = np.random.default_rng(3)
    n, m = 10007, 5
    xs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)) for _ in range(m)]
    w = [0.1, -0.25, 0.3, 1 / 3, 0.2]
    out = torch.empty(n)
    ops.host_agg(xs, w, out, mode=ops.MODE_FMA)
    wf = np.float32(w)
    acc = (np.float64(wf[0]) * xs[0].numpy().astype(np.float64)).astype(np.float32)
    for i in range(1, m):  # one fma = the exact w*x + acc (float64 holds it) rounded once
        acc = (np.float64(wf[i]) * xs[i].numpy().astype(np.float64) + acc.astype(np.float64)).astype(np.float32)
    assert np.array_equal(out.numpy().view(np.uint32), acc.view(np.uint32))
    # EXACT with out aliasing the last operand (the reference's self-last in-place call)
    ref = torch.empty(n)
    ops.host_agg(xs, w, ref)
    last = xs[-1].clone()
    ops.host_agg(xs[:-1] + [last], w, last)
    assert torch.equal(last.view(torch.int32), ref.view(torch.int32))
    with pytest.raises(ValueError):
        ops.host_agg(xs, w[:-1], out)


def test_config1_driver_unpatched(tmp_path, monkeypatch):
    """BASELINE config 1 as specified: src/experiments/decentralized_main.py, 8-device ring,
    CIFAR-10 CNN, two rounds on CPU with no GPU; the product's host reduction does every
    aggregation.  An observer wraps the product's aggregate_models (it calls straight through)
    to snapshot each call's operands and result, and every call is checked against the
    reference's own CPU loop on the snapshot (oracle/torch_path.py): operands in reference
    order (neighbors, then self), weights 1/3, every output bit."""
    import src.decentralized_client as dc
    from oracle import torch_path
    from topology_aware_learning_amd import aggregate

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_DEVICE_POOL", "0")
    assert dc.aggregate_models is aggregate.aggregate_models  # the product's own function
    real = aggregate.aggregate_models
    calls = []

    def observe(operands, weights, target, mode=ops.MODE_EXACT):
        before = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in operands]
        out = real(operands, weights, target, mode)
        calls.append((before, list(weights), [id(m) for m in operands], id(target),
                      {k: v.detach().clone() for k, v in target.state_dict().items()}))
        return out

    monkeypatch.setattr(dc, "aggregate_models", observe)
    # one worker thread for every app: the reference's 2-thread schedule lets a round's calls read
    # neighbors another call (or the next round's training) is writing, so a snapshot taken
    # beside the call would race with it; run serially, the snapshot is what the call reads
    from concurrent.futures import ThreadPoolExecutor

    from src import _parsl_compat as pc

    if not pc.HAVE_PARSL:
        serial = ThreadPoolExecutor(max_workers=1)
        for label in ("threadpool_executor", "decentral_train", "experiment"):
            monkeypatch.setitem(pc._executors, label, serial)
    topo = tmp_path / "ring8.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.cycle_graph(8)), fmt="%d")
    from src.experiments import decentralized_main

    rc = decentralized_main.main(["--dataset", "cifar10", "--aggregation_strategy", "unweighted", "--rounds", "2",
                                  "--epochs", "1", "--topology_file", str(topo), "--out_dir", str(tmp_path / "logs"),
                                  "--batch_size", "32"])
    assert rc == 0
    assert len(calls) == 16  # 8 clients x 2 rounds
    for before, w, ids, target, out in calls:
        assert len(ids) == 3 and ids[-1] == target and w == [1 / 3] * 3  # self last, in place
        ref = {k: v.clone() for k, v in before[-1].items()}
        torch_path.aggregate_call(before, w, ref)
        for k in ref:
            assert np.array_equal(ref[k].reshape(-1).numpy().view(np.uint8), out[k].reshape(-1).numpy().view(np.uint8)), k
    ckpts = sorted((tmp_path / "logs").rglob("*_ckpt.pth"))
    assert ckpts
    ck = torch.load(ckpts[-1], weights_only=False)
    assert len(ck["client_state_dicts"]) == 8


def test_config1_driver_degcent_sim_unpatched(tmp_path, monkeypatch):
    """decentralized_main.py --aggregation_strategy degCent_sim --softmax with no GPU (config 1's
    setting) on an 8-node barbell(3, 2) (unequal degrees, so the least-similar neighbor decides
    the softmax sign): every call's similarities equal the C oracle's cosine on the operands it
    read, its weights the reference rule's (oracle/reference_alg.py) on those similarities,
    and its output the reference's CPU loop with those weights, bit for bit."""
    import src.decentralized_client as dc
    import oracle
    from oracle import reference_alg as ra
    from oracle import torch_path
    from topology_aware_learning_amd import aggregate
    from topology_aware_learning_amd.arena import StateLayout

    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_DEVICE_POOL", "0")
    real_agg, real_rule = aggregate.aggregate_models, dc._w.sim_centrality
    calls, rules = [], []

    def observe(operands, weights, target, mode=ops.MODE_EXACT):
        before = [{k: v.detach().clone() for k, v in m.state_dict().items()} for m in operands]
        out = real_agg(operands, weights, target, mode)
        calls.append((before, list(weights), {k: v.detach().clone() for k, v in target.state_dict().items()}))
        return out

    def rule(order, me, cent, sims, softmax, coeff):
        rules.append((list(order), me, dict(cent), dict(sims), softmax, coeff))
        return real_rule(order, me, cent, sims, softmax, coeff)

    monkeypatch.setattr(dc, "aggregate_models", observe)
    monkeypatch.setattr(dc._w, "sim_centrality", rule)
    from concurrent.futures import ThreadPoolExecutor

    from src import _parsl_compat as pc

    if not pc.HAVE_PARSL:
        serial = ThreadPoolExecutor(max_workers=1)
        for label in ("threadpool_executor", "decentral_train", "experiment"):
            monkeypatch.setitem(pc._executors, label, serial)
    topo = tmp_path / "barbell.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.barbell_graph(3, 2)), fmt="%d")
    from src.experiments import decentralized_main

    rc = decentralized_main.main(["--dataset", "cifar10", "--aggregation_strategy", "degCent_sim", "--softmax",
                                  "--rounds", "2", "--epochs", "1", "--topology_file", str(topo),
                                  "--out_dir", str(tmp_path / "logs"), "--batch_size", "32"])
    assert rc == 0
    assert len(calls) == len(rules) == 16
    threads = torch.get_num_threads()
    signs = set()
    for (before, w, out), (order, me, cent, sims, softmax, coeff) in zip(calls, rules):
        assert order[-1] == me and len(before) == len(order)
        lay = StateLayout.from_state_dict(before[-1])
        segs = lay.param_segments(list(before[-1]))  # the CIFAR CNN: every entry a parameter
        flat = [np.concatenate([t.reshape(-1).numpy() for t in sd.values()]) for sd in before]
        for j, idx in enumerate(order[:-1]):
            ref = oracle.cosine_model(flat[-1], flat[j], segs, threads=min(threads, 1024))
            assert np.float32(sims[idx]).view(np.uint32) == ref.view(np.uint32), (me, idx)
        w_ref, c = ra.sim_centrality_weights(order, me, cent, sims, softmax, coeff)
        assert w == [float(x) for x in w_ref]
        signs.add(np.sign(c))
        ref_out = {k: v.clone() for k, v in before[-1].items()}
        torch_path.aggregate_call(before, w, ref_out)
        for k in ref_out:
            assert np.array_equal(ref_out[k].reshape(-1).numpy().view(np.uint8), out[k].reshape(-1).numpy().view(np.uint8)), k
    assert signs == {-1.0, 1.0}  # both softmax signs were taken
