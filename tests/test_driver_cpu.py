"""BASELINE config 1 plumbing: 8-device ring, CIFAR-10 CNN, one round through
src/experiments/decentralized_main.py on the CPU.

There is no GPU here, so every aggregation runs the product's host reduction (the library's
tal_host_agg_*, aggregate.py's no-GPU dispatch); nothing in the driver is patched.  Every call's
operands and output bits are checked against the reference's CPU loop in
tests/test_host_backend.py::test_config1_driver_unpatched (which observes the calls) and the
sequential 4-ring fixture; the same run goes through the HIP library in
tests/test_gpu_interface.py."""
import numpy as np
import networkx as nx
import pytest
import torch


def _run_main(args):
    from src.experiments import decentralized_main

    return decentralized_main.main(args)


def test_config1_one_round(tmp_path, monkeypatch):
    """The driver as shipped: nothing patched (the environment only selects the synthetic
    CIFAR-10 stand-in, there is no dataset download); the aggregations are the product's."""
    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "64")
    monkeypatch.setenv("TAL_DEVICE_POOL", "0")
    topo = tmp_path / "ring8.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.cycle_graph(8)), fmt="%d")
    rc = _run_main(["--dataset", "cifar10", "--aggregation_strategy", "unweighted", "--rounds", "1",
                    "--epochs", "1", "--topology_file", str(topo), "--out_dir", str(tmp_path / "logs"),
                    "--batch_size", "32"])
    assert rc == 0
    ckpts = list((tmp_path / "logs").rglob("0_ckpt.pth"))
    assert len(ckpts) == 1
    ck = torch.load(ckpts[0], weights_only=False)  # written by this test's own run
    assert ck["round_idx"] == 0 and len(ck["client_state_dicts"]) == 8
    biases = [sd["network.0.bias"] for sd in ck["client_state_dicts"]]
    assert all(torch.isfinite(b).all() for b in biases)
    assert len({tuple(b.tolist()) for b in biases}) == 8  # every client aggregated its own ring window


def test_strategy_dispatch_and_unweighted_fl_topology(tmp_path, monkeypatch):
    monkeypatch.setenv("TAL_SYNTHETIC_DATA", "1")
    monkeypatch.setenv("TAL_SYNTHETIC_SAMPLES", "32")
    monkeypatch.setenv("TAL_DEVICE_POOL", "0")
    topo = tmp_path / "ring4.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.cycle_graph(4)), fmt="%d")
    from src.decentralized_app import DecentrallearnApp, STRATEGIES
    from src.decentralized_client import centrality_module_avg, unweighted_module_avg

    assert STRATEGIES["degCent"] == (centrality_module_avg, "degree")
    app = DecentrallearnApp(dataset="cifar10", topology_path=str(topo), rounds=1, epochs=1, batch_size=32,
                            aggregation_strategy="unweighted_fl", log_dir=str(tmp_path / "l"), train=False)
    assert app.aggregation_function is unweighted_module_avg
    assert np.array_equal(app.topology, np.ones((4, 4)) - np.eye(4))
    before = [{k: v.clone() for k, v in c.model.state_dict().items()} for c in app.clients]
    assert app.run() == 0
    after = [c.model.state_dict() for c in app.clients]
    assert all(not torch.equal(a["network.0.bias"], b["network.0.bias"]) for a, b in zip(after, before))


def test_parsl_standin_dependencies():
    """The in-process Parsl stand-in: an app waits for every distinct future among its args and
    kwargs (the same future passed ten times counts once), runs once, and a failed dependency's
    exception becomes the app's (reference apps take AppFutures, decentralized_app.py:605-641)."""
    import threading
    from concurrent.futures import Future

    from src import _parsl_compat as pc

    if pc.HAVE_PARSL:
        pytest.skip("real Parsl installed")
    runs = []

    @pc.python_app(executors=["threadpool_executor"])
    def app(a, *rest, k=None):
        runs.append(threading.get_ident())
        return a + sum(rest) + (k or 0)

    f = Future()
    g = Future()
    out = app(f, f, f, 1, k=g)  # same future three times + a kwarg future
    assert not out.done()
    f.set_result(10)
    assert not out.done()
    g.set_result(5)
    assert out.result(timeout=10) == 10 * 3 + 1 + 5
    assert len(runs) == 1
    done = Future()
    done.set_result(2)
    assert app(done, done).result(timeout=10) == 4  # dependencies already resolved
    bad = Future()
    chained = app(bad, f)
    bad.set_exception(ValueError("upstream"))
    with pytest.raises(ValueError, match="upstream"):
        chained.result(timeout=10)
    assert app(app(done, 1), 1).result(timeout=10) == 4  # app futures chain
