"""Drop-in path rate (not part of the product): BASELINE config 3 (64 devices, random 8-regular
graph, ResNet-50, unweighted) through the reference call surface, i.e. the round driver
src/decentralized_app.py with its clients' models bound to the device pool:

  per_call   the default: one unweighted_module_avg app call per client (64 per round) on
             the 2-thread app pool, each a K1 launch (the reference's form)
  batched    TAL_BATCHED_ROUND=1: the round's 64 aggregations as one RoundExecutor.run (K3)

each timed per round (synchronised before and after every round: latency) and over rounds run
back to back with one synchronisation at the end (throughput: *_back_to_back).

Training is replaced by an already resolved future holding the model as it stands (no app is
submitted) so a round is the driver's own Python plus the aggregation.  Also
times RoundExecutor(pool).run directly on the round (its default plan; double-buffered, the
default, and in place) against the bench's K1 floor (64 x one K1 call).  One JSON line per measurement.

usage: python tools/dropin_rate.py [rounds] [--profile[=per_call]] [--switch-us=N]   (--profile: cProfile of the
batched rounds only, or of the per-call rounds with =per_call; top functions by cumulative and by
own time)"""
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("TAL_SYNTHETIC_DATA", "1")
os.environ.setdefault("TAL_SYNTHETIC_SAMPLES", "64")

import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    sw = [a for a in sys.argv[1:] if a.startswith("--switch-us=")]
    if sw:  # A/B probe: the interpreter's thread switch interval (default 5000 us)
        sys.setswitchinterval(int(sw[0].split("=", 1)[1]) * 1e-6)
        print(json.dumps(dict(switch_interval_us=int(sw[0].split("=", 1)[1]))), flush=True)
    rounds = int(args[0]) if args else 5
    prof_arg = [a for a in sys.argv[1:] if a.startswith("--profile")]
    profile = bool(prof_arg)
    prof_mode = prof_arg[0].split("=", 1)[1] if prof_arg and "=" in prof_arg[0] else "batched"
    from src.decentralized_app import DecentrallearnApp
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.round import RoundExecutor

    import src.decentralized_app as da
    from concurrent.futures import Future

    def no_train(future, *args):
        """Training is outside the measured path: the model as it stands, as an already resolved
        future (no app is submitted - round 4 submitted a no-op app per client to a one-thread
        executor, and the batched round spent ~1.6 ms waiting for those to pass through it).
        Round 6: the driver's own lock-free resolved future (da._Resolved), so the stand-in's
        per-future condition variable (~2 us x 64) is not counted as driver time."""
        return da._Resolved(([], (future.result() if isinstance(future, Future) else future)[1]))

    da.local_train = da.no_local_train = no_train
    tmp = Path(tempfile.mkdtemp())
    topo = tmp / "random64.txt"
    np.savetxt(topo, nx.to_numpy_array(nx.random_regular_graph(8, 64, seed=0)), fmt="%d")
    t0 = time.perf_counter()
    app = DecentrallearnApp(dataset="cifar10_resnet50", topology_path=str(topo), epochs=1, rounds=10 ** 6,
                            aggregation_strategy="unweighted", log_dir=str(tmp / "logs"), batch_size=32)
    print(json.dumps(dict(setup_s=round(time.perf_counter() - t0, 1), clients=len(app.clients),
                          params=sum(v.numel() for v in app.clients[0].model.state_dict().values()))), flush=True)
    dev = app.pool.device
    app.round_states = {0: {i: {"agg": ([{}], app.clients[i])} for i in range(len(app.clients))}}
    r = 0
    if profile:
        import cProfile
        import io
        import pstats

        app.batched_round = prof_mode == "batched"
        for _ in range(2):  # warm: plan build, pools
            for f in app._federated_round(r):
                f.result()
            app.round_states.pop(r, None)
            r += 1
        torch.cuda.synchronize(dev)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(rounds):
            for f in app._federated_round(r):
                f.result()
            torch.cuda.synchronize(dev)
            app.round_states.pop(r, None)
            r += 1
        pr.disable()
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(45)
        pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(30)
        print(out.getvalue(), flush=True)
        return
    if "--per-call-breakdown" in sys.argv:  # app-thread time inside a per-call round, by part
        import threading

        import src.decentralized_client as dc

        spent = {"aggregate_models": [], "manual_seed": []}
        lock = threading.Lock()
        orig_agg, orig_seed = dc.aggregate_models, torch.manual_seed

        def timed(name, fn):
            def w(*a, **k):
                t = time.perf_counter()
                out = fn(*a, **k)
                with lock:
                    spent[name].append(time.perf_counter() - t)
                return out
            return w

        dc.aggregate_models = timed("aggregate_models", orig_agg)
        torch.manual_seed = timed("manual_seed", orig_seed)
        app.batched_round = False
        ts = []
        for k in range(rounds + 1):
            for v in spent.values():
                v.clear()
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for f in app._federated_round(r):
                f.result()
            torch.cuda.synchronize(dev)
            if k:
                ts.append(dict(round_ms=1e3 * (time.perf_counter() - t), calls=len(spent["aggregate_models"]),
                               **{f"{n}_ms_total": 1e3 * sum(v) for n, v in spent.items()},
                               **{f"{n}_us_median": 1e6 * float(np.median(v)) for n, v in spent.items() if v}))
            app.round_states.pop(r, None)
            r += 1
        dc.aggregate_models, torch.manual_seed = orig_agg, orig_seed
        for row in ts:
            print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in row.items()}), flush=True)
    for mode in ("per_call", "batched", "per_call", "batched"):
        app.batched_round = mode == "batched"
        ts = []
        for k in range(rounds + 1):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            futs = app._federated_round(r)
            for f in futs:
                f.result()
            torch.cuda.synchronize(dev)
            if k:  # the first round of each mode warms up (plan build, app pool threads)
                ts.append(time.perf_counter() - t)
            app.round_states.pop(r, None)
            r += 1
        ms = 1e3 * float(np.median(ts))
        print(json.dumps(dict(mode=mode, rounds=len(ts), ms_per_round_median=round(ms, 3),
                              ms_per_round_all=[round(1e3 * x, 3) for x in ts],
                              params_per_s=64 * 23_574_015 / (ms * 1e-3))), flush=True)
    # the same rounds back to back with ONE synchronisation at the end (a driver never waits for
    # the GPU between rounds: round r+1's Python runs while round r's kernels do; a round's
    # futures resolve at launch and the stream orders the next round's reads after its writes)
    for mode in ("per_call", "batched"):
        app.batched_round = mode == "batched"
        for f in app._federated_round(r):  # warm
            f.result()
        app.round_states.pop(r, None)
        r += 1
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(rounds):
            for f in app._federated_round(r):
                f.result()
            app.round_states.pop(r, None)
            r += 1
        torch.cuda.synchronize(dev)
        ms = 1e3 * (time.perf_counter() - t) / rounds
        print(json.dumps(dict(mode=mode + "_back_to_back", rounds=rounds, ms_per_round=round(ms, 3),
                              params_per_s=64 * 23_574_015 / (ms * 1e-3))), flush=True)
    # where a synchronised batched round's host time goes: round start -> batch collected ->
    # RoundExecutor.run entered -> launches issued -> round returned (wrappers around the
    # driver's own methods; the GPU is synchronised before each round)
    import src.decentralized_app as dam
    import topology_aware_learning_amd.round as rmod

    marks = {}
    orig_batched, orig_run = app._batched_aggregation, rmod.RoundExecutor.run

    def batched(batch, nxt):
        marks["collected"] = time.perf_counter()
        return orig_batched(batch, nxt)

    def run(self, *a, **k):
        marks["run_entered"] = time.perf_counter()
        out = orig_run(self, *a, **k)
        marks["launched"] = time.perf_counter()
        return out

    app._batched_aggregation = batched
    rmod.RoundExecutor.run = run
    app.batched_round = True
    phases = []
    for k in range(rounds + 1):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        futs = app._federated_round(r)
        t_ret = time.perf_counter()
        for f in futs:
            f.result()
        torch.cuda.synchronize(dev)
        t_end = time.perf_counter()
        if k:
            phases.append([marks["collected"] - t, marks["run_entered"] - marks["collected"],
                           marks["launched"] - marks["run_entered"], t_ret - marks["launched"], t_end - t_ret])
        app.round_states.pop(r, None)
        r += 1
    app._batched_aggregation, rmod.RoundExecutor.run = orig_batched, orig_run
    med = np.median(np.array(phases), axis=0) * 1e3
    print(json.dumps(dict(batched_phases_ms=dict(
        driver_loops=round(float(med[0]), 3), weights_and_rows=round(float(med[1]), 3),
        plan_and_launch=round(float(med[2]), 3), futures_resolved=round(float(med[3]), 3),
        gpu_tail=round(float(med[4]), 3)))), flush=True)
    del dam
    # the K1 floor: one aggregation call per client with nothing around it
    pool = app.pool
    orders = [sorted(c.neighbors) + [c.idx] for c in app.clients]
    ws = [[1 / len(o)] * len(o) for o in orders]
    out = torch.empty(pool.layout.n_f32, device=dev)
    out_i = torch.empty(pool.layout.n_i64, dtype=torch.int64, device=dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def k1(o, w):  # the per-call product kernel: both segments in one launch
        ops.agg_model_f32([pool.row_f32(j) for j in o], [pool.row_i64(j) for j in o], w, out, out_i)

    for _ in range(3):
        k1(orders[0], ws[0])
    s.record()
    for o, w in zip(orders, ws):
        k1(o, w)
    e.record()
    e.synchronize()
    k1 = s.elapsed_time(e)
    print(json.dumps(dict(k1_floor_ms_per_round=round(k1, 3), k1_ms_per_call=round(k1 / 64, 4))), flush=True)
    # RoundExecutor.run on the whole round (default plan): double-buffered (the default since
    # round 6: out of place into the executor's placed spare, then the storage exchange) and
    # in place on the pool (double_buffer=False, round 5's form), interleaved
    exs = dict(double_buffered=RoundExecutor(pool), in_place=RoundExecutor(pool, double_buffer=False))
    for ex in exs.values():
        ex.run(orders, ws)
    ts = {k: [] for k in exs}
    for _ in range(10):
        for k, ex in exs.items():
            s.record()
            ex.run(orders, ws)
            e.record()
            e.synchronize()
            ts[k].append(s.elapsed_time(e))
    p = exs["in_place"].plan(orders, ws, list(range(64)))
    for k, ex in exs.items():
        print(json.dumps(dict(round_executor_ms=round(float(np.median(ts[k])), 3), form=k,
                              all_ms=[round(t, 3) for t in ts[k]], plan=p.spec, kernel=ops.round_kernel_name(p),
                              spare_placement=ex.placement, swaps=ex.swaps)), flush=True)
    del exs
    # the same round out of place into a scratch pool: default plan vs the tuner's pick (bench)
    from topology_aware_learning_amd.arena import ModelPool
    from topology_aware_learning_amd.round import csr_from_lists

    scratch = ModelPool(pool.layout, 64, dev)
    rp, col, w = csr_from_lists(orders, ws)
    rows = np.arange(64, dtype=np.int32)
    tuned = ops.tune_plan(rp, col, w, rows, pool.f32, scratch.f32, n=pool.layout.n_f32)
    for name, plan in (("default", ops.default_plan(rp, col, w, rows).to(dev)), ("tuned", tuned)):
        ts = []
        for _ in range(12):
            s.record()
            ops.round_f32(pool.f32, scratch.f32, plan, n=pool.layout.n_f32)
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e))
        print(json.dumps(dict(out_of_place=name, ms=round(float(np.median(ts[2:])), 3), spec=plan.spec,
                              kernel=ops.round_kernel_name(plan))), flush=True)


if __name__ == "__main__":
    main()
