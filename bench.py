#!/usr/bin/env python3
"""Benchmark: device-resident aggregated params/s at K=8 neighbors (BASELINE.json metric).

Workload (N=1, BASELINE config 3): 64 simulated devices on nx.random_regular_graph(8, 64,
seed=0), ResNet-50 state_dicts (reference layout: 23,573,962 fp32 + 53 int64 elements), every
device aggregating its 8 neighbors + itself (M = 9, self last, unweighted 1/M) — one step =
one whole aggregation round (64 aggregation calls) executed by the K3 round kernel over the
device-resident pool, inputs already in HBM, snapshot semantics, exact reference numerics.

With --gpus N > 1 (launched by torch.distributed.run, one rank per GPU) the graph has 64*N
devices (weak scaling: 64 per GPU, contiguous blocks).  The exchange moves the fewer link
bytes: neighbor models owned by other GPUs by RCCL send/recv over xGMI, overlapped with the
interior rows (halo), or every model's column blocks by two RCCL all-to-alls around the local
round (transpose; random expanders at 4+ GPUs) — topology_aware_learning_amd/transposed.py.

Prints ONE JSON line (rank 0).  See DESIGN.md for the byte accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="resnet50", choices=["resnet18", "resnet50", "vit_b16", "cifar10"])
    p.add_argument("--devices-per-gpu", type=int, default=64)
    p.add_argument("--degree", type=int, default=8)
    p.add_argument("--graph", default="random", choices=["random", "ring", "barbell", "sbm"],
                   help="random: nx.random_regular_graph(degree, devices, 0) (configs 3 / weak scaling); "
                        "ring: cycle (config 2); barbell: nx.barbell_graph(60, 8) (config 4); "
                        "sbm: 8 blocks of 32, p_in=14/31, p_out=2/224 (config 5)")
    p.add_argument("--devices", type=int, default=0, help="total devices (overrides devices-per-gpu x N)")
    p.add_argument("--mode", default=None, choices=["exact", "fma"],
                   help="default: exact for f32 (bitwise the reference), fma for bf16 (fp32 accumulation)")
    p.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                   help="model storage: f32 (the reference) or bf16 (BASELINE config 5's bf16 tolerance run)")
    p.add_argument("--c4", type=int, default=0)
    p.add_argument("--no-tune", action="store_true", help="use the model-based plan choice instead of timing candidates")
    p.add_argument("--plan", default="", help="JSON plan spec (a previous run's plan.spec): build it, no tuning")
    p.add_argument("--stream-rows", type=int, default=0,
                   help="force a streamed plan with groups of at most this many rows (profiling)")
    p.add_argument("--in-place", action="store_true",
                   help="N = 1, single-group plans: every round in place on one pool (RoundExecutor(double_buffer=False); the executor's default double-buffers like the timed loop)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bound of the CPU baseline sample (one call at a time; the two-concurrent-calls "
                        "configuration runs half as long)")
    p.add_argument("--max-params", type=int, default=0,
                   help="rehearsal only: keep the model layout's leading float entries up to this many "
                        "elements (int64 buffers kept); the config names the reduced layout")
    p.add_argument("--no-k1", action="store_true", help="skip the per-call K1 side measurement")
    p.add_argument("--host-path", action="store_true", help="also time the H2D+K1+D2H per-call path")
    p.add_argument("--placement-trials", type=int, default=16,
                   help="N = 1: candidate pools for the placement calibration (arena.select_pool_pair); "
                        "2 = none (the first two allocations)")
    p.add_argument("--sharded", action="store_true",
                   help="run the sharded (N > 1) path at N = 1 as well: a one-rank process group, the "
                        "exchange's collectives on RCCL with nothing to move (a check of that code path "
                        "on one GPU, never the benchmark)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="N > 1: nccl (RCCL over xGMI, the benchmark); gloo = rehearsal of the same "
                        "code path with the exchange staged through host memory, ranks may share a GPU")
    p.add_argument("--weights", default="unweighted", choices=["unweighted", "degcent"],
                   help="unweighted_module_avg (1/M, the metric's config) or centrality_module_avg "
                        "with softmax(10 x degree centrality): per-operand weights")
    p.add_argument("--transport", "--halo-transport", dest="halo_transport", default="device",
                   choices=["device", "cabi"],
                   help="N > 1 over nccl, either exchange: torch.distributed's RCCL (device) or the "
                        "library's own communicator (cabi, include/tal_agg.h: tal_comm_* / "
                        "tal_halo_pack / tal_halo_exchange; the all-to-alls as groups of per-peer "
                        "sends / receives; experimental: not yet run across GPUs)")
    p.add_argument("--exchange", default="auto", choices=["auto", "halo", "transpose"],
                   help="N > 1: neighbor models by RCCL P2P (halo) or column blocks by all-to-all "
                        "(transpose); auto = the smaller predicted time at the probed link rate "
                        "(transposed.choose_exchange)")
    p.add_argument("--link-probe-mb", type=int, default=1024,
                   help="N > 1: bytes each rank sends to (and receives from) every other rank in the "
                        "link probe before the round is built (gloo rehearsals: at most 8 MiB)")
    return p.parse_args()


def make_graph(kind: str, n_devices: int, degree: int, seed: int = 0):
    """BASELINE configs' topologies (SURVEY §8(d) synthetic inputs)."""
    import networkx as nx

    if kind == "random":
        return nx.random_regular_graph(degree, n_devices, seed=seed)
    if kind == "ring":
        return nx.cycle_graph(n_devices)
    if kind == "barbell":
        return nx.barbell_graph(60, 8)
    sizes = [32] * max(1, n_devices // 32)
    p = [[14 / 31 if a == b else 2 / 224 for b in range(len(sizes))] for a in range(len(sizes))]
    return nx.stochastic_block_model(sizes, p, seed=seed)


def round_spec(n_devices: int, degree: int, seed: int = 0, kind: str = "random", weights: str = "unweighted"):
    """(orders, weights) of one round: neighbors ascending then self;
    unweighted_module_avg's 1/M (client.py:431) or centrality_module_avg's softmax of 10 x the
    degree centrality (client.py:572-593, SURVEY §8(d)'s softmax-centrality variant)."""
    import networkx as nx

    from topology_aware_learning_amd import weights as tw

    g = make_graph(kind, n_devices, degree, seed)
    n_devices = g.number_of_nodes()
    orders = [sorted(g.neighbors(i)) + [i] for i in range(n_devices)]
    if weights == "degcent":
        cent = nx.degree_centrality(g)
        return orders, [tw.centrality(o, cent, True, 10.0) for o in orders]
    return orders, [tw.unweighted(len(o)) for o in orders]


SEED_BASE = 9300  # device i's model = synth.synth_state_dict(layout, SEED_BASE + i) (config 3's fixture seeds)


def reference_fixture(args, orders, weights):
    """(seed base, reference) for rowcheck.check_round: the reference's own per-model sha256
    when this workload is one tests/golden's full-round fixtures cover (BASELINE configs 3, 4
    and 5, made by the reference's apps on exactly these seeded inputs; config 5 per entry
    group), else (SEED_BASE, None) - K1 on regenerated operands.  The fixture's operand order
    must be this run's (a mismatch is a bug, not a skipped check)."""
    from topology_aware_learning_amd import synth

    if args.max_params or args.mode != "exact":
        return SEED_BASE, None
    key = (args.graph, len(orders), args.model, args.dtype, args.weights)
    name = {("random", 64, "resnet50", "f32", "unweighted"): "full_round_c3_resnet50_rr64.json",
            ("barbell", 128, "resnet50", "f32", "unweighted"): "full_round_c4_resnet50_barbell.json"}.get(key)
    if key[:3] == ("sbm", 256, "vit_b16"):
        name = "full_round_c5_vit_sbm256.json"
    if name is None or (args.graph == "random" and args.degree != 8):
        return SEED_BASE, None
    path = ROOT / "tests" / "golden" / name
    fx = json.loads(path.read_text())
    base = int(fx["seeds"][0])
    if fx["seeds"] != list(range(base, base + len(orders))):
        raise AssertionError(f"{name}: seeds are not seed_base + device id")
    if "rows" in fx:  # configs 3 / 4: one digest per segment per model
        if [r["order"] for r in fx["rows"]] != [list(o) for o in orders]:
            raise AssertionError(f"{name}: operand order differs from this run's graph")
        expected = {"f32": {i: [r["sha256_f32"]] for i, r in enumerate(fx["rows"])},
                    "i64": {i: [r["sha256_i64"]] for i, r in enumerate(fx["rows"])}}
        nf, ni = synth.layout_counts(synth.get_layout(args.model))
        return base, dict(name=name, expected=expected, ranges={"f32": [(0, nf)], "i64": [(0, ni)]})
    fn = "unweighted_module_avg" if args.weights == "unweighted" else "centrality_module_avg"
    run = next((r for r in fx["runs"] if r["dtype"] == args.dtype and r["fn"] == fn), None)
    if run is None:
        return SEED_BASE, None
    if fx["orders"] != [list(o) for o in orders]:
        raise AssertionError(f"{name}: operand order differs from this run's graph")
    seg = "f32" if args.dtype == "f32" else "b16"
    groups = run["groups"]
    expected = {seg: {i: [run["sha256"][i][str(g)] for g in groups] for i in range(len(orders))}}
    ranges = {seg: [(fx["groups"][g]["start"], fx["groups"][g]["end"]) for g in groups]}
    return base, dict(name=name + f" {args.dtype} {fn}", expected=expected, ranges=ranges)


def fill_pool(pool, seed: int):
    import torch

    g = torch.Generator(device=pool.device)
    g.manual_seed(seed)
    pool.f32.normal_(generator=g)
    pool.b16.normal_(generator=g)
    pool.i64.random_(0, 1_000_000, generator=g)


def cpu_baseline(layout_list, m: int, budget_s: float):
    """The reference loop (clone/mul/add_/load_state_dict, oracle/torch_path.py) on host cores,
    one call at a time, with torch.set_num_threads(all cores this process may run on) - SURVEY
    §8(d)(i), the reported value - and with torch's default thread count (16 on the GPU box,
    its OMP_NUM_THREADS); then the reference's effective configuration, two concurrent calls
    (Parsl ThreadPoolExecutor(max_threads=2), parsl_setup.py:75-78) at the default count.
    About budget_s seconds in all."""
    import threading

    import torch

    from oracle import torch_path

    gen = torch.Generator().manual_seed(100)
    sds, targets = [], []
    for k in range(m + 2):  # the values do not matter for the timing: seeded normal / counters
        sd = {}
        for name, shape, dt in layout_list:
            if dt == "int64":
                sd[name] = torch.randint(0, 1_000_000, tuple(shape), generator=gen)
            else:
                sd[name] = torch.randn(tuple(shape), generator=gen).to(getattr(torch, dt))
        (sds if k < m else targets).append(sd)
    w = [1 / m] * m
    n_out = sum(t.numel() for t in targets[0].values())
    default_threads = torch.get_num_threads()
    all_threads = usable_cpus()

    def one_at_a_time(threads: int, secs: float):
        """(calls, seconds, median seconds per call): the GPU box's host is shared, so a call's
        time varies with other tenants; the median per call is the reported rate."""
        torch.set_num_threads(threads)
        torch_path.aggregate_call(sds, w, targets[0])  # warm-up
        calls, t0, per = 0, time.perf_counter(), []
        while True:
            t = time.perf_counter()
            torch_path.aggregate_call(sds, w, targets[0])
            per.append(time.perf_counter() - t)
            calls += 1
            el = time.perf_counter() - t0
            if el >= secs or calls >= 1024:
                return calls, el, float(np.median(per))

    calls_all, el_all, med_all = one_at_a_time(all_threads, 0.4 * budget_s)
    calls_def, el_def, med_def = one_at_a_time(default_threads, 0.35 * budget_s)
    counts = [0, 0]
    stop = time.perf_counter() + 0.25 * budget_s

    def worker(k):
        while time.perf_counter() < stop:
            torch_path.aggregate_call(sds, w, targets[k])
            counts[k] += 1

    t1 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el2 = time.perf_counter() - t1
    torch.set_num_threads(default_threads)
    return dict(value=n_out / med_all, unit="params/s", cores=all_threads, kind="port",
                sample=f"{calls_all} reference calls (M={m}, {n_out} params) one at a time in {el_all:.2f} s "
                       f"with torch.set_num_threads({all_threads}) (every core this process may run on: "
                       "its affinity within the cgroup CPU quota), value from the median call; "
                       "torch CPU clone/mul/add_/copy_ on host state_dicts",
                ms_per_call=1e3 * med_all, window_value=calls_all * n_out / el_all,
                default_threads_value=n_out / med_def, default_threads=default_threads,
                default_threads_ms_per_call=1e3 * med_def,
                os_cpu_count=os.cpu_count(), affinity_cpus=all_threads, cpu_model=cpu_model(),
                # the reference's effective configuration: Parsl ThreadPoolExecutor(max_threads=2)
                two_concurrent_calls_value=sum(counts) * n_out / el2, two_concurrent_calls=sum(counts),
                two_concurrent_seconds=round(el2, 2))


def usable_cpus() -> int:
    """Cores this process may actually use: its CPU affinity, capped by a cgroup CPU quota
    (cgroup v2 cpu.max or v1 cfs quota / period) - on a shared box os.cpu_count() shows the whole
    machine, and that many threads on a 16-core quota would stall every parallel op."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        n = os.cpu_count() or 1
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            if parse is not None:
                q, per = parse(open(path).read())
                if q != "max":
                    n = min(n, max(1, int(int(q) / int(per))))
            else:
                q = int(open(path).read())
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                if q > 0:
                    n = min(n, max(1, q // per))
            break
        except (OSError, ValueError):
            continue
    return n


def log(msg: str) -> None:
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f"bench: {msg}", file=sys.stderr, flush=True)


def cpu_model() -> str:
    """The host CPU's model name (lscpu's "Model name", read from /proc/cpuinfo)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from topology_aware_learning_amd import ops, rowcheck, synth
    from topology_aware_learning_amd.arena import ModelPool, StateLayout, select_pool_pair

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dist_backend == "gloo":
        local %= torch.cuda.device_count()  # rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sharded = world > 1 or args.sharded
    if sharded:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    lay = synth.get_layout(args.model)
    if args.max_params:
        lay = synth.truncate_layout(lay, args.max_params)
    if args.dtype == "bf16":
        lay = synth.as_bf16(lay)
    layout = StateLayout.from_layout(lay)
    n_params = layout.n_f32 + layout.n_b16 + layout.n_i64
    if args.mode is None:
        args.mode = "exact" if args.dtype == "f32" else "fma"
    mode = ops.MODE_EXACT if args.mode == "exact" else ops.MODE_FMA
    bf16 = args.dtype == "bf16"
    n_float = layout.n_b16 if bf16 else layout.n_f32  # the streamed segment
    esize = 2 if bf16 else 4
    n_dev_total = args.devices or args.devices_per_gpu * world
    orders, weights = round_spec(n_dev_total, args.degree, kind=args.graph, weights=args.weights)
    n_dev_total = len(orders)
    M = max(len(o) for o in orders)
    # every device's model is synth's seeded model of its global id, so any rank can check any
    # output row without trusting what the exchange delivered (rowcheck)
    seed_base, reference = reference_fixture(args, orders, weights)

    if not sharded:
        from topology_aware_learning_amd import ops as _ops

        rows = n_dev_total
        row_ptr, col, w = _round_csr(orders, weights)
        out_rows = np.arange(rows, dtype=np.int32)
        seg = (lambda p: p.b16) if bf16 else (lambda p: p.f32)
        row = (lambda p, r: p.row_b16(r)) if bf16 else (lambda p, r: p.row_f32(r))
        round_fn = _ops.round_bf16 if bf16 else _ops.round_f32
        agg_fn = _ops.agg_bf16 if bf16 else _ops.agg_f32
        # pool placement (arena.select_pool_pair): as many candidate pools as fit in 70 % of the
        # free HBM, up to --placement-trials; the plan is tuned on the first pair, then a round
        # into each candidate is timed with it and the two fastest destinations are kept
        pool_bytes = rows * (4 * layout.ld_f32 + 2 * layout.ld_b16 + 8 * layout.ld_i64)
        trials = max(2, min(args.placement_trials, int(0.7 * torch.cuda.mem_get_info(dev)[0] // pool_bytes)))
        log(f"{rows} rows x {n_float} elements, {trials} candidate pools")
        cand = [ModelPool(layout, rows, dev) for _ in range(trials)]
        fill_pool(cand[0], 1234)
        tune = not (args.plan or args.stream_rows or args.no_tune or args.c4)
        if args.plan:
            plan = _ops.plan_from_spec(row_ptr, col, w, out_rows, json.loads(args.plan)).to(dev)
        elif args.stream_rows:
            plan = _ops.build_stream_plan(row_ptr, col, w, out_rows, args.stream_rows).to(dev)
        else:  # the model-based choice; with tuning, only for the placement calibration below
            plan = (_ops.build_plan(row_ptr, col, w, out_rows, c4=args.c4) if args.c4 else
                    _ops.default_plan(row_ptr, col, w, out_rows, bf16=bf16, mode=mode)).to(dev)
        ev_s, ev_e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def placement_score(a, b):
            round_fn(seg(a), seg(b), plan, n=n_float, mode=mode)
            ev_s.record()
            for _ in range(2):
                round_fn(seg(a), seg(b), plan, n=n_float, mode=mode)
            ev_e.record()
            ev_e.synchronize()
            return ev_s.elapsed_time(ev_e) / 2

        in_place = args.in_place and plan.single_group
        if in_place:  # one pool, rounds in place: keep the fastest placement, a second pool for the check
            ms = [placement_score(c, c) for c in cand]
            best = int(np.argmin(ms))
            pin, pout = cand[best], cand[(best + 1) % len(cand)]
            placement = dict(pools=len(cand), in_place_ms=[round(v, 3) for v in ms], chosen=[best])
        elif trials > 2:
            it = iter(cand)
            pin, pout, placement = select_pool_pair(lambda: next(it), placement_score, trials)
        else:  # no room for more candidates (config 5 fp32: 88.6 GB pools): the pair as allocated
            (pin, pout) = cand
            ab, ba = min(placement_score(pin, pout), placement_score(pin, pout)), min(placement_score(pout, pin), placement_score(pout, pin))
            placement = dict(pools=2, dest_ms=[round(ba, 3), round(ab, 3)], chosen=[0, 1],
                             pair_ms={"0->1": round(ab, 3), "1->0": round(ba, 3)},
                             first_pair_ms=round((ab + ba) / 2, 3), chosen_pair_ms=round((ab + ba) / 2, 3),
                             note="two pools fit in 70 % of the free HBM: no other candidate to time")
        del cand
        torch.cuda.empty_cache()  # the candidates not kept
        rowcheck.fill_owned(pin, lay, range(rows), seed_base)
        log(f"placement {placement}")
        if tune:  # time every plan candidate on the pools the steps use (once per topology)
            plan = _ops.tune_plan(row_ptr, col, w, out_rows, seg(pin), seg(pout), n=n_float, mode=mode)
            in_place = in_place and plan.single_group

        def step(a, b):
            round_fn(seg(a), seg(b), plan, n=n_float, mode=mode)
            _ops.round_i64(a.i64, b.i64, plan, n=layout.n_i64)

        # correctness check at full size: EVERY output row of the round (both segments) == K1
        # on the same operands, bitwise (K1 itself is pinned to the reference's sha256 of
        # ResNet-50 M = 9 calls; tests/test_gpu_fullsize.py pins whole rounds)
        log(f"plan {plan.spec}; checking every row against K1")
        step(pin, pout)
        chk = torch.empty(n_float, dtype=seg(pin).dtype, device=dev)
        chk_i = torch.empty(layout.n_i64, dtype=torch.int64, device=dev)
        iv = torch.int16 if bf16 else torch.int32
        bad_rows = []
        for r in range(rows):
            agg_fn([row(pin, j) for j in orders[r]], weights[r], chk, mode=mode)
            same = torch.equal(chk.view(iv), row(pout, r).view(iv))
            if layout.n_i64:
                _ops.agg_i64([pin.row_i64(j) for j in orders[r]], weights[r], chk_i)
                same = same and torch.equal(chk_i, pout.row_i64(r))
            if not same:
                bad_rows.append(r)
        parity_ok = not bad_rows
        del chk, chk_i
        ref_check = None
        if reference is not None:  # the round's outputs against the reference's own digests
            ref_check = rowcheck.check_round(pout, range(rows), lay, orders, weights, seed_base, mode,
                                             reference=reference)
            parity_ok = parity_ok and ref_check["rows_differing"] == 0
        tol = bf16_tolerance(pin, pout, orders[0], weights[0], n_float, dev) if bf16 else None

        log(f"parity {parity_ok} ({len(bad_rows)} rows differ); timing {args.steps} steps")
        pools = [pin, pin] if in_place else [pin, pout]
        for i in range(args.warmup):
            step(pools[i % 2], pools[(i + 1) % 2])
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            a, b = pools[i % 2], pools[(i + 1) % 2]
            ev[i][0].record(stream)
            round_fn(seg(a), seg(b), plan, n=n_float, mode=mode)
            ev[i][1].record(stream)
            _ops.round_i64(a.i64, b.i64, plan, n=layout.n_i64)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        k_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
        staged = plan.staged_rows()
        bytes_round = esize * n_float * (staged + rows)  # compulsory: each staged source read once, each output written once
        per_call_bytes = esize * n_float * (len(col) + rows)  # SURVEY §8(d) B summed over the round's calls
        result_extra = dict(
            kernel=_ops.round_kernel_name(plan), plan=dict(groups=plan.info.n_groups, staged_sources=staged,
                                                  c4=plan.info.c4, dense_rb=plan.info.dense_rb,
                                                  lds_reads_per_column=plan.info.dense_reads,
                                                  tuned_ms=plan.tuned_ms, candidates=plan.candidates,
                                                  spec=plan.spec),
            per_call_equivalent_GBps=per_call_bytes / (k_ms * 1e-3) / 1e9,
            parity_k3_vs_k1=dict(rows_checked=rows, rows_differing=len(bad_rows), first_bad=bad_rows[:8]),
            parity_vs_reference=ref_check,
            valu=valu_floor(len(col), rows, n_float, k_ms, mode, bf16=bool(layout.n_b16)))
        if tol is not None:
            result_extra["bf16_vs_fp32_reference_row0"] = tol
        result_extra["placement"] = placement
        result_extra["in_place"] = in_place
        steps_done = args.steps
        units = rows * n_params * steps_done
        k1 = None
        if not args.no_k1 and not bf16:
            k1 = bench_k1(layout, pin, orders, weights, mode, dev)
        hostp = bench_host_path(lay, M, dev) if args.host_path else None
    else:
        from topology_aware_learning_amd.transposed import make_round

        # per-rank progress on stderr: a first multi-GPU run that stalls names its phase
        rlog = (lambda msg: log(f"rank {rank}/{world}: {msg}"))
        rlog(f"{n_dev_total} devices, {layout.n_f32 + layout.n_b16} float params per model; probing the links")
        probe = link_probe(dist, rank, world, dev, args.dist_backend, args.link_probe_mb)
        rlog(f"link probe {probe['GBps']} GB/s per pair (min over ranks); building the round")
        sr = make_round(layout, orders, weights, rank, world, dev, exchange=args.exchange, mode=mode,
                        tune=not args.no_tune,
                        transport="host" if args.dist_backend == "gloo" else args.halo_transport,
                        link_gbps=probe["GBps"] if world > 1 else None)
        rlog(f"{sr.exchange_kind} exchange over {sr.transport}, {len(sr.own_ids)} own devices; first round")
        rowcheck.fill_owned(sr.pool_a, lay, sr.own_ids, seed_base)
        sr.step()
        torch.cuda.synchronize(dev)
        rlog("first round done; checking every owned row")
        # every output row this rank owns, against the reference's digests or K1 on operands
        # regenerated from their seeds - never on what the exchange delivered (rowcheck)
        chk = rowcheck.check_round(sr.own_rows(), sr.own_ids, lay, orders, weights, seed_base, mode,
                                   reference=reference)
        cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # collectives' scalars
        cnt = torch.tensor([chk["rows_checked"], chk["rows_differing"]], dtype=torch.int64, device=cdev)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        bad_all = [None] * world
        dist.all_gather_object(bad_all, chk["first_bad"])
        rows_checked, rows_differing = int(cnt[0].item()), int(cnt[1].item())
        parity_dist = rows_differing == 0 and rows_checked == n_dev_total
        parity_rows = dict(rows_checked=rows_checked, rows_differing=rows_differing,
                           first_bad=sorted(j for b in bad_all for j in b)[:8], reference=chk["reference"],
                           devices=n_dev_total)
        rlog(f"rows checked {rows_checked}, differing {rows_differing}; {args.warmup} warm-up + {args.steps} timed rounds")
        for _ in range(args.warmup):
            sr.step()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            sr.step(timed=True)
        torch.cuda.synchronize(dev)
        dist.barrier()
        el_local = time.perf_counter() - t0
        t = torch.tensor([el_local], device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        torch.cuda.synchronize(dev)
        k_ms = float(np.mean(sr.kernel_ms()))
        bytes_round = sr.kernel_bytes
        # DESIGN §6's model next to the measurement: per exchange kind the busiest rank's HBM
        # bytes and the busiest GPU pair's link bytes over their peaks; the binding term
        from topology_aware_learning_amd.distributed import partition_contiguous
        from topology_aware_learning_amd.transposed import XGMI_LINK_GBPS, link_model

        model = link_model(orders, partition_contiguous(n_dev_total, world), world, layout.n_f32,
                           layout.n_i64, layout.n_b16, link_gbps=probe["GBps"] if world > 1 else XGMI_LINK_GBPS)
        ms_step = 1e3 * el / args.steps
        chosen = model[sr.exchange_kind]
        result_extra = dict(kernel=",".join(sorted({ops.round_kernel_name(p) for p in sr.plans.values()})),
                            link_probe_GBps=probe["GBps"], link_probe=probe,
                            parity_rows=parity_rows, exchange=sr.exchange_kind, transport=sr.transport, link_bytes_in_per_round=sr.link_bytes,
                            link_GBps_in=sr.link_bytes / (el / args.steps) / 1e9,
                            bound_model=dict(per_exchange={k: {kk: (round(vv, 3) if isinstance(vv, float) else vv)
                                                                for kk, vv in v.items()} for k, v in model.items()},
                                             chosen=sr.exchange_kind, predicted_ms=round(chosen["predicted_ms"], 3),
                                             binds=chosen["binds"], measured_ms_per_step=round(ms_step, 3),
                                             measured_over_predicted=round(ms_step / chosen["predicted_ms"], 3),
                                             kernel_share_of_step=round(k_ms / ms_step, 3)))
        units = n_dev_total * n_params * args.steps
        parity_ok = parity_dist
        k1 = None
        hostp = None

    if rank != 0:
        if sharded:
            dist.barrier()
            dist.destroy_process_group()
        return

    achieved = bytes_round / (k_ms * 1e-3) / 1e9
    traffic = None
    if not sharded:  # PMC bytes of exactly this kernel + plan spec + workload, when profiled
        traffic = load_traffic(traffic_key(result_extra["kernel"], result_extra["plan"]["spec"],
                                           workload_key(args.graph, n_dev_total, args.model, args.dtype, args.weights)))
    cpu = None
    if not args.no_cpu_baseline and not sharded:
        log("CPU baseline")
        cpu = cpu_baseline(lay, M, args.cpu_seconds)  # bf16 layouts: the reference's loop on bf16 tensors
    value = units / el
    out = {
        "metric": "device-resident aggregated params/s at K=8 neighbors",
        "value": value,
        "unit": "params/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("bf16" if bf16 else "f32") + ("" if args.mode == "exact" else "-fma"),
        "data": f"synthetic (random {'bf16' if bf16 else 'fp32'} / int64 state_dicts of the reference layout in HBM)",
        "config": {"workload": f"{n_dev_total}-device {args.graph} graph"
                               + (f" ({args.degree}-regular, seed 0)" if args.graph == "random" else "")
                               + f", {args.model} state_dicts, max M={M} (self last), "
                               + ("unweighted, " if args.weights == "unweighted" else "degree-centrality softmax weights, ")
                               + "one full aggregation round per step, snapshot semantics",
                   "model_layout": args.model + (f" (first {args.max_params} float params: rehearsal)"
                                                 if args.max_params else ""), "devices": n_dev_total, "devices_per_gpu": args.devices_per_gpu,
                   "params_per_model": n_params, "parallelism": f"{result_extra.get('exchange', '')}-sharded x{world}" if sharded else "1 GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                     "bytes_per_launch": bytes_round, "kernel_ms": k_ms,
                     # the same plan on the first two pools allocated, before the placement
                     # calibration kept the fastest pair (arena.select_pool_pair)
                     "first_pair_frac": (bytes_round / (result_extra["placement"]["first_pair_ms"] * 1e-3) / 1e9
                                         / HBM_PEAK_GBPS) if not sharded and "first_pair_ms" in result_extra.get(
                                             "placement", {}) else None},
        "cpu_baseline": cpu,
        "parity": parity_ok,
        **result_extra,
    }
    if k1 is not None:
        out["k1_per_call"] = k1
    if hostp is not None:
        out["host_path_per_call"] = hostp
    print(json.dumps(out), flush=True)
    if sharded:
        dist.barrier()
        dist.destroy_process_group()


def link_probe(dist, rank: int, world: int, dev, backend: str, mb: int) -> dict:
    """The per-pair link rate the exchange choice and the bound model use: every rank
    sends `mb` MiB to every other rank and receives as much from each, all pairs at once in one
    P2P group (as both exchanges load the links), timed after one warm-up group; rate = bytes
    per pair / seconds, reduced with a MIN over ranks so every rank makes the same choice.
    Replaces the assumed 153 GB/s per xGMI pair (neither skill guide states one).  Over gloo
    (rehearsal) it is a host-memory rate, at most 8 MiB per pair."""
    import torch

    if world < 2:
        return dict(GBps=None, bytes_per_pair=0, seconds=None, backend=backend)
    nbytes = (min(mb, 8) if backend == "gloo" else mb) << 20
    d = dev if backend == "nccl" else torch.device("cpu")
    send = torch.ones(nbytes, dtype=torch.uint8, device=d)
    peers = [p for p in range(world) if p != rank]
    recv = [torch.empty(nbytes, dtype=torch.uint8, device=d) for _ in peers]
    ops_ = [op for p, r in zip(peers, recv) for op in (dist.P2POp(dist.isend, send, p), dist.P2POp(dist.irecv, r, p))]

    def group():
        for w in dist.batch_isend_irecv(ops_):
            w.wait()
        if d.type == "cuda":
            torch.cuda.synchronize(d)

    group()
    dist.barrier()
    t0 = time.perf_counter()
    group()
    el = time.perf_counter() - t0
    rate = torch.tensor([nbytes / el / 1e9], dtype=torch.float64, device=d)
    dist.all_reduce(rate, op=dist.ReduceOp.MIN)
    del send, recv
    if d.type == "cuda":
        torch.cuda.empty_cache()
    return dict(GBps=float(rate.item()), bytes_per_pair=nbytes, seconds_local=el, backend=backend,
                note="all pairs at once, one direction per pair; MIN over ranks")


def _round_csr(orders, weights):
    from topology_aware_learning_amd.round import csr_from_lists

    return csr_from_lists(orders, weights)


def bf16_tolerance(pin, pout, order, weights, n, dev) -> dict:
    """Row 0 of a bf16 round against the fp32 reference (K1 in exact fp32 on the same operands
    upcast): max |d| / (2^-8 |ref| + M 2^-24 sum|w x|) over the row, the SURVEY §8(a) bf16 bound."""
    import torch

    from topology_aware_learning_amd import ops

    xs = [pin.row_b16(j).float() for j in order]
    ref = torch.empty(n, dtype=torch.float32, device=dev)
    ops.agg_f32(xs, weights, ref, mode=ops.MODE_EXACT)
    mag = torch.zeros_like(ref)
    for x, w in zip(xs, weights):
        mag.add_(x.abs(), alpha=abs(float(np.float32(w))))
    bound = 2.0 ** -8 * ref.abs() + len(xs) * 2.0 ** -24 * mag
    err = (pout.row_b16(0).float() - ref).abs()
    ratio = float((err / bound.clamp_min(1e-38)).max().item())
    return dict(max_err_over_bound=ratio, within_tolerance=ratio <= 1.0,
                bound="|d| <= 2^-8 |ref| + M 2^-24 sum|w x| (SURVEY §8(a) bf16 run)")


def bench_k1(layout, pool, orders, weights, mode, dev, reps: int = 64):
    """Per-call K1 (no cross-call reuse) as the per-call product path runs it: one launch over
    the fp32 and int64 segments of a call (tal_agg_model_f32), rows rotated over the round's
    calls; SURVEY §8(d) B = 4 N (M+1) + 8 N_i64 (M+1).  HIP events around `reps` calls issued
    back to back (operand lists built beforehand), so the time is the kernels' and not the
    Python between an event and its launch (an event pair around each single call measured
    0.198 ms for a 0.157 ms kernel)."""
    import torch

    from topology_aware_learning_amd import ops

    out = torch.empty(layout.n_f32, dtype=torch.float32, device=dev)
    out_i = torch.empty(layout.n_i64, dtype=torch.int64, device=dev)
    calls = [([pool.row_f32(j) for j in orders[r % len(orders)]], [pool.row_i64(j) for j in orders[r % len(orders)]],
              weights[r % len(orders)]) for r in range(reps)]

    def call(c):
        ops.agg_model_f32(c[0], c[1], c[2], out, out_i, mode=mode)

    for c in calls[:3]:
        call(c)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        s.record()
        for c in calls:  # rotate rows: defeat the MALL
            call(c)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / len(calls))
    ms = float(np.median(ts))
    m = len(orders[0])
    b = (4 * layout.n_f32 + 8 * layout.n_i64) * (m + 1)
    return dict(kernel="k_agg_model", launches_per_call=1, ms=ms, calls_timed=len(calls), bytes=b,
                GBps=b / (ms * 1e-3) / 1e9, frac=b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                params_per_s=(layout.n_f32 + layout.n_i64) / (ms * 1e-3))


def bench_host_path(lay, m, dev, reps: int = 5):
    """Reference-shaped call: CPU state_dicts -> pinned H2D -> K1 -> D2H -> load into CPU model."""
    import torch
    import torch.nn as nn

    from topology_aware_learning_amd import synth
    from topology_aware_learning_amd.aggregate import aggregate_models

    class Holder(nn.Module):
        def __init__(self, sd):
            super().__init__()
            for i, (k, v) in enumerate(sd.items()):
                self.register_buffer(f"b{i}", v.clone())

    models = [Holder(synth.synth_state_dict(lay, 300 + i)) for i in range(m)]
    w = [1 / m] * m
    aggregate_models(models, w, models[-1])
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        aggregate_models(models, w, models[-1])
    torch.cuda.synchronize(dev)
    ms = 1e3 * (time.perf_counter() - t0) / reps
    n = sum(v.numel() for v in models[0].state_dict().values())
    return dict(ms=ms, params_per_s=n / (ms * 1e-3), note="includes pack, H2D, kernel, D2H, unpack")


VALU_LANE_OPS_PER_S = 256 * 4 * 32 * 2.4e9  # fp32 lane-ops/s: 256 CUs x 4 SIMD-32 x 2.4 GHz


def valu_floor(nnz: int, rows: int, n: int, k_ms: float, mode, bf16: bool = False) -> dict:
    """Vector-ALU floor of the round: the exact mode issues a separate multiply and add per
    operand element (no FMA; the shared-product form saves some multiplies on uniform-weight
    cliques), i.e. ~2 lane-ops per operand element.  Dense rounds (cliques) are bound here, not
    by HBM: compare floor_ms with the HBM floor bytes_per_launch / 8 TB/s.  bf16 EXACT (the
    reference's bf16 arithmetic) also rounds the product and the sum to bf16, one
    v_cvt_pk_bf16_f32 each, whose issue costs 4-5 cycles against an fp32 op's 2
    (MI355X_MICROARCH.md, per-instruction constants): 1 + 2 + 1 + 2 = 6 fp32-op equivalents per
    operand element (3 for a row's first operand).  gfx950 has no packed bf16 arithmetic that
    would fold a rounding into the multiply or the add."""
    from topology_aware_learning_amd import ops

    exact = mode == ops.MODE_EXACT
    if bf16 and exact:
        ops_round = 6 * (nnz - rows) * n + 3 * rows * n
    else:
        ops_round = (2 if exact else 1) * (nnz - rows) * n + rows * n
    floor_ms = 1e3 * ops_round / VALU_LANE_OPS_PER_S
    return dict(lane_ops=ops_round, floor_ms=floor_ms, frac=floor_ms / k_ms)


def workload_key(graph: str, devices: int, model: str, dtype: str = "f32", weights: str = "unweighted") -> str:
    return (f"{graph}-{devices}-{model}" + ("" if dtype == "f32" else f"-{dtype}")
            + ("" if weights == "unweighted" else f"-{weights}"))


def traffic_key(kernel: str, spec, workload: str) -> str:
    """profiles/traffic.json key: the round kernel, the plan spec it ran and the workload - a
    PMC byte count is only reported for the kernel and plan that produced it."""
    return f"{kernel}|{json.dumps(spec, sort_keys=True)}|{workload}"


def load_traffic(key: str):
    """HBM bytes per launch of this kernel + plan + workload from the committed rocprofv3 PMC
    summary (tools/summarize_profile.py), or None when that combination was not profiled."""
    f = ROOT / "profiles" / "traffic.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(key, {}).get("bytes_per_launch")
    except Exception:
        return None


if __name__ == "__main__":
    main()
