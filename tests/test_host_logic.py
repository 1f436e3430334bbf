"""Host-side logic of the product (weights, schedulers, centrality, layouts, plans) against the
reference's golden vectors and the oracle.  CPU only."""
import json

import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops, synth
from topology_aware_learning_amd import weights as W
from topology_aware_learning_amd.arena import StateLayout

from conftest import GOLDEN

TINY = json.loads((GOLDEN / "tiny_cases.json").read_text())
CENT = {k: {int(i): v for i, v in d.items()} for k, d in TINY["centrality"].items()}


@pytest.mark.parametrize("case", TINY["cases"], ids=lambda c: f"{c['case']}-{c['fn']}")
def test_product_weights_equal_oracle(case):
    order = case["order"]
    fn = case["fn"]
    if fn == "unweighted_module_avg":
        assert W.unweighted(case["M"]) == ra.unweighted_weights(case["M"])
    elif fn == "weighted_module_avg":
        assert W.weighted(case["data_lens"]) == ra.weighted_weights(case["data_lens"])
    elif fn == "centrality_module_avg":
        cent = CENT[case["centrality_metric"]]
        assert W.centrality(order, cent, case["softmax"], case["softmax_coeff"]) == \
            list(ra.centrality_weights(order, cent, case["softmax"], case["softmax_coeff"]))
    elif fn == "sim_centrality_module_avg":
        cent = CENT[case["centrality_metric"]]
        sims = {i: c for i, c in zip(order[:-1], case["cosine"])}
        a = W.sim_centrality(order, order[-1], cent, sims, case["softmax"], case["softmax_coeff"])
        b = ra.sim_centrality_weights(order, order[-1], cent, sims, case["softmax"], case["softmax_coeff"])
        assert a[0] == list(b[0]) and a[1] == b[1]


def test_product_onehot_weights_bitwise():
    cents = json.loads((GOLDEN / "centrality.json").read_text())
    for rec in json.loads((GOLDEN / "weights_onehot.json").read_text()):
        cent = {int(i): v for i, v in cents[rec["graph"]][rec["metric"]].items()}
        w = W.centrality(rec["order"], cent, rec["softmax"], rec["coeff"])
        assert [int(x) for x in np.asarray(w, np.float32).view(np.uint32)] == rec["w_f32_bits"]


def test_schedulers_match_reference_sequences():
    from src import aggregation_scheduler as S

    ref = json.loads((GOLDEN / "schedulers.json").read_text())
    mk = {
        "base": lambda: S.BaseScheduler(softmax_coeff=10.0),
        "exp": lambda: S.ExponentialScheduler(gamma=0.95, softmax_coeff=10.0),
        "exp_eta": lambda: S.ExponentialScheduler(gamma=0.9, eta_min=3, softmax_coeff=10.0),
        "osc": lambda: S.OscilateScheduler(T_0=5, softmax_coeff=10.0),
        "ca": lambda: S.CosineAnnealingWarmRestarts(T_0=10, eta_min=-5, softmax_coeff=10.0),
        "ca_mult2": lambda: S.CosineAnnealingWarmRestarts(T_0=4, T_mult=2, eta_min=1, softmax_coeff=100),
    }
    for name, f in mk.items():
        s = f()
        got = []
        for r in range(100):
            got.append(float(s.get_softmax_coeff()))
            s.step(r)
        assert got == ref[name], name
    raised = False
    try:
        S.CosineAnnealingWarmRestarts(T_0=66.0)
    except ValueError:
        raised = True
    assert raised == ref["ca_float_T0_raises"]


def test_centrality_dicts_match_reference():
    from src.decentralized_client import create_centrality_dict

    ref = json.loads((GOLDEN / "centrality.json").read_text())
    graphs = {"cycle_graph(8)": nx.cycle_graph(8),
              "barabasi_albert_graph(33, 2, seed=0)": nx.barabasi_albert_graph(33, 2, seed=0)}
    for name, g in graphs.items():
        got = create_centrality_dict(nx.to_numpy_array(g), np.random.default_rng(0))
        for metric in ("degree", "betweenness", "random"):
            assert {str(k): v for k, v in got[metric].items()} == ref[name][metric], (name, metric)


def test_random_coeffs_update():
    from src.decentralized_client import update_random_agg_coeffs

    d = update_random_agg_coeffs(seed=3, round_idx=4, num_clients=5, centrality_dict={})
    assert list(d["random"].values()) == np.random.default_rng(7).uniform(0, 1, 5).tolist()


def test_get_neighbors_drop_out():
    from src.decentralized_client import DecentralClient
    from torch.utils.data import TensorDataset

    ds = TensorDataset(torch.zeros(2, 1))
    c = DecentralClient(idx=0, prox_coeff=0.0, model=torch.nn.Linear(1, 1), train_data=None, test_data=None,
                        valid_data=None, global_test_data=ds, global_backdoor_test_data=None,
                        neighbors=[1, 2, 3], neighbor_probs=[1.0, 0.0, 1.0])
    np.random.seed(0)
    assert c.get_neighbors() == [1, 3]


def test_draw_neighbors_is_the_sequential_stream():
    """The driver's one-call draw per loop gives the lists and the global RNG state of one
    get_neighbors() per client in order (reference decentralized_client.py:63-71)."""
    from src.decentralized_client import DecentralClient, draw_neighbors
    from torch.utils.data import TensorDataset

    ds = TensorDataset(torch.zeros(2, 1))
    rng = np.random.default_rng(11)
    clients = []
    for i in range(40):
        k = int(rng.integers(0, 10))
        nb = sorted(rng.choice(100, size=k, replace=False).tolist())
        pr = rng.choice([0.0, 0.3, 0.5, 0.999, 1.0], size=k).tolist()
        clients.append(DecentralClient(idx=i, prox_coeff=0.0, model=torch.nn.Linear(1, 1), train_data=None,
                                       test_data=None, valid_data=None, global_test_data=ds,
                                       global_backdoor_test_data=None, neighbors=nb, neighbor_probs=pr))
    ones = [c.model_copy(update=dict(neighbor_probs=[1.0] * len(c.neighbors))) for c in clients]

    def same(sub):
        np.random.seed(4)
        seq = [c.get_neighbors() for c in sub]
        st = np.random.get_state()
        np.random.seed(4)
        assert draw_neighbors(sub) == seq
        st2 = np.random.get_state()
        assert np.array_equal(st[1], st2[1]) and st[2] == st2[2]

    # each set twice in a row (the second call reuses the concatenated probabilities); `ones`:
    # every link kept (the no-filter path)
    for sub in (clients, clients, clients[::3], clients[::3], clients[:1], [], ones, ones, ones[5:]):
        same(sub)
    clients[7].neighbor_probs[:] = [0.5] * len(clients[7].neighbor_probs)  # changed in place
    same(clients)


def test_layouts_match_reference_models():
    ref = json.loads((GOLDEN / "layouts.json").read_text())
    for name in ("cifar10", "resnet18", "resnet50"):
        assert [list(x[:1]) + [list(x[1]), x[2]] for x in synth.get_layout(name)] == \
            [[n, list(s), d] for n, s, d in ref[name]], name
    from src.modules import CifarModule
    from src.models.resnet import ResNet18, ResNet50

    for name, ctor in (("cifar10", lambda: CifarModule(10)), ("resnet18", ResNet18), ("resnet50", ResNet50)):
        lay = synth.layout_of(ctor().state_dict())
        assert [[n, list(s), d] for n, s, d in lay] == [[n, list(s), d] for n, s, d in ref[name]], name


def test_vit_b16_layout_size():
    lay = synth.get_layout("vit_b16")
    assert len(lay) == 152 and synth.layout_counts(lay) == (86567656, 0)


def test_state_layout_segments_and_aliases():
    m = torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.BatchNorm1d(4))
    m[1].num_batches_tracked.fill_(5)
    lay = StateLayout.from_state_dict(m.state_dict())
    assert lay.n_f32 == 12 + 4 + 4 * 4 and lay.n_i64 == 1
    f = torch.zeros(lay.ld_f32)
    i = torch.zeros(lay.ld_i64, dtype=torch.int64)
    lay.flatten_into(m.state_dict(), f, i)
    for k, v in lay.views(f, i).items():
        assert torch.equal(v, m.state_dict()[k])

    class Tied(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4, bias=False)
            self.b = torch.nn.Linear(4, 4, bias=False)
            self.b.weight = self.a.weight

    t = Tied()
    lay = StateLayout.from_state_dict(t.state_dict())
    assert lay.n_f32 == 16 and lay.by_name["b.weight"].alias_of == "a.weight"


def test_cosine_segments_reproduce_reference_semantics():
    """(offset, A, I, B) decomposition + the cosine formula == the reference's values."""
    lay = [(n, tuple(s), d) for n, s, d in TINY["layout"]]
    z = np.load(GOLDEN / "tiny_cases.npz")
    layout = StateLayout.from_layout(lay)
    names = synth.param_names(lay)
    segs = layout.param_segments(names)
    for case in [c for c in TINY["cases"] if c["fn"] == "sim_centrality_module_avg"][:6]:
        ci = case["case"]
        flat = lambda i: np.concatenate([z[f"c{ci}_in{i}_{n}"].reshape(-1) for n, _, d in lay if d == "float32"])
        a = flat(case["M"] - 1)
        for j, ref in enumerate(case["cosine"]):
            b = flat(j)
            tot = 0.0
            for off, A, I, B in segs:
                x = a[off: off + A * I * B].reshape(A, I, B).astype(np.float64)
                y = b[off: off + A * I * B].reshape(A, I, B).astype(np.float64)
                nx_ = np.maximum(np.sqrt((x * x).sum(1)), 1e-6)
                ny_ = np.maximum(np.sqrt((y * y).sum(1)), 1e-6)
                tot += float(((x * y).sum(1) / nx_ / ny_).mean())
            got = tot / len(segs)
            if ci % 3 == 0:  # fp32 overflow rows: covered by the fp32 restatement in the oracle tests
                continue
            assert abs(got - ref) < 1e-5


def test_narrow_plan_orders_rows_by_operand_count():
    """Narrow plans (c4 16 / 32) reorder each group's rows by operand count (descending, stable);
    every row keeps its operands, weights and output row."""
    g = nx.stochastic_block_model([32] * 4, [[0.45 if a == b else 0.02 for b in range(4)] for a in range(4)], seed=1)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(g.number_of_nodes())]
    ws = [W.unweighted(len(o)) for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    rows = len(orders)
    out_rows = np.random.default_rng(0).permutation(rows).astype(np.int32)
    want = {int(out_rows[r]): (col[row_ptr[r]:row_ptr[r + 1]].tolist(), w[row_ptr[r]:row_ptr[r + 1]].astype(np.float32).tolist())
            for r in range(rows)}
    for c4, budget in ((16, 160 * 1024), (32, 40 * 1024)):
        plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=budget)
        i, h = plan.info, plan.host
        grp_row = h[i.off_grp_row_ptr: i.off_grp_row_ptr + i.n_groups + 1]
        grp_src = h[i.off_grp_src_ptr: i.off_grp_src_ptr + i.n_groups + 1]
        src_row = h[i.off_src_row: i.off_src_row + i.total_src]
        rp = h[i.off_row_ptr: i.off_row_ptr + i.rows + 1]
        slot = h[i.off_op_slot: i.off_op_slot + i.nnz]
        wf = h[i.off_op_w: i.off_op_w + i.nnz].view(np.float32)
        orow = h[i.off_out_row: i.off_out_row + i.rows]
        assert sorted(orow.tolist()) == list(range(rows))
        got = {}
        for gi in range(i.n_groups):
            srcs = src_row[grp_src[gi]: grp_src[gi + 1]]
            counts = np.diff(rp[grp_row[gi]: grp_row[gi + 1] + 1])
            assert np.all(np.diff(counts) <= 0)  # descending operand counts within the group
            for r in range(grp_row[gi], grp_row[gi + 1]):
                got[int(orow[r])] = ([int(srcs[slot[k]]) for k in range(rp[r], rp[r + 1])],
                                     [float(x) for x in wf[rp[r]: rp[r + 1]]])
        assert got == want


def test_narrow_roww_encoding():
    """Row-uniform weights: 16-bit slots in batches of 4 padded with the zero tile that keeps
    -0 (slot ns for a weight with the sign bit clear, ns + 1 otherwise), one weight per row."""
    g = nx.random_regular_graph(4, 24, seed=5)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(24)]
    for sign in (1.0, -1.0):
        ws = [[sign / len(o)] * len(o) for o in orders]
        row_ptr, col, w = ra.round_csr(orders, ws)
        plan = ops.build_plan(row_ptr, col, w, np.arange(24, dtype=np.int32), c4=16, lds_bytes=80 * 1024)
        i, h = plan.info, plan.host
        assert i.narrow_roww == 1 and i.n_groups == 1
        rp = h[i.off_nrow_ptr: i.off_nrow_ptr + i.rows + 1]
        slots = h[i.off_npairs: i.off_npairs + (i.npairs + 1) // 2].view(np.uint16)[: i.npairs]
        rw = h[i.off_nrow_w: i.off_nrow_w + i.rows].view(np.float32)
        src = h[i.off_src_row: i.off_src_row + i.total_src]
        ns = i.total_src
        orow = h[i.off_out_row: i.off_out_row + i.rows]
        for r in range(i.rows):
            assert rp[r] % 4 == 0 and rp[r + 1] % 4 == 0
            run = slots[rp[r]: rp[r + 1]] // 16
            o = orders[orow[r]]
            assert [int(src[x]) for x in run[: len(o)]] == o
            assert np.all(run[len(o):] == (ns if sign > 0 else ns + 1)) and len(run) - len(o) < 4
            assert rw[r] == np.float32(sign / len(o))
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    ws[3] = list(np.linspace(0.1, 0.2, len(orders[3])))  # one non-uniform row: pairs
    row_ptr, col, w = ra.round_csr(orders, ws)
    plan = ops.build_plan(row_ptr, col, w, np.arange(24, dtype=np.int32), c4=16, lds_bytes=80 * 1024)
    assert plan.info.narrow_roww == 0


@pytest.mark.parametrize("c4", [16, 32])
def test_narrow_roww_pass_uniform_batches(c4):
    """ROWW rows ordered by operand count; every pass of 64 / c4 consecutive rows padded to the
    batch count of its first row (the kernel's row loop then counts on the scalar unit); the
    padding reads the zero tile."""
    g = nx.barabasi_albert_graph(61, 3, seed=2)  # degrees 3 .. 30
    orders = [sorted(g.neighbors(i)) + [i] for i in range(61)]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    plan = ops.build_plan(row_ptr, col, w, np.arange(61, dtype=np.int32), c4=c4, lds_bytes=160 * 1024)
    i, h = plan.info, plan.host
    assert i.narrow_roww == 1 and i.n_groups == 1
    rp = h[i.off_nrow_ptr: i.off_nrow_ptr + i.rows + 1]
    slots = h[i.off_npairs: i.off_npairs + (i.npairs + 1) // 2].view(np.uint16)[: i.npairs]
    orow = h[i.off_out_row: i.off_out_row + i.rows]
    src = h[i.off_src_row: i.off_src_row + i.total_src]
    lens = [len(orders[orow[r]]) for r in range(i.rows)]
    assert lens == sorted(lens, reverse=True)
    rpw = 64 // c4
    for r in range(i.rows):
        lead = r // rpw * rpw
        assert rp[r + 1] - rp[r] == 4 * ((lens[lead] + 3) // 4)
        run = slots[rp[r]: rp[r + 1]] // c4
        assert [int(src[x]) for x in run[: lens[r]]] == orders[orow[r]]
        assert np.all(run[lens[r]:] == i.total_src)  # the -0.0 tile (positive weights)


def test_narrow_roww_needs_16bit_slots():
    """ROWW slots are 16-bit (slot * c4): a round whose sources could overflow them takes the
    pairs form instead of silently wrapping."""
    n = 5000
    orders = [[(i - 1) % n, (i + 1) % n, i] for i in range(n)]
    orders = [sorted(o[:2]) + [o[2]] for o in orders]
    row_ptr, col, w = ra.round_csr(orders, [ra.unweighted_weights(3)] * n)
    plan = ops.build_plan(row_ptr, col, w, np.arange(n, dtype=np.int32), c4=16, lds_bytes=80 * 1024)
    assert plan.info.narrow_roww == 0


def test_round_plan_reconstructs_csr():
    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    ws = [W.unweighted(len(o)) for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(64, dtype=np.int32)[::-1].copy()
    for c4, budget, dense in ((64, ops.LDS_BUDGET, 0), (64, 20 * 1024, 0), (128, 40 * 1024, 0),
                              (64, ops.LDS_BUDGET, 8), (128, 40 * 1024, 8), (16, ops.LDS_BUDGET, 0),
                              (32, 12 * 1024, 0), (16, 160 * 1024, 8)):
        plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=budget, dense=dense)
        i, h = plan.info, plan.host
        grp_row = h[i.off_grp_row_ptr: i.off_grp_row_ptr + i.n_groups + 1]
        grp_src = h[i.off_grp_src_ptr: i.off_grp_src_ptr + i.n_groups + 1]
        src_row = h[i.off_src_row: i.off_src_row + i.total_src]
        rp = h[i.off_row_ptr: i.off_row_ptr + i.rows + 1]
        slot = h[i.off_op_slot: i.off_op_slot + i.nnz]
        wf = h[i.off_op_w: i.off_op_w + i.nnz].view(np.float32)
        assert np.array_equal(rp, row_ptr) and np.array_equal(h[i.off_out_row: i.off_out_row + i.rows], out_rows)
        assert np.array_equal(wf, w.astype(np.float32))
        assert grp_row[0] == 0 and grp_row[-1] == 64 and np.all(np.diff(grp_row) > 0)
        rec = np.empty_like(col)
        for gi in range(i.n_groups):
            srcs = src_row[grp_src[gi]: grp_src[gi + 1]]
            assert len(set(srcs.tolist())) == len(srcs) <= i.max_src
            assert np.all(np.diff(srcs) > 0)  # staged in ascending pool-row order
            for r in range(grp_row[gi], grp_row[gi + 1]):
                for k in range(rp[r], rp[r + 1]):
                    rec[k] = srcs[slot[k]]
        assert np.array_equal(rec, col)
        assert i.dense_rb == (dense if c4 >= 64 else 0)  # narrow tiles are sparse only
        if i.dense_rb:
            blk_ptr = h[i.off_grp_blk_ptr: i.off_grp_blk_ptr + i.n_groups + 1]
            tabs = h[i.off_blk_tab: i.off_blk_tab + i.n_blocks]
            reads = 0
            for gi in range(i.n_groups):
                for lb in range(blk_ptr[gi + 1] - blk_ptr[gi]):
                    t0 = tabs[blk_ptr[gi] + lb]
                    n_used = h[t0]
                    assert n_used % 4 == 0 and t0 % 8 == 0
                    e_slot = h[t0 + 8: t0 + 8 + n_used]
                    e_mask = h[t0 + 8 + n_used: t0 + 8 + 2 * n_used]
                    e_w = h[t0 + 8 + 2 * n_used: t0 + 8 + 2 * n_used + n_used * dense].reshape(n_used, dense)
                    ent = np.concatenate([e_slot[:, None], e_mask[:, None], e_w], axis=1)
                    real = ent[:, 1] != 0
                    assert np.all(np.diff(ent[real, 0]) > 0) and np.all(ent[~real, 2:] == 0)
                    ent = ent[real]
                    n_used = len(ent)
                    rows_here = 0
                    for rr in range(dense):
                        r = grp_row[gi] + lb * dense + rr
                        if r >= grp_row[gi + 1]:
                            assert not np.any(ent[:, 1] & (1 << rr))
                            continue
                        rows_here += 1
                        used = {slot[k]: w[k] for k in range(rp[r], rp[r + 1] - 1)}  # self excluded
                        for e in range(n_used):
                            bit = bool(ent[e, 1] & (1 << rr))
                            assert bit == (int(ent[e, 0]) in used)
                            if bit:
                                assert ent[e, 2 + rr].view(np.float32) == np.float32(used[int(ent[e, 0])])
                    reads += n_used + rows_here
            assert reads == i.dense_reads
        assert i.lds_bytes <= budget
        if budget == ops.LDS_BUDGET:
            assert i.n_groups == 1 and i.total_src == 64


def _emulate_stream(plan, pool):
    """The streamed kernel's walk (k_round_stream) in numpy fp32: chunk by chunk, batches of 4
    table entries, own model captured when its chunk passes and added last."""
    i, h = plan.info, plan.host
    cs = i.stream_cs
    grp_row = h[i.off_grp_row_ptr: i.off_grp_row_ptr + i.n_groups + 1]
    grp_src = h[i.off_grp_src_ptr: i.off_grp_src_ptr + i.n_groups + 1]
    src_row = h[i.off_src_row: i.off_src_row + i.total_src]
    rp = h[i.off_row_ptr: i.off_row_ptr + i.rows + 1]
    slot = h[i.off_op_slot: i.off_op_slot + i.nnz]
    wf = h[i.off_op_w: i.off_op_w + i.nnz].view(np.float32)
    out_row = h[i.off_out_row: i.off_out_row + i.rows]
    blk_ptr = h[i.off_grp_blk_ptr: i.off_grp_blk_ptr + i.n_groups + 1]
    tabs = h[i.off_blk_tab: i.off_blk_tab + i.n_blocks]
    out = np.zeros_like(pool)
    for gi in range(i.n_groups):
        srcs = src_row[grp_src[gi]: grp_src[gi + 1]]
        nch = (len(srcs) + cs - 1) // cs
        for lb in range(blk_ptr[gi + 1] - blk_ptr[gi]):
            t0 = tabs[blk_ptr[gi] + lb]
            nu = h[t0]
            e_slot = h[t0 + 8: t0 + 8 + nu]
            e_mask = h[t0 + 8 + nu: t0 + 8 + 2 * nu]
            e_w = h[t0 + 8 + 2 * nu: t0 + 8 + 2 * nu + 8 * nu].view(np.float32).reshape(nu, 8)
            rows = [grp_row[gi] + lb * 8 + r for r in range(8) if grp_row[gi] + lb * 8 + r < grp_row[gi + 1]]
            acc = np.full((8, pool.shape[1]), -0.0, np.float32)
            e = 0
            for k in range(nch):
                lo, hi = k * cs, k * cs + cs
                while e < nu:
                    if e_slot[e] >= hi:
                        break
                    assert np.all((e_slot[e: e + 4] >= lo) & (e_slot[e: e + 4] < hi))  # one chunk per batch
                    for u in range(4):
                        x = pool[srcs[e_slot[e + u]]]
                        for r in range(8):
                            if e_mask[e + u] & (1 << r):
                                acc[r] = acc[r] + np.float32(e_w[e + u, r]) * x
                    e += 4
            assert e == nu
            for r, gr in enumerate(rows):
                q = rp[gr + 1] - 1
                out[out_row[gr]] = acc[r] + wf[q] * pool[srcs[slot[q]]]
    return out


@pytest.mark.parametrize("graph", ["clique", "barbell", "ring", "random"])
def test_stream_plan_walk_matches_oracle(graph):
    rng = np.random.default_rng(5)
    if graph == "clique":
        n_dev = 40
        orders = [[j for j in range(n_dev) if j != i] + [i] for i in range(n_dev)]
    elif graph == "barbell":
        g = nx.barbell_graph(30, 3)
        n_dev = g.number_of_nodes()
        orders = [sorted(g.neighbors(i)) + [i] for i in range(n_dev)]
    elif graph == "ring":
        n_dev = 70
        orders = [sorted({(i - 1) % n_dev, (i + 1) % n_dev}) + [i] for i in range(n_dev)]
    else:
        g = nx.gnp_random_graph(150, 0.1, seed=3)
        n_dev = 150
        orders = [sorted(g.neighbors(i)) + [i] for i in range(n_dev)]
    ws = [[float(x) for x in rng.dirichlet(np.ones(len(o)))] for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(n_dev, dtype=np.int32)
    pool = rng.standard_normal((n_dev, 7)).astype(np.float32)
    pool[0, 0] = -0.0
    ref = oracle.round_f32(pool, row_ptr, col, w, out_rows)
    for max_rows, max_src in ((64, 0), (128, 0), (16, 0), (64, 24)):
        plan = ops.build_stream_plan(row_ptr, col, w, out_rows, max_rows, max_src)
        i = plan.info
        assert i.stream_cs in (16, 32) and i.c4 == 64 and i.dense_rb == 8
        assert i.max_rows <= min(max_rows, 4 * i.stream_cs)
        got = _emulate_stream(plan, pool)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (graph, max_rows, max_src)


def test_stream_plan_rejects_non_reference_order():
    row_ptr = np.array([0, 3], np.int32)
    col = np.array([2, 1, 0], np.int32)  # unsorted neighbors
    with pytest.raises(Exception, match="reference order"):
        ops.build_stream_plan(row_ptr, col, np.full(3, 1 / 3), np.zeros(1, np.int32))


def test_round_plan_capacity_error():
    row_ptr = np.array([0, 300], np.int32)
    col = np.arange(300, dtype=np.int32)
    w = np.full(300, 1 / 300)
    with pytest.raises(Exception, match="LDS"):
        ops.build_plan(row_ptr, col, w, np.zeros(1, np.int32), c4=64, lds_bytes=64 * 1024)


def test_prox_plan_covers_parameter_segments():
    from topology_aware_learning_amd.aggregate import layout_of_module
    from topology_aware_learning_amd.prox import ProxPlan
    from _models import TinyNet

    m = TinyNet()
    lay = layout_of_module(m)
    names = [n for n, _ in m.named_parameters()]
    pl = ProxPlan(lay, names, "cpu")
    h = pl.plan.numpy()
    ptr = h[: pl.n_seg + 1]
    ch = h[pl.n_seg + 1:].reshape(-1, 3)
    assert len(ch) == pl.n_chunks == ptr[-1]
    for s, name in enumerate(names):
        e = lay.by_name[name]
        rows = ch[ptr[s]: ptr[s + 1]]
        assert np.all(rows[:, 0] == s)
        assert rows[0, 1] == e.offset and rows[:, 2].sum() == e.numel
        assert np.all(rows[1:, 1] == rows[:-1, 1] + rows[:-1, 2])  # contiguous chunks


def _orders_of(g):
    return [sorted(g.neighbors(i)) + [i] for i in sorted(g.nodes)]


def test_find_cliques_barbell_complete_and_rejections():
    import networkx as nx

    from oracle import reference_alg as ra
    from topology_aware_learning_amd import ops

    g = nx.barbell_graph(12, 4)  # cliques 0..11 and 16..27, path 12..15
    orders = _orders_of(g)
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    rp, col, w = ra.round_csr(orders, ws)
    out = np.arange(len(orders), dtype=np.int32)[::-1].copy()
    cliques, rest = ops.find_cliques(rp, col, w, out)
    assert len(cliques) == 2
    for srcs, w32, outs, _ in cliques:
        assert len(srcs) == 12 and len(outs) == 11  # the bridge node has one more neighbor
        assert w32 == np.float32(1 / 12)
        for i, o in outs.items():  # member i's row: every other member ascending, then itself
            r = int(np.flatnonzero(out == o)[0])
            assert list(col[rp[r]: rp[r + 1]]) == [s for s in srcs if s != srcs[i]] + [srcs[i]]
    assert sorted(rest) == [12, 13, 14, 15]  # the path; the bridge rows 11 and 16 are attached
    for srcs, w32, outs, att in cliques:
        assert len(att) == 1 and bin(att[0]["mask"]).count("1") == 11 and len(att[0]["ext"]) == 1
    # a complete graph is one block; a ring has none
    oc = _orders_of(nx.complete_graph(20))
    rp, col, w = ra.round_csr(oc, [ra.unweighted_weights(20)] * 20)
    cl, rest = ops.find_cliques(rp, col, w, np.arange(20))
    assert len(cl) == 1 and len(cl[0][2]) == 20 and rest == []
    orr = _orders_of(nx.cycle_graph(16))
    rp, col, w = ra.round_csr(orr, [ra.unweighted_weights(3)] * 16)
    assert ops.find_cliques(rp, col, w, np.arange(16))[0] == []
    # per-operand weights (centrality) and self not last are not cliques
    cent = nx.degree_centrality(nx.complete_graph(20))
    wc = [ra.centrality_weights(o, cent, True, 10.0) for o in oc]
    wc[0] = [0.5] + [0.5 / 19] * 19
    rp, col, w = ra.round_csr(oc, wc)
    assert all(len(c[2]) < 20 for c in ops.find_cliques(rp, col, w, np.arange(20), min_rows=2)[0])
    shuffled = [o[-1:] + o[:-1] for o in oc]
    rp, col, w = ra.round_csr(shuffled, [ra.unweighted_weights(20)] * 20)
    assert ops.find_cliques(rp, col, w, np.arange(20))[0] == []


def test_clique_plan_table_and_spec():
    import networkx as nx

    from oracle import reference_alg as ra
    from topology_aware_learning_amd import ops

    orders = _orders_of(nx.barbell_graph(60, 8))
    rp, col, w = ra.round_csr(orders, [ra.unweighted_weights(len(o)) for o in orders])
    out = np.arange(len(orders), dtype=np.int32)
    p = ops.build_clique_plan(rp, col, w, out)
    assert p.n_cliques == 2 and p.mmax == 60 and p.clique_rows == 120  # + the two bridge rows
    t = p.table.reshape(p.n_cliques, ops.CLIQUE_WORDS)
    assert list(t[:, 0]) == [60, 60] and (t[:, 1].view(np.float32) == np.float32(1 / 60)).all()
    assert p.rest is not None and p.rest.rows == 8 and p.full.rows == 128
    assert p.staged_rows() == 120 + 2 + p.rest.staged_rows()  # + each bridge's path neighbor
    q = ops.plan_from_spec(rp, col, w, out, {"clique": 1})
    assert np.array_equal(q.table, p.table)
    assert ops.round_kernel_name(p) == "k_round_clique"
    ring = _orders_of(nx.cycle_graph(16))
    rp, col, w = ra.round_csr(ring, [ra.unweighted_weights(3)] * 16)
    assert ops.build_clique_plan(rp, col, w, np.arange(16)) is None


def _bench_round(kind, n, deg):
    import bench
    from topology_aware_learning_amd.round import csr_from_lists

    orders, weights = bench.round_spec(n, deg, kind=kind)
    rp, col, w = csr_from_lists(orders, weights)
    return rp, col, w, np.arange(len(orders), dtype=np.int32)


@pytest.mark.parametrize("kind,n,deg,form", [
    ("ring", 32, 2, "sparse-wide"),      # config 2: c4 64/128 sparse won (0.55-0.58 ms), dense 0.72-0.85
    ("random", 64, 8, "sparse-wide"),    # config 3: c4 64 sparse 2.45 ms, dense 6.22 ms
    ("barbell", 128, 0, "clique"),       # config 4: K3c 4.95 ms, best LDS-tiled plan 10.3 ms
    ("sbm", 256, 0, "narrow-16"),        # config 5: narrow c4 16 (one group) 36.5 ms, c4 64 83 ms
])
def test_default_plan_forms(kind, n, deg, form):
    """The untimed plan the round components build (RoundExecutor, ShardedRound,
    TransposedRound with tune=False) has the form that won the round-1 tuner A/B on the driver's
    box for each BASELINE config (BENCH_r01 / profiles/r01/config_c*.json candidates)."""
    p = ops.default_plan(*_bench_round(kind, n, deg))
    if form == "clique":
        assert isinstance(p, ops.CliquePlan) and p.n_cliques == 2 and p.rest.info.dense_rb == 0
        return
    assert isinstance(p, ops.RoundPlan) and p.info.dense_rb == 0 and p.info.stream_cs == 0
    if form == "sparse-wide":
        assert p.info.c4 >= 64 and p.info.n_groups == 1
    else:
        assert p.info.c4 == 16 and p.info.n_groups == 1 and p.staged_rows() == 256


def test_default_plan_bf16_per_operand_weights():
    """Config 5 with degree-centrality softmax weights: bf16 FMA rounds default to the narrow
    kernel's two-chunk broadcast form (c4 = 32, 16 wavefronts, one workgroup per CU: 23.0-23.3
    ms in round 4 against K3r's 29.8), fp32 rounds (either mode) to its 8-wavefront form (42.2 ms against 46.0 for the
    cost model's two-group pairs plan), each one group so RoundExecutor runs it in place; bf16
    EXACT keeps the narrow pairs form, and unweighted rounds the narrow ROWW form."""
    import bench
    from topology_aware_learning_amd.round import csr_from_lists

    orders, ws = bench.round_spec(256, 8, kind="sbm", weights="degcent")
    rp, col, w = csr_from_lists(orders, ws)
    rows = np.arange(len(orders), dtype=np.int32)
    p = ops.default_plan(rp, col, w, rows, bf16=True, mode=ops.MODE_FMA)
    assert isinstance(p, ops.RoundPlan) and p.info.narrow_bcast == 16 and p.info.bc_wg_per_cu == 1
    assert p.info.c4 == 32 and p.single_group and p.spec["bcast"] == 16 and p.staged_rows() == 256
    for kw in (dict(bf16=False, mode=ops.MODE_FMA), dict(bf16=False)):
        q = ops.default_plan(rp, col, w, rows, **kw)
        assert isinstance(q, ops.RoundPlan) and q.info.narrow_bcast == 8 and q.info.bc_wg_per_cu == 2
        assert q.single_group and q.staged_rows() == 256
    q = ops.default_plan(rp, col, w, rows, bf16=True, mode=ops.MODE_EXACT)
    assert isinstance(q, ops.RoundPlan) and q.info.c4 == 16 and not q.info.narrow_roww and not q.info.narrow_bcast
    orders, ws = bench.round_spec(256, 8, kind="sbm")
    rp, col, w = csr_from_lists(orders, ws)
    for kw in (dict(bf16=True, mode=ops.MODE_FMA), dict(bf16=False)):
        q = ops.default_plan(rp, col, w, rows, **kw)
        assert isinstance(q, ops.RoundPlan) and q.info.narrow_roww


def test_auto_dense_only_for_cliques():
    """dense_rb = -1 (library's choice) keeps random graphs sparse and takes dense row blocks on
    a complete graph (one LDS read serves every row of a block)."""
    p = ops.build_plan(*_bench_round("random", 64, 8), c4=64, lds_bytes=80 * 1024, dense=-1)
    assert p.info.dense_rb == 0
    g = nx.complete_graph(40)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(40)]
    from topology_aware_learning_amd.round import csr_from_lists

    rp, col, w = csr_from_lists(orders, [[1 / 40] * 40] * 40)
    p = ops.build_plan(rp, col, w, np.arange(40, dtype=np.int32), c4=64, lds_bytes=160 * 1024, dense=-1)
    assert p.info.dense_rb == 8


# DESIGN.md §6 "Busiest-pair volumes" table (GB per round, contiguous blocks): halo / transpose
_DESIGN_LINK_TABLE = {
    ("barbell", 128, "resnet50"): {2: (0.09, 6.03), 4: (3.02, 1.51), 8: (1.51, 0.38)},
    ("sbm", 256, "vit_b16"): {2: (30.13, 44.32), 4: (12.12, 11.08), 8: (4.85, 2.77)},
    ("random", None, "resnet50"): {2: (6.03, 6.03), 4: (5.85, 3.02), 8: (4.81, 1.51)},
}


def test_link_model_matches_design_table():
    """bench.py's N > 1 bound model (transposed.link_model) reproduces DESIGN §6's busiest-pair
    table for configs 4 and 5 and the weak-scaling graph at 2 / 4 / 8 GPUs, chooses the
    exchange with the smaller busiest pair (as choose_exchange does), and names the binding
    term consistently with its own times."""
    import bench
    from topology_aware_learning_amd import synth
    from topology_aware_learning_amd.arena import StateLayout
    from topology_aware_learning_amd.distributed import partition_contiguous
    from topology_aware_learning_amd.transposed import choose_exchange, link_model

    for (kind, nd, model), rows in _DESIGN_LINK_TABLE.items():
        lay = StateLayout.from_layout(synth.get_layout(model))
        for world, (halo_gb, tr_gb) in rows.items():
            orders, _ = bench.round_spec(nd or 64 * world, 8, kind=kind)
            owner = partition_contiguous(len(orders), world)
            m = link_model(orders, owner, world, lay.n_f32, lay.n_i64, lay.n_b16)
            assert round(m["halo"]["busiest_pair_bytes"] / 1e9, 2) == halo_gb, (kind, world)
            assert round(m["transpose"]["busiest_pair_bytes"] / 1e9, 2) == tr_gb, (kind, world)
            for v in m.values():
                assert v["predicted_ms"] == max(v["hbm_ms"], v["link_ms"])
                assert v["binds"] == ("xgmi" if v["link_ms"] > v["hbm_ms"] else "hbm")
            ch = choose_exchange(orders, owner, world, lay.n_f32, lay.n_i64, lay.n_b16)
            assert ch == ("transpose" if tr_gb < 0.9 * halo_gb else "halo"), (kind, world)
    # one rank (bench.py --sharded): no link at all, both exchanges bound by HBM
    orders, _ = bench.round_spec(64, 8, kind="random")
    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    m = link_model(orders, partition_contiguous(64, 1), 1, lay.n_f32, lay.n_i64, lay.n_b16)
    for v in m.values():
        assert v["busiest_pair_bytes"] == 0 and v["binds"] == "hbm" and v["predicted_ms"] > 0


def test_reg_plan_table_layout():
    """build_reg_plan (K3r): every row in exactly one group, each group's operands among its
    <= 64 sources (the list padded to 16 x NB entries with its first source), rows paired in
    operand-count order, each pair's trip records {A idx x4, B idx x4, A w x4, B w x4} holding
    the rows' operands in reference order as 2 x slot with their fp32 weights, the rest of a
    pair's trips the neutral operand (offset 32 x NB, weight +0.0), one record of read-ahead
    padding after the last (tal_agg.h K3r layout)."""
    import bench
    from oracle import reference_alg as ra
    from topology_aware_learning_amd import ops

    for weights in ("unweighted", "degcent"):
        orders, ws = bench.round_spec(256, 8, kind="sbm", weights=weights)
        row_ptr, col, w = ra.round_csr(orders, ws)
        out_rows = np.arange(len(orders), dtype=np.int32)[::-1].copy()
        p = ops.build_reg_plan(row_ptr, col, w, out_rows)
        t = p.table
        nb = (p.max_src + 15) // 16
        span, neutral = 16 * nb, 32 * nb
        grp = t[: 4 * p.n_groups].reshape(-1, 4)
        pairs = p.pair_records()
        assert p.max_src <= 64 and p.off_pairs % 4 == 0 and p.off_rec % 16 == 0
        assert len(t) == p.off_rec + 16 * (p.trips + 1)
        seen = []
        for g, (s0, ns, p0, npair) in enumerate(grp):
            assert s0 == g * span and ns <= 64
            srcs = t[p.off_src + s0: p.off_src + s0 + ns]
            assert list(srcs) == sorted(set(srcs.tolist()))
            assert np.all(t[p.off_src + s0 + ns: p.off_src + s0 + span] == srcs[0])
            counts = []
            for k, (oa, ob, trips, boff) in enumerate(pairs[p0: p0 + npair]):
                assert boff % 64 == 0 and trips >= 1
                rec = t[boff // 4: boff // 4 + 16 * trips].reshape(trips, 16)
                idx_a, idx_b = rec[:, 0:4].reshape(-1), rec[:, 4:8].reshape(-1)
                w_a, w_b = rec[:, 8:12].reshape(-1).view(np.uint32), rec[:, 12:16].reshape(-1).view(np.uint32)
                assert ob >= 0 or k == npair - 1
                lens = []
                for out, idx, wv in ((oa, idx_a, w_a), (ob, idx_b, w_b)):
                    if out < 0:
                        assert np.all(idx == neutral) and np.all(wv == 0)
                        continue
                    r = int(np.flatnonzero(out_rows == out)[0])
                    seen.append(r)
                    m = len(orders[r])
                    lens.append(m)
                    assert [srcs[i // 2] for i in idx[:m]] == list(orders[r]) and np.all(idx[:m] % 2 == 0)
                    assert np.array_equal(wv[:m], np.float32(ws[r]).view(np.uint32))
                    assert np.all(idx[m:] == neutral) and np.all(wv[m:] == 0)
                assert trips == (max(lens) + 3) // 4
                counts.extend(lens)
            assert counts == sorted(counts, reverse=True)
        assert sorted(seen) == list(range(len(orders)))
    assert ops.build_reg_plan(row_ptr, col, w, out_rows, max_src=8) is None  # a row has 9+ sources


def test_select_pool_pair_keeps_first_unless_clearly_faster():
    """Placement calibration (arena.select_pool_pair): a pair is chosen by its best-of-two round
    trip; the first two allocations stay unless another pair beats them by more than 2 % (on
    a VALU-bound round all placements run alike and the minimum is noise)."""
    from topology_aware_learning_amd.arena import select_pool_pair

    def run(dest_ms, noise=0.0):
        made = iter(range(len(dest_ms)))
        calls = []

        def score(a, b):
            calls.append((a, b))
            return dest_ms[b] * (1 + noise * (len(calls) % 3 - 1))

        a, b, rep = select_pool_pair(lambda: next(made), score, len(dest_ms))
        return (a, b), rep

    # pools 2 and 3 write 20 % faster: kept
    pair, rep = run([2.4, 2.4, 2.0, 2.0, 2.4, 2.4])
    assert set(pair) == {2, 3} and rep["first_pair_ms"] == 2.4 and rep["chosen_pair_ms"] == 2.0
    # all alike within 1 % (noise): the first two stay
    pair, _ = run([4.20, 4.21, 4.17, 4.18, 4.19, 4.22], noise=0.004)
    assert pair == (0, 1)


def test_binding_check_sees_last_entry_and_hooks_uninstall():
    """the O(1) binding check also compares the last entry (a Tensor.set_ of it,
    which no hook sees, unbinds the model); uninstall_hooks() restores torch, after which every
    check is the full per-entry one; bind() installs the hooks again."""
    import torch.nn as nn

    from topology_aware_learning_amd import arena
    from topology_aware_learning_amd.arena import ModelPool, StateLayout, bound_row

    def make():
        return nn.Sequential(nn.Linear(3, 4), nn.BatchNorm1d(4), nn.Linear(4, 2))

    m = make()
    lay = StateLayout.from_state_dict(m.state_dict())
    pool = ModelPool(lay, 2, "cpu")
    pool.bind(m, 1)
    assert bound_row(m) == (pool, 1)
    last = list(m.state_dict().values())[-1]  # the last entry (the final Linear's bias)
    with torch.no_grad():
        m[2].bias.set_(torch.zeros(2))  # re-pointed without any hook firing
    assert bound_row(m) is None
    m2 = make()
    pool.bind(m2, 0)
    assert bound_row(m2) == (pool, 0)
    orig_apply = arena._RESTORE[0][2]
    arena.uninstall_hooks()
    assert nn.Module._apply is orig_apply and "data" not in nn.Parameter.__dict__
    assert bound_row(m2) == (pool, 0)  # full check, still bound
    m2[0].weight.data = torch.zeros(4, 3)  # no hook now: the full check sees it
    assert bound_row(m2) is None
    m3 = make()
    pool.bind(m3, 0)
    assert arena._HOOKS and bound_row(m3) == (pool, 0)
    del last


@pytest.mark.parametrize("graph,devices,model,dtype,weights,mode,fixture", [
    ("random", 64, "resnet50", "f32", "unweighted", "exact", "full_round_c3_resnet50_rr64.json"),
    ("barbell", 128, "resnet50", "f32", "unweighted", "exact", "full_round_c4_resnet50_barbell.json"),
    ("sbm", 256, "vit_b16", "f32", "unweighted", "exact", "full_round_c5_vit_sbm256.json f32 unweighted_module_avg"),
    ("sbm", 256, "vit_b16", "f32", "degcent", "exact", "full_round_c5_vit_sbm256.json f32 centrality_module_avg"),
    ("sbm", 256, "vit_b16", "bf16", "unweighted", "exact", "full_round_c5_vit_sbm256.json bf16 unweighted_module_avg"),
    ("sbm", 256, "vit_b16", "bf16", "unweighted", "fma", None),
    ("random", 512, "resnet50", "f32", "unweighted", "exact", None)])
def test_bench_reference_fixture_choice(graph, devices, model, dtype, weights, mode, fixture):
    """bench.reference_fixture: the BASELINE configs the reference's full-round fixtures cover
    get their per-model digests (operand order checked against this run's graph, seeds =
    base + device id); other workloads (bf16 FMA, weak scaling) fall back to K1 on regenerated
    operands."""
    import argparse

    import bench

    a = argparse.Namespace(graph=graph, model=model, dtype=dtype, weights=weights, mode=mode, max_params=0, degree=8)
    orders, ws = bench.round_spec(devices, 8, kind=graph, weights=weights)
    base, ref = bench.reference_fixture(a, orders, ws)
    if fixture is None:
        assert ref is None and base == bench.SEED_BASE
        return
    assert ref["name"] == fixture
    assert base == {"c3": 9300, "c4": 9400, "c5": 9500}[fixture.split("_")[2]]
    for seg, exp in ref["expected"].items():
        assert sorted(exp) == list(range(devices))
        assert all(len(v) == len(ref["ranges"][seg]) for v in exp.values())
    a.max_params = 4096  # a cut layout is never the fixture's
    assert bench.reference_fixture(a, orders, ws)[1] is None


def test_app_seed_matches_torch_manual_seed_cpu():
    """Without a GPU runtime the apps' seeding defers to torch.manual_seed (same CPU state)."""
    import torch

    from src.decentralized_client import manual_seed

    torch.manual_seed(11)
    ref = torch.default_generator.get_state()
    torch.manual_seed(12)
    manual_seed(11)
    assert torch.equal(torch.default_generator.get_state(), ref)


def test_default_plan_rows_wider_than_a_tile():
    """A row of more distinct sources than one LDS tile holds (unweighted_fl over 700 clients):
    fp32 rounds get the streamed form, bf16 rounds the wide-row form (groups of 16 rows), rows
    out of reference order one K1 call per row - never a capacity error (host-side plan
    building, no GPU)."""
    import networkx as nx

    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.round import csr_from_lists

    g = nx.complete_graph(700)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(700)]
    rp, col, w = csr_from_lists(orders, [[1 / 700] * 700 for _ in orders])
    rows = np.arange(700, dtype=np.int32)
    p = ops.default_plan(rp, col, w, rows)
    assert ops.round_kernel_name(p) == "k_round_stream" and not p.single_group
    q = ops.default_plan(rp, col, w, rows, bf16=True)
    assert ops.round_kernel_name(q, bf16=True) == "k_round_wide" and not q.single_group
    assert q.spec == {"stream_rows": ops.WIDE_ROWS, "stream_src": 0}
    assert ops.round_kernel_name(ops.plan_from_spec(rp, col, w, rows, q.spec), bf16=True) == "k_round_wide"
    self_first = [[i] + sorted(g.neighbors(i)) for i in range(700)]
    rp2, col2, w2 = csr_from_lists(self_first, [[1 / 700] * 700 for _ in self_first])
    assert isinstance(ops.default_plan(rp2, col2, w2, rows), ops.RowCallPlan)
    assert isinstance(ops.default_plan(rp2, col2, w2, rows, bf16=True), ops.RowCallPlan)


def test_pool_row_addresses_and_cpu_pool_refused():
    """ModelPool.row_ptrs is the row views' data_ptr (padded rows, every segment), and the
    per-call pool path refuses a host pool before touching the library (no GPU needed)."""
    import pytest
    import torch

    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.arena import ModelPool, StateLayout

    lay = StateLayout.from_layout([("w", (1001,), "float32"), ("h", (7,), "bfloat16"), ("n", (), "int64")])
    pool = ModelPool(lay, 5, "cpu")
    for seg, view in (("f32", pool.row_f32), ("b16", pool.row_b16), ("i64", pool.row_i64)):
        assert pool.row_ptrs(seg, [0, 3, 4]) == [view(r).data_ptr() for r in (0, 3, 4)]
    with pytest.raises(ValueError, match="device pool"):
        ops.agg_pool_rows(pool, [0, 1], [0.5, 0.5], 1)
    assert torch.equal(pool.f32, torch.zeros_like(pool.f32))


def test_tune_candidates_by_workload_class():
    """The tuner times only forms that won a workload of the same class: no broadcast form on
    uniform-weight rounds (config 3: 6.2-9.9 ms against 2.0 in BENCH_r05), the measured winners
    on per-operand-weight rounds (config 5 degree centrality)."""
    import bench
    from topology_aware_learning_amd.round import csr_from_lists

    orders, ws = bench.round_spec(64, 8)  # config 3: unweighted
    rp, col, w = csr_from_lists(orders, ws)
    rows = np.arange(len(orders), dtype=np.int32)
    assert ops.rows_uniform(rp, w)
    keys = [k for k, _ in ops.tune_candidates(rp, col, w, rows)]
    assert keys[0] == ("default",) and not any(k[0] == "bcast" for k in keys)
    orders, ws = bench.round_spec(256, 8, kind="sbm", weights="degcent")
    rp, col, w = csr_from_lists(orders, ws)
    rows = np.arange(len(orders), dtype=np.int32)
    assert not ops.rows_uniform(rp, w)
    for bf16 in (False, True):
        keys = [k for k, _ in ops.tune_candidates(rp, col, w, rows, bf16=bf16, mode=ops.MODE_FMA)]
        bc = {k[1:] for k in keys if k[0] == "bcast"}
        assert bc and bc <= set(ops.BCAST_CANDIDATES)


def test_exchange_choice_follows_measured_link_rate():
    """With a measured link rate (bench.py's probe) the 'auto' exchange is the one with the smaller
    predicted time: below the crossover rate the link binds and the transpose's smaller busiest
    pair wins; above it both are HBM-bound and the halo's fewer local bytes win.  Without a rate:
    the busiest-pair byte rule (unchanged)."""
    import bench
    from topology_aware_learning_amd import synth
    from topology_aware_learning_amd.arena import StateLayout
    from topology_aware_learning_amd.distributed import partition_contiguous
    from topology_aware_learning_amd.transposed import choose_exchange, exchange_crossover_gbps, link_model

    cases = [("sbm", 256, "vit_b16", 8), ("random", None, "resnet50", 4), ("random", None, "resnet50", 8),
             ("barbell", 128, "resnet50", 4)]
    flipped = 0
    for kind, nd, model, world in cases:
        lay = StateLayout.from_layout(synth.get_layout(model))
        orders, _ = bench.round_spec(nd or 64 * world, 8, kind=kind)
        owner = partition_contiguous(len(orders), world)
        args = (orders, owner, world, lay.n_f32, lay.n_i64, lay.n_b16)
        x = exchange_crossover_gbps(*args)
        if choose_exchange(*args) != "transpose":
            continue
        if x is None:  # the transpose also moves fewer local bytes (random graph at 8 ranks): any rate
            assert choose_exchange(*args, link_gbps=1e6) == choose_exchange(*args, link_gbps=10.0) == "transpose"
            continue
        assert x > 153.0  # at the assumed 153 GB/s the byte rule's transpose stands
        assert choose_exchange(*args, link_gbps=0.99 * x) == "transpose"
        assert choose_exchange(*args, link_gbps=1.01 * x) == "halo"
        m = link_model(*args, link_gbps=1.01 * x)
        assert m["transpose"]["predicted_ms"] >= 0.9 * m["halo"]["predicted_ms"]
        flipped += 1
    assert flipped >= 2


def test_cosine_plan_streams_column_tensors():
    """K2's plan (host code, no GPU): column tensors with B < 32 (and 16-element runs) are the
    streamed chunks, first, each Ob = 28 // B output blocks (1 from B = 28); the others direct;
    the scratch covers outputs, means and two model slots of norms per pair of a launch."""
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd.arena import StateLayout

    lay = synth.get_layout("resnet50")
    segs = StateLayout.from_layout(lay).param_segments(synth.param_names(lay))
    segs += [(0, 3, 50, 32), (0, 2, 70, 28), (0, 4, 2, 7)]
    plan = ops.build_cosine_plan(segs)
    h = plan.host
    n_seg, n_out, n_staged = int(h[0]), int(h[1]), int(h[3])
    sg = h[4: 4 + 7 * n_seg].reshape(n_seg, 7)
    ch = h[4 + 7 * n_seg:].reshape(-1, 4)
    assert len(ch) == plan.n_chunks
    streamed = [(s, a, i, b) for s, (o, a, i, b) in enumerate(segs) if i > 1 and 1 < b < 32]
    want = sum(-(-a // max(1, 28 // b)) for _, a, _, b in streamed)
    assert n_staged == want
    assert all(ch[:n_staged, 3] == 1) and all(ch[n_staged:, 3] == 0)
    for s, a, i, b in streamed:
        per = max(1, 28 // b) * b
        assert sg[s][6] == per
        rows = ch[:n_staged][ch[:n_staged, 0] == s]
        assert list(rows[:, 1]) == list(range(0, a * b, per)) and rows[:, 2].sum() == a * b
    assert set(ch[n_staged:, 0]) == set(range(n_seg)) - {s for s, *_ in streamed}
    import ctypes

    from topology_aware_learning_amd import _lib

    P64 = ctypes.POINTER(ctypes.c_int64)
    for n_pairs in (1, 8, 40):
        got = _lib.load().tal_cosine_scratch_bytes(h.ctypes.data_as(P64), n_pairs)
        assert got == 4 * (3 * n_out + n_seg) * min(n_pairs, 32)
