"""Pin the oracle (C restatement + numpy host logic + torch CPU port) against golden vectors
generated from the reference itself (tests/golden/make_golden.py).  CPU only."""
import functools
import hashlib
import json

import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from oracle import torch_path
from topology_aware_learning_amd import synth

from conftest import GOLDEN

TINY = json.loads((GOLDEN / "tiny_cases.json").read_text())
TINYZ = np.load(GOLDEN / "tiny_cases.npz")
CENT = {k: {int(i): v for i, v in d.items()} for k, d in TINY["centrality"].items()}
LAYOUT = [(n, tuple(s), d) for n, s, d in TINY["layout"]]


def case_weights(case):
    """The weight vector the reference app used, restated by the oracle."""
    order, M = case["order"], case["M"]
    fn = case["fn"]
    if fn in ("unweighted_module_avg",):
        return ra.unweighted_weights(M), order
    if fn == "weighted_module_avg":
        return ra.weighted_weights(case["data_lens"]), order
    if fn == "scale_agg":
        return [1 / M], [order[-1]]
    if fn == "test_agg":
        return None, order
    cent = CENT[case["centrality_metric"]]
    if fn == "centrality_module_avg":
        return ra.centrality_weights(order, cent, case["softmax"], case["softmax_coeff"]), order
    sims = {idx: c for idx, c in zip(order[:-1], case["cosine"])}
    w, _ = ra.sim_centrality_weights(order, order[-1], cent, sims, case["softmax"], case["softmax_coeff"])
    return w, order


def inputs(ci, M):
    return [{n: TINYZ[f"c{ci}_in{i}_{n}"] for n, _, _ in LAYOUT} for i in range(M)]


def bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype == np.float32:
        return np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
            a[~np.isnan(a)].view(np.uint32), b[~np.isnan(b)].view(np.uint32))
    return np.array_equal(a, b)


@pytest.mark.parametrize("case", TINY["cases"], ids=lambda c: f"{c['case']}-{c['fn']}-M{c['M']}")
def test_c_oracle_matches_reference_apps(case):
    ci, M = case["case"], case["M"]
    w, order = case_weights(case)
    ins = inputs(ci, M)
    for name, _, dt in LAYOUT:
        ref = TINYZ[f"c{ci}_out_{name}"]
        if w is None:  # test_agg: untouched self model
            assert bits_equal(ins[-1][name], ref)
            continue
        xs = [ins[-1][name]] if case["fn"] == "scale_agg" else [x[name] for x in ins]
        got = oracle.agg_f32(xs, w) if dt == "float32" else oracle.agg_i64(xs, w)
        assert bits_equal(got.reshape(ref.shape), ref), (name, case["fn"])


BF16 = json.loads((GOLDEN / "bf16_cases.json").read_text())
BF16Z = np.load(GOLDEN / "bf16_cases.npz")
BF16_CENT = {k: {int(i): v for i, v in d.items()} for k, d in BF16["centrality"].items()}


def bf16_case_weights(case):
    order, M, fn = case["order"], case["M"], case["fn"]
    if fn == "unweighted_module_avg":
        return ra.unweighted_weights(M)
    if fn == "weighted_module_avg":
        return ra.weighted_weights(case["data_lens"])
    if fn == "scale_agg":
        return [1 / M]
    return ra.centrality_weights(order, BF16_CENT[case["centrality_metric"]], case["softmax"], case["softmax_coeff"])


@pytest.mark.parametrize("case", BF16["cases"], ids=lambda c: f"{c['case']}-{c['fn']}-M{c['M']}")
def test_c_oracle_bf16_matches_reference_apps(case):
    """bf16 models through the reference's own loop (tests/golden/bf16_cases.*, generated from
    the reference): the exact-mode bf16 restatement reproduces every output bit."""
    ci, M = case["case"], case["M"]
    w = bf16_case_weights(case)
    for name, _, dt in BF16["layout"]:
        ins = [BF16Z[f"c{ci}_in{i}_{name}"] for i in range(M)]
        ref = BF16Z[f"c{ci}_out_{name}"]
        xs = [ins[-1]] if case["fn"] == "scale_agg" else ins
        if dt == "bfloat16":
            got = oracle.agg_bf16([x.reshape(-1) for x in xs], w, exact=True)
        else:
            got = oracle.agg_i64([x.reshape(-1) for x in xs], w)
        assert np.array_equal(got.reshape(ref.shape), ref), (name, case["fn"])


def test_bf16_fixture_covers_rounding_cases():
    """The fixture exercises bf16 rounding: results differ from fp32-accumulate-then-round."""
    differs = 0
    for case in BF16["cases"]:
        if case["fn"] != "unweighted_module_avg" or case["M"] < 9:
            continue
        ci, M = case["case"], case["M"]
        w = bf16_case_weights(case)
        ins = [BF16Z[f"c{ci}_in{i}_fc.weight"].reshape(-1) for i in range(M)]
        differs += int(np.sum(oracle.agg_bf16(ins, w, exact=True) != oracle.agg_bf16(ins, w, exact=False)))
    assert differs > 0


@pytest.mark.parametrize("case", [c for c in TINY["cases"] if c["fn"] != "test_agg"][::3],
                         ids=lambda c: f"{c['case']}-{c['fn']}")
def test_torch_port_matches_reference_apps(case):
    ci, M = case["case"], case["M"]
    w, _ = case_weights(case)
    ins = inputs(ci, M)
    sds = [{k: torch.from_numpy(v.copy()) for k, v in d.items()} for d in ins]
    if case["fn"] == "scale_agg":
        sds = [sds[-1]]
    target = {k: v.clone() for k, v in sds[-1].items()}
    torch_path.aggregate_call(sds, w, target)
    for name, _, _ in LAYOUT:
        assert bits_equal(target[name].numpy(), TINYZ[f"c{ci}_out_{name}"]), name


def test_truncation_fixture_values():
    """9 x 1000 at w=1/9 -> 999 through the reference."""
    hit = 0
    for case in TINY["cases"]:
        if case["fn"] == "unweighted_module_avg" and case["M"] == 9 and case["case"] % 5 != 4 and case["case"] % 7 != 6:
            assert int(TINYZ[f"c{case['case']}_out_bn.num_batches_tracked"]) == 999
            hit += 1
    assert hit >= 1


@pytest.mark.parametrize("case", [c for c in TINY["cases"] if c["fn"] == "sim_centrality_module_avg"],
                         ids=lambda c: f"{c['case']}")
def test_cosine_restatement_matches_reference(case):
    ci, M = case["case"], case["M"]
    ins = inputs(ci, M)
    pnames = synth.param_names(LAYOUT)
    for j, ref in enumerate(case["cosine"]):
        got = ra.cosine_similarity([ins[-1][n] for n in pnames], [ins[j][n] for n in pnames])
        assert abs(got - ref) < 1e-5, (j, got, ref)


@pytest.mark.parametrize("case", [c for c in TINY["cases"] if c["fn"] == "sim_centrality_module_avg"],
                         ids=lambda c: f"{c['case']}")
def test_cosine_oracle_bitwise_reference(case):
    """The C oracle's cosine (torch's CPU reduction order, cosine_oracle.c) equals the
    reference's cosine_similarity values bit for bit."""
    from topology_aware_learning_amd.arena import StateLayout

    ci, M = case["case"], case["M"]
    ins = inputs(ci, M)
    layout = StateLayout.from_layout(LAYOUT)
    segs = layout.param_segments(synth.param_names(LAYOUT))
    flat = [np.concatenate([ins[j][n].reshape(-1) for n, _, d in LAYOUT if d == "float32"]) for j in range(M)]
    for j, ref in enumerate(case["cosine"]):
        got = oracle.cosine_model(flat[-1], flat[j], segs)
        assert got.view(np.uint32) == np.float32(ref).view(np.uint32), (j, got, ref)


def test_onehot_weights_bitwise():
    for rec in json.loads((GOLDEN / "weights_onehot.json").read_text()):
        cent = {k: {int(i): v for i, v in d.items()} for k, d in
                json.loads((GOLDEN / "centrality.json").read_text())[rec["graph"]].items()}
        w = ra.centrality_weights(rec["order"], cent[rec["metric"]], rec["softmax"], rec["coeff"])
        assert [int(x) for x in np.asarray(w, np.float32).view(np.uint32)] == rec["w_f32_bits"], rec["node"]


def test_sequential_round_fixture():
    meta = json.loads((GOLDEN / "round_4ring.json").read_text())
    z = np.load(GOLDEN / "round_4ring.npz")
    names = [n for n, _, d in meta["layout"] if d == "float32"]
    pool = np.stack([np.concatenate([z[f"in{i}_{n}"].reshape(-1) for n in names]) for i in range(4)])
    orders = meta["orders"]
    ws = [ra.unweighted_weights(len(o)) for o in orders]
    seq = ra.sequential_round_f32(pool, orders, ws, range(4))
    ref = np.stack([np.concatenate([z[f"seq{i}_{n}"].reshape(-1) for n in names]) for i in range(4)])
    assert bits_equal(seq, ref)
    # snapshot semantics differ from the reference's in-place order (SURVEY finding 5)
    row_ptr, col, w = ra.round_csr(orders, ws)
    snap = oracle.round_f32(pool, row_ptr, col, w, np.arange(4))
    assert bits_equal(snap[0], ref[0]) and not bits_equal(snap[1:], ref[1:])


BIG = json.loads((GOLDEN / "big_sha256.json").read_text())
LAYOUTS = json.loads((GOLDEN / "layouts.json").read_text())


@pytest.mark.parametrize("idx", range(len(BIG["cases"])))
def test_c_oracle_full_size_sha256(idx):
    case = BIG["cases"][idx]
    lay = [(n, tuple(s), d) for n, s, d in LAYOUTS[case["model"]]]
    cent = {k: {int(i): v for i, v in d.items()} for k, d in BIG["centrality"].items()}
    order = case["order"]
    if case["fn"] == "unweighted_module_avg":
        w = ra.unweighted_weights(len(order))
    elif case["fn"] == "weighted_module_avg":
        w = ra.weighted_weights(case["data_lens"])
    else:
        w = ra.centrality_weights(order, cent[case["centrality_metric"]], case["softmax"], case["softmax_coeff"])
    sds = [synth.synth_state_dict(lay, s) for s in case["seeds"]]
    for name, _, dt in lay:
        xs = [sd[name].numpy().reshape(-1) for sd in sds]
        out = oracle.agg_f32(xs, w) if dt == "float32" else oracle.agg_i64(xs, w)
        assert hashlib.sha256(out.tobytes()).hexdigest() == case["sha256"][name], name


RING32 = json.loads((GOLDEN / "big_round_resnet18_ring32.json").read_text())


@functools.lru_cache(maxsize=1)
def ring32_pools():
    """BASELINE config 2's inputs at full size (ResNet-18, 32 devices): [32, n] fp32 / int64
    pools, each row the model's entries of that dtype concatenated in state_dict order."""
    from topology_aware_learning_amd import synth

    lay = [(n, tuple(s), d) for n, s, d in json.loads((GOLDEN / "layouts.json").read_text())["resnet18"]]
    f, i = [], []
    for seed in RING32["seeds"]:
        sd = synth.synth_state_dict(lay, seed)
        f.append(np.concatenate([v.reshape(-1).numpy() for v in sd.values() if v.dtype == torch.float32]))
        i.append(np.concatenate([v.reshape(-1).numpy() for v in sd.values() if v.dtype == torch.int64]))
    return np.stack(f), np.stack(i)


def test_oracle_full_size_ring32_round():
    """The C oracle's snapshot round over BASELINE config 2 at full size (32 x 11.2 M params)
    reproduces the reference's outputs (sha256 per output model, make_golden.py big_round)."""
    f, i = ring32_pools()
    orders = [r["order"] for r in RING32["rows"]]
    rp, col, w = ra.round_csr(orders, [ra.unweighted_weights(len(o)) for o in orders])
    out = oracle.round_f32(f, rp, col, w, np.arange(32))
    iout = oracle.round_i64(i, rp, col, w, np.arange(32))
    for r, row in enumerate(RING32["rows"]):
        assert hashlib.sha256(out[r].tobytes()).hexdigest() == row["sha256_f32"], r
        assert hashlib.sha256(iout[r].tobytes()).hexdigest() == row["sha256_i64"], r


NEAR = json.loads((GOLDEN / "near_ties.json").read_text())
NEARZ = np.load(GOLDEN / "near_ties.npz")


@pytest.mark.parametrize("case", NEAR["cases"], ids=lambda c: f"{c['case']}-{c['kind']}")
def test_cosine_oracle_near_ties(case):
    """Near-tied similarities (fp32 ties, 1-4 ulp gaps, fp32 order != exact order): the C
    oracle reproduces the reference's values bitwise, and with them its least-similar pick and
    the aggregation output (oracle weights + oracle aggregation)."""
    from topology_aware_learning_amd.arena import StateLayout

    lay = [(n, tuple(s), d) for n, s, d in NEAR["layout"]]
    layout = StateLayout.from_layout(lay)
    segs = layout.param_segments(synth.param_names(lay))
    ci, order = case["case"], case["order"]
    M = len(order)
    ins = [{n: NEARZ[f"c{ci}_in{i}_{n}"] for n, _, _ in lay} for i in range(M)]
    flat = [np.concatenate([ins[j][n].reshape(-1) for n, _, d in lay if d == "float32"]) for j in range(M)]
    sims = {}
    for j, ref in enumerate(case["cosine"]):
        got = oracle.cosine_model(flat[-1], flat[j], segs)
        assert got.view(np.uint32) == np.float32(ref).view(np.uint32), (j, got, ref)
        sims[order[j]] = float(got)
    cent = {int(i): v for i, v in NEAR["centrality"]["degree"].items()}
    w, _ = ra.sim_centrality_weights(order, order[-1], cent, sims, NEAR["softmax"], NEAR["softmax_coeff"])
    for n, _, d in lay:
        if d != "float32":
            continue
        out = oracle.agg_f32([ins[j][n].reshape(-1) for j in range(M)], w)
        assert np.array_equal(out.view(np.uint32), NEARZ[f"c{ci}_out_{n}"].reshape(-1).view(np.uint32)), n


def test_config5_fixture_pins_every_entry_group():
    """BASELINE config 5's reference digests (make_golden.py full_c5, round 4): fp32 unweighted,
    fp32 degree-centrality softmax and bf16 unweighted each cover EVERY entry group of every one
    of the 256 output models (rounds 1-3 pinned one group of the latter two), and the groups
    tile the ViT-B/16 segments without gaps."""
    import json

    fx = json.loads((GOLDEN / "full_round_c5_vit_sbm256.json").read_text())
    ng = len(fx["groups"])
    assert ng >= 8 and fx["groups"][0]["start"] == 0
    for a, b in zip(fx["groups"], fx["groups"][1:]):
        assert b["start"] == a["end"]
    kinds = {(r["dtype"], r["fn"]) for r in fx["runs"]}
    assert kinds == {("f32", "unweighted_module_avg"), ("f32", "centrality_module_avg"), ("bf16", "unweighted_module_avg")}
    for r in fx["runs"]:
        assert r["groups"] == list(range(ng)), (r["dtype"], r["fn"])
        assert len(r["sha256"]) == 256
        assert all(sorted(int(k) for k in row) == list(range(ng)) and all(len(v) == 64 for v in row.values())
                   for row in r["sha256"])
