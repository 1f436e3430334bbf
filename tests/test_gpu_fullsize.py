"""BASELINE configs 3, 4 and 5 at full size against the REFERENCE's own outputs.

The fixtures (tests/golden/make_golden.py full_c3 / full_c4 / full_c5) hold the sha256 of every
output model of one snapshot round computed by the reference's aggregation apps
(/root/reference/src/decentralized_client.py:418-448 unweighted_module_avg, :553-612
centrality_module_avg; driven per client as decentralized_app.py:605-641 does) on the seeded
synthetic inputs of topology_aware_learning_amd/synth.py.  Here the same inputs are generated
on the GPU (synth.fill_rows_torch, bitwise the host generator), one round runs through the K3
kernels for every plan form the tuner can pick, and every output row is hashed:

  config 3  random 8-regular graph, 64 x ResNet-50, M = 9          (the benchmark's round)
  config 4  barbell(60, 8), 128 x ResNet-50, M = 3..61              (K3c clique blocks)
  config 5  SBM 8 x 32, 256 x ViT-B/16, M ~ 17                      (K3n narrow tiles),
            per entry group, every group of every output model (round 4; rounds 1-3 pinned one
            group of the latter two): fp32 unweighted, fp32 degree-centrality softmax
            (per-operand weights), bf16 EXACT (the reference's bf16 ops)
"""
from __future__ import annotations

import hashlib
import json
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import reference_alg as ra
from topology_aware_learning_amd import ops, synth
from topology_aware_learning_amd import weights as tw
from topology_aware_learning_amd.arena import ModelPool, StateLayout

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _fixture(name: str) -> dict:
    return json.loads((GOLDEN / name).read_text())


def row_digests(seg: torch.Tensor, n_rows: int, ranges, view=torch.int32):
    """sha256 of seg[r, a:b] for every row r < n_rows and (a, b) in ranges (bit patterns as
    `view`), rows copied to the host one at a time and hashed on a thread pool."""
    lo = min(a for a, _ in ranges)
    hi = max(b for _, b in ranges)
    out = [[None] * len(ranges) for _ in range(n_rows)]
    pending = []

    def h(buf, a, b):
        return hashlib.sha256(memoryview(buf[a:b])).hexdigest()

    with ThreadPoolExecutor(16) as ex:
        for r in range(n_rows):
            host = seg[r, lo:hi].view(view).cpu().numpy()
            for k, (a, b) in enumerate(ranges):
                pending.append((r, k, ex.submit(h, host, a - lo, b - lo)))
            if len(pending) > 64:
                for rr, kk, f in pending:
                    out[rr][kk] = f.result()
                pending = []
        for rr, kk, f in pending:
            out[rr][kk] = f.result()
    return out


def _pools(cuda, lay, seeds, dtype="float32"):
    layout = StateLayout.from_layout(lay)
    pin = ModelPool(layout, len(seeds), cuda)
    pout = ModelPool(layout, len(seeds), cuda)
    if dtype == "float32":
        synth.fill_rows_torch(pin.f32, lay, seeds)
    else:
        synth.fill_rows_torch(pin.b16, lay, seeds, dtype="bfloat16")
    if layout.n_i64:
        synth.fill_rows_torch(pin.i64, lay, seeds, dtype="int64")
    torch.cuda.synchronize(cuda)
    return layout, pin, pout


def _plan(orders, ws, spec, bf16=False):
    rp, col, w = ra.round_csr(orders, ws)
    out_rows = np.arange(len(orders), dtype=np.int32)
    if spec is None:
        return ops.default_plan(rp, col, w, out_rows, bf16=bf16)
    return ops.plan_from_spec(rp, col, w, out_rows, spec)


# ------------------------------------------------------------------------------------------
# configs 3 and 4: ResNet-50, fp32 + int64 segments, every output model
# ------------------------------------------------------------------------------------------
_RESNET = {}


def _resnet_round(cuda, name):
    if name not in _RESNET:
        _RESNET.clear()
        torch.cuda.empty_cache()
        fx = _fixture(name)
        lay = synth.get_layout("resnet50")
        layout, pin, pout = _pools(cuda, lay, fx["seeds"])
        _RESNET[name] = (fx, layout, pin, pout)
    return _RESNET[name]


def _check_resnet_round(cuda, name, spec):
    fx, layout, pin, pout = _resnet_round(cuda, name)
    orders = [r["order"] for r in fx["rows"]]
    plan = _plan(orders, [ra.unweighted_weights(len(o)) for o in orders], spec).to(cuda)
    pout.f32.fill_(float("nan"))
    pout.i64.fill_(-1)
    ops.round_f32(pin.f32, pout.f32, plan, n=layout.n_f32)
    ops.round_i64(pin.i64, pout.i64, plan, n=layout.n_i64)
    torch.cuda.synchronize(cuda)
    f = row_digests(pout.f32, len(orders), [(0, layout.n_f32)])
    i = row_digests(pout.i64, len(orders), [(0, layout.n_i64)], view=torch.int64)
    bad = [r for r, row in enumerate(fx["rows"])
           if f[r][0] != row["sha256_f32"] or i[r][0] != row["sha256_i64"]]
    assert not bad, f"{len(bad)} output models differ from the reference, first rows {bad[:8]}"


@pytest.mark.parametrize("spec", [None, {"c4": 64, "lds": 81920, "dense": 0}, {"c4": 128, "lds": 163840, "dense": 0},
                                  {"c4": 128, "lds": 81920, "dense": 0}, {"c4": 32, "lds": 81920, "dense": 0},
                                  {"c4": 16, "lds": 81920, "dense": 0}, {"c4": 64, "lds": 81920, "dense": 8},
                                  {"stream_rows": 64, "stream_src": 0}, {"reg": 1}])
def test_config3_full_round_vs_reference(cuda, spec):
    """The benchmark's round (64-device random 8-regular graph, ResNet-50, M = 9) at full size:
    all 64 output models bitwise the reference's, for every plan form the tuner can pick."""
    _check_resnet_round(cuda, "full_round_c3_resnet50_rr64.json", spec)


@pytest.mark.parametrize("spec", [None, {"c4": 128, "lds": 163840, "dense": 0}, {"c4": 64, "lds": 163840, "dense": 8},
                                  {"c4": 16, "lds": 81920, "dense": 0}, {"reg": 1}])
def test_config4_full_round_vs_reference(cuda, spec):
    """barbell(60, 8), 128 x ResNet-50 at full size: the K3c clique blocks with their attached
    bridge rows (default plan) and the LDS-tiled forms, all 128 output models bitwise the
    reference's."""
    _check_resnet_round(cuda, "full_round_c4_resnet50_barbell.json", spec)


# ------------------------------------------------------------------------------------------
# config 5: ViT-B/16 on the SBM, digests per entry group
# ------------------------------------------------------------------------------------------
def _c5_weights(fx, run, orders):
    if run["fn"] == "unweighted_module_avg":
        return [ra.unweighted_weights(len(o)) for o in orders]
    import networkx as nx

    sizes = [32] * 8
    p = [[14 / 31 if a == b else 2 / 224 for b in range(8)] for a in range(8)]
    cent = nx.degree_centrality(nx.stochastic_block_model(sizes, p, seed=0))
    return [tw.centrality(o, cent, run["softmax"], run["softmax_coeff"]) for o in orders]


def _check_c5(cuda, dtype, fn, spec, mode=ops.MODE_EXACT):
    fx = _fixture("full_round_c5_vit_sbm256.json")
    run = next(r for r in fx["runs"] if r["dtype"] == dtype and r["fn"] == fn)
    orders = fx["orders"]
    lay = synth.vit_b16_layout() if dtype == "f32" else synth.as_bf16(synth.vit_b16_layout())
    torch.cuda.empty_cache()
    layout, pin, pout = _pools(cuda, lay, fx["seeds"], "float32" if dtype == "f32" else "bfloat16")
    plan = _plan(orders, _c5_weights(fx, run, orders), spec, bf16=dtype == "bf16").to(cuda)
    if dtype == "f32":
        ops.round_f32(pin.f32, pout.f32, plan, n=layout.n_f32, mode=mode)
        seg, view = pout.f32, torch.int32
    else:
        ops.round_bf16(pin.b16, pout.b16, plan, n=layout.n_b16, mode=mode)
        seg, view = pout.b16, torch.int16
    torch.cuda.synchronize(cuda)
    del pin
    gids = run["groups"]
    ranges = [(fx["groups"][g]["start"], fx["groups"][g]["end"]) for g in gids]
    got = row_digests(seg, len(orders), ranges, view=view)
    del pout, seg
    torch.cuda.empty_cache()
    bad = [(r, g) for r in range(len(orders)) for k, g in enumerate(gids)
           if got[r][k] != run["sha256"][r][str(g)]]
    assert not bad, f"{len(bad)} (model, entry group) outputs differ from the reference, first {bad[:8]}"


@pytest.mark.parametrize("spec", [None, {"c4": 32, "lds": 163840, "dense": 0}, {"reg": 1}])
def test_config5_full_round_vs_reference(cuda, spec):
    """SBM-256 x ViT-B/16 fp32 at full size (88.6 GB of models): every (output model, entry
    group) bitwise the reference's unweighted_module_avg."""
    _check_c5(cuda, "f32", "unweighted_module_avg", spec)


@pytest.mark.parametrize("spec", [None, {"reg": 1}, {"c4": 16, "lds": 163840, "dense": 0},
                                  {"c4": 16, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 2},
                                  {"c4": 32, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 1}])
def test_config5_degree_centrality_vs_reference(cuda, spec):
    """The per-operand-weight form (centrality_module_avg, degree, softmax coeff 10) of config 5
    at full width: every entry group of every output model bitwise the reference's, through the
    default plan (the broadcast form, 8 wavefronts x 2), K3r, the pairs form and the 16 x 2
    broadcast form, and the two-chunk broadcast form (c4 = 32, one workgroup per CU)."""
    _check_c5(cuda, "f32", "centrality_module_avg", spec)


def test_config5_bf16_exact_vs_reference(cuda):
    """Config 5 on bf16 models (model.to(torch.bfloat16)) in EXACT mode: every entry group of
    every output model bitwise the reference's own bf16 arithmetic."""
    _check_c5(cuda, "bf16", "unweighted_module_avg", None)


@pytest.mark.parametrize("fn,spec", [("unweighted_module_avg", None),
                                     ("centrality_module_avg", None),
                                     ("centrality_module_avg", {"reg": 1}),
                                     ("centrality_module_avg", {"c4": 16, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 2}),
                                     ("centrality_module_avg", {"c4": 32, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 1})])
def test_config5_bf16_fma_full_width_within_bound(cuda, fn, spec):
    """Config 5's bf16 tolerance run (FMA: fp32 accumulation, one rounding) at full width: all
    256 output models x all 86.6 M columns within the SURVEY §8(a) bound
        |got - ref| <= 2^-8 |ref| + M_r 2^-24 sum_i |w_i x_i|
    against an fp32 EXACT round of the same bf16-valued inputs (the fp32 round kernel that
    test_config5_full_round_vs_reference pins to the reference's sha256), column chunk by
    column chunk; the default plan (per-operand weights: the broadcast form) and K3r."""
    fx = _fixture("full_round_c5_vit_sbm256.json")
    orders = fx["orders"]
    run = dict(fn=fn, softmax=True, softmax_coeff=10.0)
    ws = _c5_weights(fx, run, orders)
    lay = synth.as_bf16(synth.vit_b16_layout())
    torch.cuda.empty_cache()
    layout, pin, pout = _pools(cuda, lay, fx["seeds"], "bfloat16")
    n = layout.n_b16
    plan = _plan(orders, ws, spec, bf16=True) if spec is not None else None
    if plan is None:
        rp, col, w = ra.round_csr(orders, ws)
        plan = ops.default_plan(rp, col, w, np.arange(len(orders), dtype=np.int32), bf16=True, mode=ops.MODE_FMA)
    plan = plan.to(cuda)
    ops.round_bf16(pin.b16, pout.b16, plan, n=n, mode=ops.MODE_FMA)
    rp, col, w = ra.round_csr(orders, ws)
    plan32 = ops.default_plan(rp, col, w, np.arange(len(orders), dtype=np.int32)).to(cuda)
    m_r = torch.tensor([len(o) for o in orders], dtype=torch.float32, device=cuda)[:, None]
    chunk = 1 << 23
    worst = 0.0
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        x32 = pin.b16[:, c0:c1].float().contiguous()
        ref = torch.empty_like(x32)
        ops.round_f32(x32, ref, plan32, n=c1 - c0)
        mag = torch.empty_like(x32)
        ops.round_f32(x32.abs_(), mag, plan32, n=c1 - c0)  # weights are positive: sum |w x|
        bound = 2.0 ** -8 * ref.abs() + m_r * 2.0 ** -24 * mag
        err = (pout.b16[:, c0:c1].float() - ref).abs()
        ratio = float((err / bound.clamp_min(1e-38)).max())
        worst = max(worst, ratio)
        assert ratio <= 1.0, (c0, ratio)
        del x32, ref, mag, bound, err
    del pin, pout
    torch.cuda.empty_cache()
    assert worst > 0.0  # the comparison saw real rounding
