"""K2's streamed column chunks (round 6): a column tensor [A, I, B] with B < 32 runs as two
kernels that walk i in 16-element steps through LDS - every model's norms (torch's FMA chains),
then each pair's products (the four streams' level-0 runs pushed into their cascades every 64
elements) - k_cos_col_norms / k_cos_col_prods; the other tensors run the direct form.  Bitwise
the oracle (torch's CPU order, oracle/cosine_oracle.c) at the edges: column tensors with B from
2 to 31 (output blocks per chunk 14 .. 1, the tensor's last chunk partial), I below 4 (only the
remainder), I not a multiple of the step (a partial last step) or of 4 (row_sum's remainder),
streams whose length is not a multiple of the run (a partial last run), 1,024 and 16,400
elements (the cascade's second and third levels), B = 32 (the direct form); row tensors of every
size class; segments starting at every 4-byte offset inside a 16-byte chunk; pairs sharing one
`a` and pairs that do not; more pairs than one launch takes; a whole ResNet-50 model.
Reference: cosine_similarity, /root/reference/src/decentralized_client.py:661-681.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle
from topology_aware_learning_amd import ops, synth
from topology_aware_learning_amd.arena import StateLayout

pytestmark = pytest.mark.gpu

# (A, I, B): column kind B > 1, row kind B == 1
_SHAPES = [
    (64, 3, 9), (61, 3, 9),            # conv1: 28 slabs per chunk, the last chunk partial
    (8, 512, 9), (3, 511, 9),          # one slab per chunk (4,608 floats: the capacity); 511: a partial run
    (6, 256, 9), (5, 128, 9), (9, 64, 9),
    (4, 100, 2), (3, 37, 31), (2, 148, 31),  # B 2 / 31; 148 x 31 = 4,588
    (3, 4609, 1), (2, 513, 9),         # one element past the capacity: the direct form
    (5, 4608, 1), (7, 2048, 1), (33, 512, 1),
    (40, 7, 1), (9, 8, 1), (11, 13, 1), (6, 100, 1), (3, 1030, 1),
    (2, 1024, 9), (1, 16400, 3), (3, 1001, 5), (2, 70, 28), (5, 33, 14), (4, 2, 7), (3, 50, 32),
]


def _models(rng, segs, n):
    total = max(o + a * i * b for o, a, i, b in segs)
    return [rng.standard_normal(total).astype(np.float32) for _ in range(n)]


def _check(cuda, rows, segs, a_idx, b_idx):
    dev = [torch.from_numpy(r).to(cuda) for r in rows]
    plan = ops.build_cosine_plan(segs)
    got = ops.cosine([dev[j] for j in a_idx], [dev[j] for j in b_idx], plan).cpu().numpy()
    for k, (ja, jb) in enumerate(zip(a_idx, b_idx)):
        ref = np.float32(oracle.cosine_model(rows[ja], rows[jb], segs))
        assert got[k].view(np.uint32) == ref.view(np.uint32), (segs, k, got[k], ref)


@pytest.mark.parametrize("shape", _SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("mis", [0, 1, 3])
def test_staged_shapes_vs_oracle(cuda, shape, mis):
    """One tensor per plan, its segment starting `mis` floats past a 16-byte boundary."""
    a, i, b = shape
    segs = [(mis, a, i, b)]
    rng = np.random.default_rng(a * 1000 + i * 10 + b + mis)
    rows = _models(rng, segs, 4)
    _check(cuda, rows, segs, [0, 0, 0], [1, 2, 3])
    _check(cuda, rows, segs, [1, 2, 3], [0, 0, 0])  # each pair a different `a`


def test_staged_all_shapes_one_plan(cuda):
    """Every shape above in one model (staged and direct chunks in one launch pair), odd offsets."""
    segs, off = [], 5
    for a, i, b in _SHAPES:
        segs.append((off, a, i, b))
        off += a * i * b + 3
    rows = _models(np.random.default_rng(11), segs, 5)
    _check(cuda, rows, segs, [0, 0, 0, 0], [1, 2, 3, 4])


def test_staged_more_pairs_than_one_launch(cuda):
    segs = [(0, 8, 64, 9), (4608, 16, 72, 1), (4608 + 1152, 30, 1, 1)]
    rows = _models(np.random.default_rng(3), segs, 36)
    _check(cuda, rows, segs, [0] * 35, list(range(1, 36)))
    _check(cuda, rows, segs, list(range(18)), list(range(18, 36)))  # 18 pairs, each its own a


def test_staged_resnet50_model(cuda):
    """A whole ResNet-50 parameter set (161 tensors: 3 x 3 convs streamed, 1 x 1 convs and 1-D
    parameters direct) for 3 pairs, against the oracle."""
    lay = synth.get_layout("resnet50")
    layout = StateLayout.from_layout(lay)
    segs = layout.param_segments(synth.param_names(lay))
    flat = []
    for s in (9300, 9301, 9302, 9303):
        sd = synth.synth_state_dict(lay, s)
        flat.append(torch.cat([v.reshape(-1) for (n, _, d), v in zip(lay, sd.values()) if d == "float32"]).numpy())
    _check(cuda, flat, segs, [0, 0, 0], [1, 2, 3])


def test_streamed_and_direct_from_two_threads(cuda):
    """A plan with streamed and direct chunks forks its direct chunks onto the device's side
    stream and joins them back through per-call events: two host threads, each on its own torch
    stream, calling K2 at once get the oracle's values."""
    import threading

    segs, off = [], 1
    for a, i, b in [(8, 512, 9), (33, 512, 1), (61, 3, 9), (40, 7, 1), (30, 1, 1)]:
        segs.append((off, a, i, b))
        off += a * i * b + 5
    rows = _models(np.random.default_rng(21), segs, 5)
    dev = [torch.from_numpy(r).to(cuda) for r in rows]
    plan = ops.build_cosine_plan(segs)
    ref = [np.float32(oracle.cosine_model(rows[0], rows[j], segs)) for j in (1, 2, 3, 4)]
    got, errs = {}, []

    def run(k):
        try:
            s = torch.cuda.Stream(cuda)
            with torch.cuda.stream(s):
                for _ in range(5):
                    out = ops.cosine([dev[0]] * 4, dev[1:], plan)
                s.synchronize()
            got[k] = out.cpu().numpy()
        except Exception as exc:  # pragma: no cover - reported below
            errs.append(exc)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs
    for k in range(2):
        assert [int(v.view(np.uint32)) for v in got[k]] == [int(v.view(np.uint32)) for v in ref]
