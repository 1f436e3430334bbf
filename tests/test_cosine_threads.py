"""cosine_similarity on tensors with >= 32768 outputs (ViT-B/16's patch embedding: 196,608),
whose per-tensor mean torch computes as a two-pass parallel sum in an order set by the intra-op
thread count (oracle/cosine_oracle.c par_sum; tal_agg.h K2).  Pinned by the reference's own
cosine_similarity at 1..64 threads (tests/golden/cosine_threads.json, make_golden.py
cosine_threads).  Reference: src/decentralized_client.py:661-681."""
import json

import numpy as np
import pytest
import torch

import oracle
from topology_aware_learning_amd import synth
from topology_aware_learning_amd.arena import StateLayout

from _models import cos_pair_state
from conftest import GOLDEN

FIX = json.loads((GOLDEN / "cosine_threads.json").read_text())
VIT = synth.vit_b16_layout()


def _case_inputs(case):
    lay = VIT if case["entries"] is None else [VIT[i] for i in case["entries"]]
    a, b = cos_pair_state(VIT, case["seed_a"], case["seed_b"], case["entries"], case["mix"])
    layout = StateLayout.from_layout(lay)
    segs = layout.param_segments([n for n, _, _ in lay])
    flat = [np.concatenate([v.reshape(-1).numpy() for v in sd.values()]) for sd in (a, b)]
    return flat, segs


def _ids(c):
    return f"{'all' if c['entries'] is None else len(c['entries'])}-{c['seed_a']}-{c['seed_b']}-{c['mix']}"


def test_fixture_exercises_the_thread_count():
    """At least one case gives different reference values at different thread counts (the
    fixture pins the parallel order, not only the serial one)."""
    assert any(len(set(c["bits"].values())) > 2 for c in FIX["cases"])
    assert max(int(t) for c in FIX["cases"] for t in c["bits"]) >= 64


@pytest.mark.parametrize("case", FIX["cases"], ids=_ids)
def test_oracle_cosine_threads_bitwise_reference(case):
    flat, segs = _case_inputs(case)
    for t, bits in case["bits"].items():
        got = oracle.cosine_model(flat[0], flat[1], segs, threads=int(t))
        assert int(got.view(np.uint32)) == bits, (t, got, np.uint32(bits).view(np.float32))


def test_oracle_cosine_threads_below_grain_is_serial():
    """Tensors under 32768 outputs (every reference CNN's) do not depend on the thread count."""
    rng = np.random.default_rng(5)
    a, b = rng.standard_normal(512 * 9 * 9, dtype=np.float32), rng.standard_normal(512 * 9 * 9, dtype=np.float32)
    segs = [(0, 512, 9, 9)]  # a ResNet conv: 512 x 9 outputs (4608), each over 9 inputs
    base = oracle.cosine_model(a, b, segs, threads=1)
    for t in (2, 8, 64):
        assert oracle.cosine_model(a, b, segs, threads=t).view(np.uint32) == base.view(np.uint32)


@pytest.mark.parametrize("case", FIX["cases"], ids=_ids)
def test_host_k2_cosine_threads_bitwise_reference(case):
    """The library's host K2 (tal_host_cosine, what a process without a GPU runs) at every
    thread count the fixture holds: the reference's value bit for bit."""
    from topology_aware_learning_amd import ops

    flat, segs = _case_inputs(case)
    a, b = (torch.from_numpy(x) for x in flat)
    for t, bits in case["bits"].items():
        plan = ops.build_cosine_plan(segs, threads=int(t))
        got = ops.host_cosine([a, a], [b, a], plan).numpy()
        assert int(got[0].view(np.uint32)) == bits, (t, got[0], np.uint32(bits).view(np.float32))
        assert got[1] == np.float32(1.0) or abs(float(got[1]) - 1.0) < 1e-6


@pytest.mark.skipif(torch.cuda.is_available(), reason="the host K2 runs only without a GPU")
def test_interface_cosine_follows_process_threads_on_host():
    """src.decentralized_client.cosine_similarity with no GPU visible (the host K2) follows the
    calling process's torch thread count, as the reference's call does."""
    import torch.nn as nn

    import src.decentralized_client as dc

    case = next(c for c in FIX["cases"] if c["entries"] == [1] and len(set(c["bits"].values())) > 2)
    a, b = cos_pair_state(VIT, case["seed_a"], case["seed_b"], case["entries"], case["mix"])

    def holder(sd):
        m = nn.Module()
        for k, v in enumerate(sd.values()):
            m.register_parameter(f"p{k}", nn.Parameter(v.clone(), requires_grad=False))
        return m

    ma, mb = holder(a), holder(b)
    saved = torch.get_num_threads()
    try:
        for t in ("1", "3", "5", "8"):
            torch.set_num_threads(int(t))
            got = np.float32(dc.cosine_similarity(ma, mb))
            assert int(got.view(np.uint32)) == case["bits"][t], t
    finally:
        torch.set_num_threads(saved)


@pytest.mark.gpu
@pytest.mark.parametrize("case", FIX["cases"], ids=_ids)
def test_k2_cosine_threads_bitwise_reference(case):
    from topology_aware_learning_amd import ops

    flat, segs = _case_inputs(case)
    dev = torch.device("cuda", 0)
    a, b = (torch.from_numpy(x).to(dev) for x in flat)
    for t, bits in case["bits"].items():
        plan = ops.build_cosine_plan(segs, threads=int(t))
        got = ops.cosine([a, a], [b, a], plan).cpu().numpy()
        assert int(got[0].view(np.uint32)) == bits, (t, got[0], np.uint32(bits).view(np.float32))
        assert got[1] == np.float32(1.0) or abs(float(got[1]) - 1.0) < 1e-6


@pytest.mark.gpu
def test_interface_cosine_follows_process_threads():
    """src.decentralized_client.cosine_similarity (the reference's call surface) uses the
    calling process's torch thread count, as the reference's own call does."""
    import torch.nn as nn

    import src.decentralized_client as dc

    case = next(c for c in FIX["cases"] if c["entries"] == [1] and len(set(c["bits"].values())) > 2)
    a, b = cos_pair_state(VIT, case["seed_a"], case["seed_b"], case["entries"], case["mix"])
    dev = torch.device("cuda", 0)

    def holder(sd):
        m = nn.Module()
        for k, v in enumerate(sd.values()):
            m.register_parameter(f"p{k}", nn.Parameter(v.clone().to(dev), requires_grad=False))
        return m

    ma, mb = holder(a), holder(b)
    saved = torch.get_num_threads()
    try:
        for t in ("1", "3", "5", "8"):
            torch.set_num_threads(int(t))
            got = np.float32(dc.cosine_similarity(ma, mb))
            assert int(got.view(np.uint32)) == case["bits"][t], t
    finally:
        torch.set_num_threads(saved)
