"""GPU: the persistent round kernels' tile walk (tal_set_tile_walk) changes only the order in
which HBM is touched.  Every walk must write every output column of every row exactly as the
default walk does: the output pool is prefilled with a different pattern before each run, so a
tile a walk skips (or writes twice from a stale register) shows up.  The default walk itself is
pinned against the oracle by test_gpu_kernels / test_gpu_bcast; here one oracle check per form
anchors the comparison."""
import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import ops
from topology_aware_learning_amd.round import csr_from_lists

pytestmark = pytest.mark.gpu

SPECS = [
    {"c4": 64, "lds": 81920, "dense": 0},                               # persistent (config 3 default)
    {"c4": 32, "lds": 81920, "dense": 0},                               # narrow c4 32
    {"c4": 16, "lds": 81920, "dense": 0},                               # narrow c4 16
    {"c4": 16, "lds": 163840, "dense": 0, "bcast": 8, "bcwg": 2},       # broadcast 8 x 2
    {"c4": 32, "lds": 163840, "dense": 0, "bcast": 16, "bcwg": 1},      # two-chunk broadcast
]
WALKS = [0, 2, 3, 16, 64]


def _round(graph, weighted):
    g = {"regular": lambda: nx.random_regular_graph(8, 64, seed=0),
         "sbm": lambda: nx.stochastic_block_model([32] * 4, [[0.45 if a == b else 0.01 for b in range(4)]
                                                            for a in range(4)], seed=0)}[graph]()
    orders = [sorted(g.neighbors(i)) + [i] for i in sorted(g.nodes)]
    if weighted:
        cent = nx.degree_centrality(g)
        ws = [ra.centrality_weights(o, cent, True, 10.0) for o in orders]
    else:
        ws = [ra.unweighted_weights(len(o)) for o in orders]
    return orders, ws


@pytest.fixture(autouse=True)
def _reset_walk():
    yield
    ops.set_tile_walk(1)


def test_walk_argument_checked():
    for bad in (-1, 65):
        with pytest.raises(ops._lib.TalError):
            ops.set_tile_walk(bad)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("weighted", [False, True], ids=["unweighted", "degcent"])
@pytest.mark.parametrize("graph", ["regular", "sbm"])
@pytest.mark.parametrize("si", range(len(SPECS)), ids=[str(i) for i in range(len(SPECS))])
def test_walks_bitwise_default(cuda, si, graph, weighted, dtype):
    spec = SPECS[si]
    orders, ws = _round(graph, weighted)
    rows = len(orders)
    rp, col, w = csr_from_lists(orders, ws)
    out_rows = np.arange(rows, dtype=np.int32)
    try:
        plan = ops.plan_from_spec(rp, col, w, out_rows, spec).to(cuda)
    except ops._lib.TalError as exc:  # a form this round's shape cannot take
        pytest.skip(f"{spec}: {exc}")
    # 9,500 float4 (even: bf16 pools take the 16-B staging lanes) + a 3-element tail; the tile
    # count is a multiple of no grid size
    n = 4 * 9500 + 3
    ld = 38016
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    gen = torch.Generator(device="cpu").manual_seed(5)
    src = (torch.randn(rows, ld, generator=gen) * 3).to(tdt).to(cuda)
    run = ops.round_f32 if dtype == "f32" else ops.round_bf16
    mode = ops.MODE_EXACT if dtype == "f32" else ops.MODE_FMA  # bf16: the FMA tolerance run's mode
    outs = []
    for k, walk in enumerate([1] + WALKS):
        ops.set_tile_walk(walk)
        dst = torch.full((rows, ld), float(k + 1) * 0.5, dtype=tdt, device=cuda)
        run(src, dst, plan, n=n, mode=mode)
        outs.append(dst[:, :n].cpu())
    torch.cuda.synchronize()
    if dtype == "f32":  # the default walk against the oracle, so the comparison has an anchor
        x = src[:, :n].cpu().numpy()
        for r in (0, rows // 2, rows - 1):
            exp = oracle.agg_f32([x[j] for j in orders[r]], ws[r])
            assert np.array_equal(exp.view(np.uint32), outs[0][r].numpy().view(np.uint32)), r
    ref = outs[0].view(torch.int16 if dtype == "bf16" else torch.int32)
    for walk, o in zip(WALKS, outs[1:]):
        got = o.view(torch.int16 if dtype == "bf16" else torch.int32)
        bad = (got != ref).any(dim=1).nonzero().flatten().tolist()
        assert not bad, f"walk {walk}: rows {bad[:8]} differ from the default walk"
