"""Gossip matrices / effective neighbors against the reference's values
(tests/golden/gossip.json, from src/effective_neighbors.py via make_golden.py), and the round
as the linear map W . X.  CPU only."""
import json

import networkx as nx
import numpy as np
import pytest
import torch

import oracle
from oracle import reference_alg as ra
from topology_aware_learning_amd import gossip

from conftest import GOLDEN

G = json.loads((GOLDEN / "gossip.json").read_text())


def _graph(case):
    g = nx.Graph()
    g.add_nodes_from(range(case["n"]))
    g.add_edges_from(case["edges"])
    return g


@pytest.mark.parametrize("name", list(G))
def test_gossip_matrix_bits_match_reference(name):
    case = G[name]
    W = gossip.gossip_matrix(_graph(case))
    assert W.dtype == torch.float32
    assert np.array_equal(W.numpy().view(np.uint32), np.array(case["W_bits"], np.uint32))


@pytest.mark.parametrize("name", list(G))
def test_effective_neighbors_match_reference(name):
    case = G[name]
    W = torch.from_numpy(np.array(case["W_bits"], np.uint32).view(np.float32))
    eff = gossip.effective_neighbors(W, 0.9, mode="all", start_at=1)
    assert np.allclose(eff.numpy(), case["eff_all_g09"], rtol=2e-4, atol=1e-5)
    assert abs(float(gossip.effective_neighbors(W, 0.5, mode="mean")) - case["eff_mean_g05"]) <= 2e-4 * abs(case["eff_mean_g05"])
    assert gossip.placement_locations(_graph(case), 0.9, 4) == case["placement4"]


@pytest.mark.parametrize("name", list(G))
def test_round_realizes_gossip_matrix(name):
    """orders_from_matrix(W) is a round in reference operand order whose linear map is W; the
    oracle's sequential fp32 round equals W . X up to the fp32 accumulation bound."""
    case = G[name]
    W = np.array(case["W_bits"], np.uint32).view(np.float32).astype(np.float64)
    orders, weights = gossip.orders_from_matrix(W)
    assert np.array_equal(gossip.round_matrix(orders, weights, len(W)), W)
    for o in orders:
        assert o[:-1] == sorted(o[:-1]) and o[-1] not in o[:-1]
    rng = np.random.default_rng(7)
    X = rng.standard_normal((len(W), 257)).astype(np.float32)
    row_ptr, col, w = ra.round_csr(orders, weights)
    got = oracle.round_f32(X, row_ptr, col, w, np.arange(len(W), dtype=np.int32))
    ref = W @ X.astype(np.float64)
    bound = np.abs(W) @ np.abs(X.astype(np.float64)) * (max(len(o) for o in orders) + 1) * 2.0 ** -24
    assert np.all(np.abs(got - ref) <= bound + 1e-30)


def test_round_matrix_sums_duplicates_and_checks_lengths():
    W = gossip.round_matrix([[1, 1, 0]], [[0.25, 0.25, 0.5]], 2)
    assert W.tolist() == [[0.5, 0.5]]
    with pytest.raises(ValueError):
        gossip.round_matrix([[0, 1]], [[1.0]], 2)
