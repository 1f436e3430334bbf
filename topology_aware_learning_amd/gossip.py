"""Gossip matrices and the effective-number-of-neighbors analysis.

A snapshot round is linear: OUT = W . X with W[i, j] = the weight row i gives model j.  This
module builds that dense W from a round's (orders, weights) -- the CSR the K3 kernels run --
and the other way round, so the batched round can be validated against W . X and the
reference's gossip processes can run on the device pool.  It also restates the reference's
topology analysis (reference src/effective_neighbors.py, itself adapted from the
"topology-in-decentralized-learning" code):

  gossip_matrix            Topology.gossip_matrix                 effective_neighbors.py:36-45
  random_walk_covariance   random_walk_covariance_static          effective_neighbors.py:482-500
  effective_neighbors      effective_number_of_neighbors (static) effective_neighbors.py:467-479
  placement_locations      get_n_placement_locations              effective_neighbors.py:531-566

These are host-side analysis helpers (n x n, n <= a few hundred); the aggregation itself stays
on the HIP kernels.
"""
from __future__ import annotations

from math import sqrt
from typing import List, Sequence, Tuple

import networkx as nx
import numpy as np
import scipy.linalg
import torch


def round_matrix(orders: Sequence[Sequence[int]], weights: Sequence[Sequence[float]],
                 n_cols: int | None = None) -> np.ndarray:
    """Dense float64 W of one snapshot round: W[i, j] = sum of row i's weights on model j."""
    n_rows = len(orders)
    n_cols = n_cols if n_cols is not None else 1 + max(max(o) for o in orders)
    W = np.zeros((n_rows, n_cols), np.float64)
    for i, (o, w) in enumerate(zip(orders, weights)):
        if len(o) != len(w):
            raise ValueError(f"row {i}: {len(o)} operands but {len(w)} weights")
        for j, x in zip(o, w):
            W[i, j] += float(x)
    return W


def orders_from_matrix(W) -> Tuple[List[List[int]], List[List[float]]]:
    """The round that applies W in reference operand order (ascending neighbors, then self):
    row i lists the j != i with W[i, j] != 0, then i itself (always, even at weight 0, as the
    reference's aggregating client is always an operand: decentralized_app.py:625)."""
    W = np.asarray(W, dtype=np.float64)
    orders, weights = [], []
    for i in range(W.shape[0]):
        nb = [int(j) for j in np.flatnonzero(W[i]) if j != i]
        orders.append(nb + [i])
        weights.append([float(W[i, j]) for j in nb] + [float(W[i, i])])
    return orders, weights


def gossip_matrix(graph: nx.Graph, weight: float | None = None) -> torch.Tensor:
    """Metropolis-style gossip matrix of the reference (float32, as there):
    W[i, j] = 1 / (max(deg i, deg j) + 1) for each neighbor j (or `weight`), and the diagonal
    takes the rest of the row, 1 - sum_j W[i, j]."""
    n = graph.number_of_nodes()
    nodes = sorted(graph.nodes)
    if nodes != list(range(n)):
        raise ValueError("graph nodes must be 0..n-1")
    deg = {i: len(list(graph.neighbors(i))) for i in nodes}
    m = torch.zeros([n, n])
    for i in nodes:
        for j in graph.neighbors(i):
            m[i, j] = 1 / (max(deg[i], deg[j]) + 1) if weight is None else weight
        m[i, i] = 1 - m[i, :].sum()
    return m


def random_walk_covariance(W: torch.Tensor, gamma: float, start_at: int = 1) -> torch.Tensor:
    """Asymptotic E[x x^T] of x <- W (sqrt(gamma) x + noise) for a static W: through the
    eigen-decomposition when W is symmetric, else a discrete Lyapunov solve."""
    if W.allclose(W.T):
        lam, Q = torch.linalg.eigh(W)
        num = lam.square() if start_at == 1 else 1
        return (Q * (num / (1 - gamma * lam.square()))) @ Q.T
    rhs = W @ W.T if start_at == 1 else torch.eye(len(W), dtype=W.dtype)
    out = scipy.linalg.solve_discrete_lyapunov(sqrt(gamma) * W.cpu().numpy(), rhs.cpu().numpy())
    return torch.from_numpy(out).to(W.device)


def effective_neighbors(W: torch.Tensor, gamma: float, mode: str = "mean", start_at: int = 1):
    """Effective number of neighbors 1 / (1 - gamma) / Var[x_i] (per worker: mode "all";
    averaged variance: "mean"; largest variance: "worst")."""
    var = random_walk_covariance(W, gamma, start_at=start_at).diag()
    if mode == "mean":
        return 1 / (1 - gamma) / var.mean()
    if mode == "worst":
        return 1 / (1 - gamma) / var.max()
    if mode == "all":
        return 1 / (1 - gamma) / var
    raise ValueError("Unknown mode")


def placement_locations(graph: nx.Graph, gamma: float, n: int) -> List[int]:
    """n nodes spread over the ranking of the per-node effective neighbors averaged over
    start_at = 0..len-1 (the reference evaluates gamma = 0.9 whatever `gamma` is given)."""
    W = gossip_matrix(graph)
    acc = torch.zeros(len(graph))
    for i in range(len(graph)):
        acc += effective_neighbors(W, gamma=0.9, mode="all", start_at=i)
    acc /= len(graph)
    interval = len(graph) // n
    picks = list(range(0, interval * n, interval))
    _, ind = torch.sort(acc)
    return torch.index_select(ind, 0, torch.tensor(picks)).tolist()
