"""TEST INFRASTRUCTURE — numpy restatement of the host-side logic on the aggregation path.

Each function cites the reference line it restates (msakarvadia/topology_aware_learning @
2025-06-14).  It is written literally (same float64 operations in the same order) so that the
fp32-rounded weights are bit-identical; tests/test_oracle_golden.py pins it against weights
extracted from the reference (tests/golden/weights_onehot.json) and the app outputs
(tests/golden/tiny_cases.*).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np


def unweighted_weights(m: int) -> List[float]:
    # decentralized_client.py:431  w = 1 / len(neighbor_futures)
    w = 1 / m
    return [w] * m


def weighted_weights(data_lens: Sequence[int]) -> List[float]:
    # decentralized_client.py:396-397
    return [x / sum(data_lens) for x in data_lens]


def _softmax(x):
    # decentralized_client.py:522-525 / :582-585
    e_x = np.exp(x - np.max(x))
    return e_x / e_x.sum()


def centrality_weights(order: Sequence[int], cent: Dict[int, float], softmax: bool, coeff: float):
    # decentralized_client.py:572-593
    weights = [cent[idx] for idx in order]
    if softmax:
        weights = [x * coeff for x in weights]
        return list(_softmax(weights))
    return [i / sum(weights) for i in weights]


def sim_centrality_weights(order: Sequence[int], self_idx: int, cent: Dict[int, float],
                           sims: Dict[int, float], softmax: bool, coeff: float):
    # decentralized_client.py:471-533; sims = cosine(self, neighbor) for every non-self operand
    weights = []
    nbhd = {}
    for idx in order:
        weights.append(cent[idx])
        nbhd[idx] = cent[idx]
    client_weight = nbhd[self_idx]
    min_similarity = min(sims, key=sims.get)
    if nbhd[min_similarity] < client_weight:
        coeff = -abs(coeff)
    else:
        coeff = abs(coeff)
    if softmax:
        weights = [x * coeff for x in weights]
        return list(_softmax(weights)), coeff
    return [i / sum(weights) for i in weights], coeff


def cosine_similarity(params_a: Sequence[np.ndarray], params_b: Sequence[np.ndarray]) -> float:
    """decentralized_client.py:661-681 in fp32 like torch: per parameter, 1-D tensors get a
    trailing unit dim, nn.CosineSimilarity(dim=1, eps=1e-6) = sum over dim 1 of
    (x / max(|x|, eps)) * (y / max(|y|, eps)) with the norms computed first (an fp32 norm that
    overflows is inf and zeroes its row, as in torch), mean over the remaining elements, then
    the average over parameters."""
    total = 0.0
    with np.errstate(over="ignore", invalid="ignore"):
        for a, b in zip(params_a, params_b):
            a = np.asarray(a, dtype=np.float32)
            b = np.asarray(b, dtype=np.float32)
            if a.ndim < 2:
                a = a.reshape(-1, 1)
                b = b.reshape(-1, 1)
            na = np.maximum(np.sqrt((a * a).sum(axis=1, keepdims=True, dtype=np.float32)), np.float32(1e-6))
            nb = np.maximum(np.sqrt((b * b).sum(axis=1, keepdims=True, dtype=np.float32)), np.float32(1e-6))
            total += float(((a / na) * (b / nb)).sum(axis=1, dtype=np.float32).astype(np.float64).mean())
    return total / len(params_a)


def round_csr(neighbors: Sequence[Sequence[int]], weights: Sequence[Sequence[float]]):
    """One round's operand lists as CSR (row r = device r; operands in reference order:
    neighbor_idxs then self, decentralized_app.py:616-629)."""
    row_ptr = [0]
    col: List[int] = []
    w: List[float] = []
    for ops, ws in zip(neighbors, weights):
        col.extend(ops)
        w.extend(ws)
        row_ptr.append(len(col))
    return np.array(row_ptr, np.int32), np.array(col, np.int32), np.array(w, np.float64)


def sequential_round_f32(pool: np.ndarray, orders: Sequence[Sequence[int]], weights, rows: Sequence[int]):
    """In-place round processed in client order with one aggregation thread: each call reads
    the pool as left by the previous calls (decentralized_app.py:605-641 + client.py:413)."""
    from oracle import agg_f32

    pool = pool.copy()
    for r, order, w in zip(rows, orders, weights):
        pool[r] = agg_f32([pool[j] for j in order], w)
    return pool
