"""Host-side aggregation weights of every reference app (float64, reference arithmetic).

The weights are computed with the same Python/NumPy float64 operations, in the same order, as
the reference so that their fp32 rounding (done by the kernel, as torch does for
`python_float * fp32_tensor`) is bit-identical.  Pinned by tests/golden/weights_onehot.json
and tests/golden/tiny_cases.* (reference outputs).
"""
from __future__ import annotations

from typing import Dict, List, Mapping, Sequence, Tuple

import numpy as np


def unweighted(m: int) -> List[float]:
    """unweighted_module_avg / scale_agg: w = 1 / len(neighbor_futures)
    (decentralized_client.py:431, :628)."""
    w = 1 / m
    return [w] * m


def weighted(data_lens: Sequence[int]) -> List[float]:
    """weighted_module_avg: len(train_data_i) / sum (decentralized_client.py:396-397)."""
    return [x / sum(data_lens) for x in data_lens]


def _softmax(x):
    """decentralized_client.py:522-525 (identical at :582-585)."""
    e_x = np.exp(x - np.max(x))
    return e_x / e_x.sum()


def centrality(order: Sequence[int], cent: Mapping[int, float], softmax: bool, coeff: float) -> List[float]:
    """centrality_module_avg (decentralized_client.py:572-593): softmax(coeff * c) or c / sum(c)."""
    ws = [cent[idx] for idx in order]
    if softmax:
        ws = [x * coeff for x in ws]
        return [float(v) for v in _softmax(ws)]
    return [i / sum(ws) for i in ws]


def sim_sign_coeff(order: Sequence[int], self_idx: int, cent: Mapping[int, float],
                   sims: Mapping[int, float], coeff: float) -> float:
    """sim_centrality_module_avg's sign rule (decentralized_client.py:493-516): if the least
    similar neighbor has lower centrality than the aggregating client, coeff = -|coeff|."""
    nbhd: Dict[int, float] = {}
    for idx in order:
        nbhd[idx] = cent[idx]
    client_weight = nbhd[self_idx]
    min_similarity = min(sims, key=sims.get)
    if nbhd[min_similarity] < client_weight:
        return -abs(coeff)
    return abs(coeff)


def sim_centrality(order: Sequence[int], self_idx: int, cent: Mapping[int, float],
                   sims: Mapping[int, float], softmax: bool, coeff: float) -> Tuple[List[float], float]:
    """sim_centrality_module_avg weights (decentralized_client.py:471-533)."""
    coeff = sim_sign_coeff(order, self_idx, cent, sims, coeff)
    ws = [cent[idx] for idx in order]
    if softmax:
        ws = [x * coeff for x in ws]
        return [float(v) for v in _softmax(ws)], coeff
    return [i / sum(ws) for i in ws], coeff
