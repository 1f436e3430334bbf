"""TEST INFRASTRUCTURE — the reference's CPU aggregation loop restated with the same torch ops.

This is the "port" CPU baseline bench.py times on the GPU box's host cores (the reference
itself cannot travel there).  It performs exactly the reference's operations:

    decentralized_client.py:399-411   partial = w * torch.clone(value); avg[name] (+)= partial
    decentralized_client.py:413       model.load_state_dict(avg)   -> copy_ per entry

so it costs what the reference costs (clone + mul + add_ per operand, copy_ per entry).
tests/test_oracle_golden.py checks it bit-for-bit against the reference's own outputs.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Mapping, Sequence

import torch


def aggregate(state_dicts: Sequence[Mapping[str, torch.Tensor]], weights: Sequence[float]):
    avg: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    with torch.no_grad():
        for sd, w in zip(state_dicts, weights):
            for name, value in sd.items():
                partial = w * torch.clone(value)
                if name not in avg:
                    avg[name] = partial
                else:
                    avg[name] += partial
    return avg


def load_into(target: Mapping[str, torch.Tensor], avg: Mapping[str, torch.Tensor]) -> None:
    """load_state_dict's per-entry copy_ (dtype-converting: fp32 -> int64 truncates)."""
    with torch.no_grad():
        for name, t in target.items():
            t.copy_(avg[name])


def aggregate_call(state_dicts, weights, target) -> None:
    load_into(target, aggregate(state_dicts, [float(w) for w in weights]))
