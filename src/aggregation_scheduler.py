"""Per-round schedules of the aggregation softmax coefficient.

Mirror of the reference's src/aggregation_scheduler.py (same classes, arguments and values).
The driver asks `get_softmax_coeff()` once per aggregation call and calls `step(round_idx)`
once per round (reference decentralized_app.py:638, :642).  Pinned by
tests/golden/schedulers.json (100-round sequences produced by the reference).
"""
from __future__ import annotations

import math


class ScheduledOptim:
    """Warm-up style annealing (reference :6-27; not selectable from the CLI)."""

    def __init__(self, softmax_coeff, n_warmup_steps):
        self.softmax_coeff = softmax_coeff
        self.n_warmup_steps = n_warmup_steps
        self.n_steps = 0

    def _get_softmax_scale(self):
        return min(self.n_steps ** (-0.5), self.n_steps * self.n_warmup_steps ** (-1.5))

    def get_softmax_coeff(self):
        self.softmax_coeff -= 1 * self._get_softmax_scale()
        return self.softmax_coeff

    def step(self, round_idx=None):
        self.n_steps += 1


class BaseScheduler:
    """Constant coefficient (reference :30-44)."""

    def __init__(self, softmax_coeff: float = 100):
        self.softmax_coeff = softmax_coeff

    def get_softmax_coeff(self):
        return self.softmax_coeff

    def step(self, round_idx=None):
        return


class CosineAnnealingWarmRestarts(BaseScheduler):
    """eta_min + (c - eta_min) * (1 + cos(pi * T_cur / T_i)) / 2 with warm restarts
    (reference :47-110).  Like the reference it requires integer T_0 / T_mult."""

    def __init__(self, T_0: int, T_mult: int = 1, eta_min: float = 0.0, last_round: int = -1,
                 softmax_coeff: float = 100):
        if T_0 <= 0 or not isinstance(T_0, int):
            raise ValueError(f"Expected positive integer T_0, but got {T_0}")
        if T_mult < 1 or not isinstance(T_mult, int):
            raise ValueError(f"Expected integer T_mult >= 1, but got {T_mult}")
        if not isinstance(eta_min, (float, int)):
            raise ValueError(f"Expected float or int eta_min, but got {eta_min} of type {type(eta_min)}")
        self.T_0 = T_0
        self.T_i = T_0
        self.T_mult = T_mult
        self.eta_min = eta_min
        self.T_cur = last_round
        self.softmax_coeff = softmax_coeff

    def get_softmax_coeff(self):
        cos_part = (1 + math.cos(math.pi * self.T_cur / self.T_i)) / 2
        return self.eta_min + (self.softmax_coeff - self.eta_min) * cos_part

    def step(self, round_idx=None):
        # As in the reference, a bare step() before any indexed step reads `last_round`
        # before it exists; the driver always passes round_idx.
        if round_idx is None and self.last_round < 0:
            round_idx = 0
        if round_idx is None:
            round_idx = self.last_round + 1
            self.T_cur = self.T_cur + 1
            if self.T_cur >= self.T_i:
                self.T_cur = self.T_cur - self.T_i
                self.T_i = self.T_i * self.T_mult
        elif round_idx < 0:
            raise ValueError(f"Expected non-negative round, but got {round_idx}")
        elif round_idx >= self.T_0:
            if self.T_mult == 1:
                self.T_cur = round_idx % self.T_0
            else:
                n = int(math.log(round_idx / self.T_0 * (self.T_mult - 1) + 1, self.T_mult))
                self.T_cur = round_idx - self.T_0 * (self.T_mult ** n - 1) / (self.T_mult - 1)
                self.T_i = self.T_0 * self.T_mult ** n
        else:
            self.T_i = self.T_0
            self.T_cur = round_idx
        self.last_round = math.floor(round_idx)


class ExponentialScheduler(BaseScheduler):
    """coeff * gamma^t floored at eta_min (reference :113-135)."""

    def __init__(self, gamma: float, eta_min: float = 1, softmax_coeff: float = 100):
        self.gamma = gamma
        self.softmax_coeff = softmax_coeff
        self.eta_min = eta_min

    def get_softmax_coeff(self):
        return self.eta_min if self.softmax_coeff < self.eta_min else self.softmax_coeff

    def step(self, round_idx=None):
        self.softmax_coeff *= self.gamma


class OscilateScheduler(BaseScheduler):
    """+coeff / -coeff, flipping every T_0 rounds (reference :138-162)."""

    def __init__(self, T_0: int, softmax_coeff: float = 100):
        self.T_0 = T_0
        self.sign = 1
        self.cylce_step = 0  # (sic) attribute name kept from the reference
        self.softmax_coeff = softmax_coeff

    def get_softmax_coeff(self):
        return self.sign * self.softmax_coeff

    def step(self, round_idx=None):
        self.cylce_step += 1
        if self.cylce_step == self.T_0:
            self.sign = -self.sign
            self.cylce_step = 0
