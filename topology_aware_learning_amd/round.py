"""A whole aggregation round over a device-resident model pool (K3).

The reference submits one aggregation app per selected client per round
(src/decentralized_app.py:605-641); each reads its neighbors' freshly trained models and the
client's own (self last, :625).  With every model of the round resident in one ``ModelPool``
the round is one sparse mix ``OUT = W . X``: row r of W holds the round's weights for client r
in reference operand order.  ``RoundExecutor`` turns that into a tile plan once per distinct
operand/weight pattern and launches one LDS-tiled kernel per segment, reading each source
model once per column tile instead of once per aggregation that uses it.

Round semantics ("snapshot"): every aggregation of the round reads the models as they were
before the round.  The reference's in-place writes from two threads make
its own round order-dependent; ``sequential=True`` reproduces its single-thread order
(client index order, each call seeing the previous calls' writes) as one K1 call per client.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops
from .arena import ModelPool


def csr_from_lists(orders: Sequence[Sequence[int]], weights: Sequence[Sequence[float]]):
    row_ptr = [0]
    col: List[int] = []
    w: List[float] = []
    for o, ws in zip(orders, weights):
        if len(o) != len(ws) or len(o) == 0:
            raise ValueError("each aggregation needs one weight per operand and >= 1 operand")
        col.extend(int(x) for x in o)
        w.extend(float(x) for x in ws)
        row_ptr.append(len(col))
    return np.array(row_ptr, np.int32), np.array(col, np.int32), np.array(w, np.float64)


class RoundExecutor:
    """Rounds over one pool.

    Double-buffered (the default for device pools, `double_buffer=None`): the executor keeps a
    spare pool of the same shape; each round reads `pool` and writes the spare (rows the round
    does not aggregate are copied across), then the two pools exchange their memory
    (ModelPool.swap_with: one storage pointer exchange per segment, no bytes moved), so the
    models bound to `pool` read the round's output and the spare holds the previous state, the
    next round's destination.  Every plan runs out of place this way, at the out-of-place rate:
    an in-place round costs 5-6 % more on the same destination (profiles/r05/r05p).
    The spare is allocated on the first round: `placement_trials` candidates (at most as many
    as fit in 60 % of the free HBM) are each timed as the round's destination and the fastest is
    kept (where in HBM the written pool sits changes the round time by up to 25 %, see
    arena.select_pool_pair and DESIGN §5 "Pool placement"); `placement` records the times.  With
    no room for a spare the executor falls back to the form below.

    carried_rows=k: rows >= k are not carried into the spare (MultiPool's ghost rows, refreshed
    from their owners before every read).

    double_buffer=False (and pools whose segments are views of a larger storage): single-group
    plans run in place on `pool`, whose placement is the caller's (`calibrated_pool`
    places it before models are bound); multi-group plans write a scratch pool (snapshot
    semantics, placed like the spare) and copy the aggregated rows back."""

    def __init__(self, pool: ModelPool, scratch: Optional[ModelPool] = None, mode: int = ops.MODE_EXACT,
                 placement_trials: int = 4, double_buffer: Optional[bool] = None,
                 carried_rows: Optional[int] = None):
        self.pool = pool
        self.scratch = scratch
        self.mode = mode
        self.placement_trials = placement_trials
        self.placement: Optional[dict] = None
        self._plans: Dict[Tuple, ops.RoundPlan] = {}
        if double_buffer is None:
            double_buffer = scratch is None and pool.device.type == "cuda" and pool.whole_storage()
        self.double_buffer = double_buffer
        # rows a double-buffered round carries into the spare when it does not aggregate them:
        # all (None), or rows below this (a MultiPool pool: its ghost rows are refreshed from their
        # owners before every read, so the stale copies the exchange leaves there are never read)
        self.carried_rows = pool.rows if carried_rows is None else int(carried_rows)
        self.spare: Optional[ModelPool] = None
        self.swaps = 0

    def _new_scratch(self, plan, need: int = 1) -> Optional[ModelPool]:
        """The scratch / spare pool, placed by timing `placement_trials` candidates as the
        round's destination; None when fewer than `need` pools fit in 60 % of the free HBM."""
        lay = self.pool.layout
        make = lambda: ModelPool(lay, self.pool.rows, self.pool.device)  # noqa: E731
        pool_bytes = sum(t.numel() * t.element_size() for _, t, _ in self.pool.segments())
        fit = int(0.6 * torch.cuda.mem_get_info(self.pool.device)[0] // max(1, pool_bytes))
        if fit < need:
            return None
        trials = min(self.placement_trials, fit)
        if trials <= 1:
            return make()
        seg = "b16" if lay.n_b16 else "f32"
        n = lay.n_b16 if lay.n_b16 else lay.n_f32
        run = ops.round_bf16 if lay.n_b16 else ops.round_f32
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        cands, ms = [], []
        for _ in range(trials):
            c = make()
            run(getattr(self.pool, seg), getattr(c, seg), plan, n=n, mode=self.mode)
            s.record()
            for _ in range(2):
                run(getattr(self.pool, seg), getattr(c, seg), plan, n=n, mode=self.mode)
            e.record()
            e.synchronize()
            cands.append(c)
            ms.append(round(s.elapsed_time(e) / 2, 3))
        best = int(np.argmin(ms))
        self.placement = dict(scratch_ms=ms, chosen=best)
        keep = cands[best]
        del cands, c  # (the loop variable still held the last candidate)
        torch.cuda.empty_cache()
        return keep

    def plan(self, orders, weights, out_rows) -> ops.RoundPlan:
        key = (tuple(map(tuple, orders)), tuple(tuple(map(float, w)) for w in weights), tuple(out_rows))
        p = self._plans.get(key)
        if p is None:
            row_ptr, col, w = csr_from_lists(orders, weights)
            p = ops.default_plan(row_ptr, col, w, np.asarray(out_rows, np.int32),
                                 bf16=bool(self.pool.layout.n_b16), mode=self.mode).to(self.pool.device)
            rest = sorted(set(range(self.carried_rows)) - set(int(r) for r in out_rows))
            # rows a double-buffered round does not aggregate: copied into the spare before the swap
            p.rest_rows = torch.as_tensor(rest, dtype=torch.long, device=self.pool.device) if rest else None
            if len(self._plans) > 64:
                self._plans.clear()
            self._plans[key] = p
        return p

    def run(self, orders: Sequence[Sequence[int]], weights: Sequence[Sequence[float]],
            out_rows: Optional[Sequence[int]] = None, sequential: bool = False,
            plan: Optional[ops.RoundPlan] = None) -> None:
        """Aggregate pool rows: out_rows[r] <- sum_k weights[r][k] * pool[orders[r][k]].
        plan: what self.plan(orders, weights, out_rows) returned for these same lists (a caller
        that repeats a round passes it back instead of having the lists hashed again)."""
        if out_rows is None:
            out_rows = list(range(len(orders)))
        if len(orders) == 0:
            return
        lay = self.pool.layout
        if sequential:
            for r, o, w in zip(out_rows, orders, weights):
                if lay.n_f32:
                    ops.agg_f32([self.pool.row_f32(j) for j in o], w, self.pool.row_f32(r), mode=self.mode)
                if lay.n_b16:
                    ops.agg_bf16([self.pool.row_b16(j) for j in o], w, self.pool.row_b16(r), mode=self.mode)
                if lay.n_i64:
                    ops.agg_i64([self.pool.row_i64(j) for j in o], w, self.pool.row_i64(r))
            return
        if plan is None:
            plan = self.plan(orders, weights, out_rows)
        if self.double_buffer:
            if self.spare is None:
                self.spare = self._new_scratch(plan, need=1)
                if self.spare is None:  # no room for a second pool: in place / scratch from now on
                    self.double_buffer = False
            if self.spare is not None:
                self._launch(plan, self.spare)
                if plan.rest_rows is not None:
                    for (_, src, _), (_, dst, _) in zip(self.pool.segments(), self.spare.segments()):
                        dst.index_copy_(0, plan.rest_rows, src.index_select(0, plan.rest_rows))
                # stream-ordered: the next reader of either pool runs behind this round's writes
                self.pool.swap_with(self.spare)
                self.swaps += 1
                return
        # every workgroup stages all sources of its tile before writing: with one group in place
        # is safe; otherwise the round goes through the scratch pool
        if not plan.single_group and self.scratch is None:
            self.scratch = self._new_scratch(plan)
        dst = self.pool if plan.single_group else self.scratch
        self._launch(plan, dst)
        if dst is self.pool:
            return
        idx = torch.as_tensor(list(out_rows), dtype=torch.long, device=self.pool.device)
        for _, t, _ in self.pool.segments():
            src = {id(self.pool.f32): self.scratch.f32, id(self.pool.b16): self.scratch.b16,
                   id(self.pool.i64): self.scratch.i64}[id(t)]
            t.index_copy_(0, idx, src.index_select(0, idx))


    def _launch(self, plan, dst: ModelPool) -> None:
        lay = self.pool.layout
        if lay.n_f32:
            ops.round_f32(self.pool.f32, dst.f32, plan, n=lay.n_f32, mode=self.mode)
        if lay.n_b16:
            ops.round_bf16(self.pool.b16, dst.b16, plan, n=lay.n_b16, mode=self.mode)
        if lay.n_i64:
            ops.round_i64(self.pool.i64, dst.i64, plan, n=lay.n_i64)


def calibrated_pool(layout, rows: int, device, trials: int = 8, degree: int = 8) -> ModelPool:
    """A ModelPool placed where an in-place round runs fast.

    The HBM placement of the pool a round writes changes its time bimodally (config 3: ~2.05
    vs ~2.45-2.6 ms for the same plan; arena.select_pool_pair), and a device-resident driver
    rounds in place on the pool its models are bound to for the whole run.  So the pool is
    chosen once, before binding: up to `trials` candidates (as many as fit in 60 % of the free
    HBM) each time one in-place K3 round of a random `degree`-regular graph over their rows,
    and the fastest is kept (`placement_ms` records the times).  trials <= 1 allocates one."""
    import networkx as nx

    device = torch.device(device)
    make = lambda: ModelPool(layout, rows, device)  # noqa: E731
    row_bytes = 4 * layout.ld_f32 + 2 * layout.ld_b16 + 8 * layout.ld_i64
    if device.type == "cuda":
        trials = min(trials, int(0.6 * torch.cuda.mem_get_info(device)[0] // max(1, rows * row_bytes)))
    if trials <= 1 or rows < 3:
        return make()
    d = min(degree, rows - 1)
    if (d * rows) % 2:
        d -= 1
    g = nx.random_regular_graph(d, rows, seed=0) if d >= 2 else nx.cycle_graph(rows)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(rows)]
    rp, col, w = csr_from_lists(orders, [[1.0 / len(o)] * len(o) for o in orders])
    plan = ops.default_plan(rp, col, w, np.arange(rows, dtype=np.int32), bf16=bool(layout.n_b16)).to(device)
    if not plan.single_group:
        return make()
    seg, n = ("b16", layout.n_b16) if layout.n_b16 else ("f32", layout.n_f32)
    run = ops.round_bf16 if layout.n_b16 else ops.round_f32
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cands, ms = [], []
    for _ in range(trials):
        c = make()
        t = getattr(c, seg)
        run(t, t, plan, n=n)
        s.record()
        for _ in range(2):
            run(t, t, plan, n=n)
        e.record()
        e.synchronize()
        cands.append(c)
        ms.append(round(s.elapsed_time(e) / 2, 3))
    best = int(np.argmin(ms))
    keep = cands[best]  # still all zeros: the rounds mixed zero rows
    keep.placement_ms = dict(in_place_ms=ms, chosen=best)
    del cands, c, t  # (the loop variables still held the last candidate)
    torch.cuda.empty_cache()
    return keep
