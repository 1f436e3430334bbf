"""Sharded rounds with a transposed exchange: column blocks of every model instead of whole
neighbor models (the alternative to distributed.ShardedRound's halo exchange).

Aggregation is element-wise over a model's parameters, so a round can be split by columns as
well as by devices.  Rank g keeps its own devices' models (rows, as the halo path does) and,
for one round:
  1. packs its models' column block p (p = 0 .. world-1) into a send buffer, by destination;
  2. one all-to-all: rank g receives column block g of EVERY device's model ([R, b], R = all
     devices, rank-major order);
  3. the K3 kernel runs the whole round on that block (R rows, n/world columns: the same HBM
     bytes as the rank's own rows at full width);
  4. a second all-to-all returns each output block to the model's owner, which unpacks it.
Each element still sums its operands in reference order, so the result is bitwise the halo
path's / the reference's.

Link volume per rank is 2 x (world-1)/world of its own models whatever the topology; the halo
exchange moves every distinct remote neighbor model once per receiving rank, which on a random
expander (the weak-scaling bench graph) is most of the graph.  `choose_exchange` picks the
smaller; every rank computes the same answer from the same inputs, so all ranks issue the same
collectives.  Both all-to-alls use every xGMI link at once (RCCL, one call per segment).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .arena import ModelPool, StateLayout
from .distributed import (_ESIZE, ShardedRound, _pool_segs, build_shard, float_segments, partition_contiguous,
                          run_round_segments, spot_check_row, tune_segment)
from .round import csr_from_lists


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


def column_blocks(n: int, world: int, align: int = 4):
    """Equal column blocks of an n-element segment over `world` ranks: width b (a multiple of
    `align`, so every block row is 16-B aligned), block p = columns [p*b, p*b + w_p), w_p <= b
    (the last blocks may be short or empty)."""
    b = _round_up(-(-n // world), align) if n else 0
    return b, [(p * b, max(0, min(b, n - p * b))) for p in range(world)]


def pack_columns(pool: torch.Tensor, rows: int, blocks, b: int, out: torch.Tensor) -> torch.Tensor:
    """out[p, r, :w_p] = pool[r, block p] for the first `rows` rows (out viewed [world, rows, b])."""
    o = out.view(len(blocks), rows, b)
    for p, (c0, w) in enumerate(blocks):
        if w:
            o[p, :, :w].copy_(pool[:rows, c0: c0 + w])
    return out


def unpack_columns(src: torch.Tensor, rows: int, blocks, b: int, pool: torch.Tensor) -> torch.Tensor:
    """Inverse of pack_columns: pool[r, block p] = src[p, r, :w_p]."""
    s = src.view(len(blocks), rows, b)
    for p, (c0, w) in enumerate(blocks):
        if w:
            pool[:rows, c0: c0 + w].copy_(s[p, :, :w])
    return pool


def positions(owner, world: int):
    """Rank-major device order: own lists per rank, their offsets, and pos[global id] (the row
    of each device in a rank's column-block buffer after the forward all-to-all)."""
    owner = np.asarray(owner)
    own_by_rank = [np.flatnonzero(owner == p).tolist() for p in range(world)]
    base = np.zeros(world + 1, dtype=np.int64)
    base[1:] = np.cumsum([len(o) for o in own_by_rank])
    pos = np.empty(len(owner), dtype=np.int64)
    for p, ids in enumerate(own_by_rank):
        pos[ids] = base[p] + np.arange(len(ids))
    return own_by_rank, base, pos


def exchange_bytes(orders, owner, world: int, n_f32: int, n_i64: int, n_b16: int = 0) -> dict:
    """Largest per-rank link volume of one round (bytes in or out, whichever is larger) for
    each exchange: 'halo' = distinct remote neighbor models, 'transpose' = 2 x (world-1)/world
    of the rank's own models."""
    owner = np.asarray(owner)
    row = 4 * n_f32 + 2 * n_b16 + 8 * n_i64
    specs = [build_shard(orders, [[1.0] * len(o) for o in orders], owner, r, world) for r in range(world)]
    halo = max(max(len(s.halo), sum(len(v) for v in s.send.values())) for s in specs) * row
    own = max(len(s.own) for s in specs)
    return dict(halo=int(halo), transpose=int(2 * own * row * (world - 1) // world))


def choose_exchange(orders, owner, world: int, n_f32: int, n_i64: int, n_b16: int = 0) -> str:
    """'transpose' when it moves clearly fewer bytes than the halo (random expanders at 4+
    ranks), else 'halo' (rings, cliques, community graphs; 2 ranks)."""
    if world < 2:
        return "halo"
    b = exchange_bytes(orders, owner, world, n_f32, n_i64, n_b16)
    return "transpose" if b["transpose"] < 0.9 * b["halo"] else "halo"


@dataclass
class _ColSeg:
    n: int                  # elements per model
    b: int                  # block width (row stride of the work buffers)
    blocks: list            # (first column, width) per rank
    send: torch.Tensor      # [world, own, b]  my models' blocks, by destination rank
    work_in: torch.Tensor   # [R, b]           block `rank` of every device's model (rank-major)
    work_out: torch.Tensor  # [R, b]           the round's output for that block
    back: torch.Tensor      # [world, own, b]  my models' output blocks, by source rank


class TransposedRound:
    """One rank's device-resident round with the transposed exchange (module docstring).  The
    models update in place in pool_a: the send buffer holds the inputs before any output lands
    (snapshot semantics)."""

    def __init__(self, layout: StateLayout, orders, weights, rank: int, world: int, device,
                 mode: int = ops.MODE_EXACT, owner: Optional[np.ndarray] = None, group=None,
                 tune: bool = False, transport: str = "device"):
        self.layout = layout
        self.transport = transport  # "host": all-to-alls staged through host memory (gloo rehearsal)
        self.device = torch.device(device)
        self.mode = mode
        self.group = group
        self.rank, self.world = rank, world
        n_dev = len(orders)
        owner = partition_contiguous(n_dev, world) if owner is None else np.asarray(owner, np.int32)
        self.own_by_rank, self.base, self.pos = positions(owner, world)
        self.own = self.own_by_rank[rank]
        self.local_rows = len(self.own)
        self.rows_all = n_dev
        inv = np.empty(n_dev, dtype=np.int64)
        inv[self.pos] = np.arange(n_dev)
        self.orders_pos = [[int(self.pos[j]) for j in orders[int(inv[q])]] for q in range(n_dev)]
        self.weights_pos = [[float(x) for x in weights[int(inv[q])]] for q in range(n_dev)]
        self.pool_a = ModelPool(layout, self.local_rows, self.device)
        self.segs: Dict[str, _ColSeg] = {}
        for g, n, dt in (("f32", layout.n_f32, torch.float32), ("b16", layout.n_b16, torch.bfloat16),
                         ("i64", layout.n_i64, torch.int64)):
            if not n:
                continue
            b, blocks = column_blocks(n, world)

            def z(*shape, dt=dt):
                return torch.zeros(*shape, dtype=dt, device=self.device)

            self.segs[g] = _ColSeg(n, b, blocks, z(world, self.local_rows, b), z(n_dev, b), z(n_dev, b),
                                   z(world, self.local_rows, b))
        self.w_me = {g: s.blocks[rank][1] for g, s in self.segs.items()}
        rp, col, w = csr_from_lists(self.orders_pos, self.weights_pos)
        out_rows = np.arange(n_dev, dtype=np.int32)
        tg = tune_segment(layout)
        f = self.segs.get(tg)
        if tune and f is not None and self.w_me[tg]:
            self.plan = ops.tune_plan(rp, col, w, out_rows, f.work_in, f.work_out, n=self.w_me[tg], mode=mode)
        else:
            self.plan = ops.build_plan(rp, col, w, out_rows, dense=0 if layout.n_b16 else -1).to(self.device)
        self.plans = {"round": self.plan}
        self.staged_sources = self.plan.staged_rows()
        self.exchange_kind = "transpose"
        self._events: list = []
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=group)

    # phases: step() runs them in order; the virtual-rank GPU test interleaves ranks between them
    def pack(self) -> None:
        pools = _pool_segs(self.pool_a)
        for g, s in self.segs.items():
            pack_columns(pools[g], self.local_rows, s.blocks, s.b, s.send)

    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits) -> None:
        if self.transport == "host":
            o = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_to_all_single(o, inp.view(-1).cpu(), out_splits, in_splits, group=self.group)
            out.view(-1).copy_(o)
        else:
            dist.all_to_all_single(out.view(-1), inp.view(-1), out_splits, in_splits, group=self.group)

    def forward_exchange(self) -> None:
        for s in self.segs.values():
            self._all_to_all(s.work_in, s.send, [len(o) * s.b for o in self.own_by_rank],
                             [self.local_rows * s.b] * self.world)

    def compute(self) -> None:
        run_round_segments(self.layout, {g: s.work_in for g, s in self.segs.items()},
                           {g: s.work_out for g, s in self.segs.items()}, self.plan, self.mode, n_of=self.w_me)

    def backward_exchange(self) -> None:
        for s in self.segs.values():
            self._all_to_all(s.back, s.work_out, [self.local_rows * s.b] * self.world,
                             [len(o) * s.b for o in self.own_by_rank])

    def unpack(self) -> None:
        pools = _pool_segs(self.pool_a)
        for g, s in self.segs.items():
            unpack_columns(s.back, self.local_rows, s.blocks, s.b, pools[g])

    def step(self, timed: bool = False) -> None:
        """One round: pack, all-to-all, K3 on this rank's column block, all-to-all back, unpack.
        With timed=True the kernels are bracketed by events (kernel_ms())."""
        self.pack()
        self.forward_exchange()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if timed else None
        if ev:
            ev[0].record()
        self.compute()
        if ev:
            ev[1].record()
            self._events.append(ev)
        self.backward_exchange()
        self.unpack()

    def kernel_ms(self) -> List[float]:
        out = [e[0].elapsed_time(e[1]) for e in self._events]
        self._events = []
        return out

    def own_rows(self) -> ModelPool:
        return self.pool_a

    @property
    def kernel_bytes(self) -> int:
        """Algorithmic HBM bytes of one round's K3 launch (staged sources + written rows)."""
        return sum(_ESIZE[g] * self.w_me[g] for g, _ in float_segments(self.layout)) * (
            self.staged_sources + self.rows_all)

    @property
    def link_bytes(self) -> int:
        """Bytes this rank receives over the links per round (both all-to-alls)."""
        r = 0
        for g, s in self.segs.items():
            r += _ESIZE[g] * s.b * ((self.rows_all - self.local_rows) + self.local_rows * (self.world - 1))
        return r

    def spot_check(self) -> bool:
        """After a step: the first row of this rank's column block == K1 on its operands'
        blocks (bitwise)."""
        segs = {g: s for g, s in self.segs.items() if g != "i64"}
        ops_ = {g: [s.work_in[j] for j in self.orders_pos[0]] for g, s in segs.items()}
        return spot_check_row(self.layout, ops_, self.weights_pos[0], {g: s.work_out[0] for g, s in segs.items()},
                              self.mode, n_of=self.w_me)


def make_round(layout: StateLayout, orders, weights, rank: int, world: int, device, exchange: str = "auto",
               mode: int = ops.MODE_EXACT, owner: Optional[np.ndarray] = None, group=None, tune: bool = False,
               transport: str = "device"):
    """This rank's sharded round with the given exchange ('halo' | 'transpose' | 'auto');
    transport 'host' stages the exchange through host memory (gloo rehearsal runs only)."""
    owner = partition_contiguous(len(orders), world) if owner is None else np.asarray(owner, np.int32)
    if exchange == "auto":
        exchange = choose_exchange(orders, owner, world, layout.n_f32, layout.n_i64, layout.n_b16)
    cls = {"halo": ShardedRound, "transpose": TransposedRound}[exchange]
    r = cls(layout, orders, weights, rank, world, device, mode=mode, owner=owner, group=group, tune=tune,
            transport=transport)
    r.exchange_kind = exchange
    return r
