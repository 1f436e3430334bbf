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


def positions_own_first(owner, world: int, rank: int):
    """TransposedRound's row order on rank `rank`: its own models first, then every other
    rank's in ascending rank order (each rank's models contiguous, in id order).  Own rows
    first means the forward all-to-all receives into one contiguous tail of the work buffer and
    the rank's own column block never passes through RCCL: it is packed straight into the
    head rows and unpacked straight from them.  Returns (own lists per rank, first row of each
    rank's models, pos[global id])."""
    owner = np.asarray(owner)
    own_by_rank = [np.flatnonzero(owner == p).tolist() for p in range(world)]
    order = [rank] + [p for p in range(world) if p != rank]
    row_base = np.zeros(world, dtype=np.int64)
    pos = np.empty(len(owner), dtype=np.int64)
    r = 0
    for p in order:
        row_base[p] = r
        pos[own_by_rank[p]] = r + np.arange(len(own_by_rank[p]))
        r += len(own_by_rank[p])
    return own_by_rank, row_base, pos


def exchange_bytes(orders, owner, world: int, n_f32: int, n_i64: int, n_b16: int = 0) -> dict:
    """Link volumes of one round for each exchange.  'halo' / 'transpose': the largest per-rank
    volume (bytes in or out, whichever is larger): distinct remote neighbor models, resp.
    2 x (world-1)/world of the rank's own models.  'halo_link' / 'transpose_link': the largest
    volume on one directed GPU pair (each pair has its own xGMI link): the halo's biggest
    per-peer message, resp. 2 x own / world (both all-to-alls spread every rank's models evenly
    over its links)."""
    owner = np.asarray(owner)
    row = 4 * n_f32 + 2 * n_b16 + 8 * n_i64
    specs = [build_shard(orders, [[1.0] * len(o) for o in orders], owner, r, world) for r in range(world)]
    halo = max(max(len(s.halo), sum(len(v) for v in s.send.values())) for s in specs) * row
    halo_link = max([len(v) for s in specs for v in list(s.send.values()) + list(s.recv.values())] or [0]) * row
    own = max(len(s.own) for s in specs)
    return dict(halo=int(halo), transpose=int(2 * own * row * (world - 1) // world),
                halo_link=int(halo_link),
                transpose_link=int(-(-2 * own * row // world)) if world > 1 else 0)  # one rank: no link


HBM_GBPS = 8000.0       # MI355X HBM3E peak per GPU (MI355X_MICROARCH.md)
XGMI_LINK_GBPS = 153.0  # one xGMI link per GPU pair, one direction (7 links per GPU)


def link_model(orders, owner, world: int, n_f32: int, n_i64: int, n_b16: int = 0,
               link_gbps: float = XGMI_LINK_GBPS) -> dict:
    """DESIGN §6's bound per exchange kind, for rank-level reporting next to a measured round:
    local HBM bytes of the busiest rank (halo: its staged sources - own and received - read once
    plus its own rows written; transpose: the round over every model's column block plus the
    packing and unpacking of its own models), the busiest directed GPU pair's bytes, each over
    its rate (HBM 8 TB/s; one GPU pair's link: `link_gbps`, the assumed 153 GB/s unless a run
    measured it - bench.py's link probe), predicted_ms = the larger, and which binds."""
    owner = np.asarray(owner)
    row = 4 * n_f32 + 2 * n_b16 + 8 * n_i64
    specs = [build_shard(orders, [[1.0] * len(o) for o in orders], owner, r, world) for r in range(world)]
    vol = exchange_bytes(orders, owner, world, n_f32, n_i64, n_b16)
    n_dev = len(orders)
    local = {
        "halo": max(len({j for i in s.orders_local for j in i}) + len(s.own) for s in specs) * row,
        # K3 over [n_dev, n / world] (sources + outputs) + pack (read own, write the send buffer
        # and the own block's work rows) + unpack (read the received blocks and the own block's
        # output rows, write own rows); the own block is one of these copies, never RCCL's
        "transpose": -(-2 * n_dev * row // world) + 4 * max(len(s.own) for s in specs) * row,
    }
    out = {}
    for kind in ("halo", "transpose"):
        pair = vol[kind + "_link"]
        hbm_ms = local[kind] / (HBM_GBPS * 1e6)
        link_ms = pair / (link_gbps * 1e6)
        out[kind] = dict(local_bytes=int(local[kind]), busiest_pair_bytes=int(pair), rank_link_bytes=int(vol[kind]),
                         hbm_ms=hbm_ms, link_ms=link_ms, predicted_ms=max(hbm_ms, link_ms),
                         binds="xgmi" if link_ms > hbm_ms else "hbm")
    return out


def choose_exchange(orders, owner, world: int, n_f32: int, n_i64: int, n_b16: int = 0,
                    link_gbps: Optional[float] = None) -> str:
    """'transpose' when it is clearly (10 %) cheaper than the halo, else 'halo'.  Without a
    measured link rate: by the busiest link's bytes (random expanders at 4+ ranks, 60-cliques
    spread over 4 GPUs go to the transpose; rings, community graphs, 2 ranks to the halo) - both
    exchanges use the pairs' links concurrently, so the busiest pair sets the link time.  With
    one (`link_gbps`, bench.py's probe): by link_model's predicted time, max(HBM, busiest pair /
    link_gbps), so a fast link hands the choice to the local bytes, which favour the halo (the
    transpose packs and unpacks every own model and reduces every model's column block)."""
    if world < 2:
        return "halo"
    if link_gbps is None:
        b = exchange_bytes(orders, owner, world, n_f32, n_i64, n_b16)
        return "transpose" if b["transpose_link"] < 0.9 * b["halo_link"] else "halo"
    m = link_model(orders, owner, world, n_f32, n_i64, n_b16, link_gbps=link_gbps)
    return "transpose" if m["transpose"]["predicted_ms"] < 0.9 * m["halo"]["predicted_ms"] else "halo"


def exchange_crossover_gbps(orders, owner, world: int, n_f32: int, n_i64: int, n_b16: int = 0) -> Optional[float]:
    """The link rate above which choose_exchange(link_gbps=...) stops picking the transpose
    (None when it never picks it, or picks it at any rate): the smallest r with
    max(hbm_t, Lt / r) >= 0.9 max(hbm_h, Lh / r)."""
    m = link_model(orders, owner, world, n_f32, n_i64, n_b16, link_gbps=1.0)
    ht, hh = m["transpose"]["hbm_ms"], m["halo"]["hbm_ms"]
    lt, lh = m["transpose"]["link_ms"], m["halo"]["link_ms"]  # ms at 1 GB/s: bytes / 1e6
    lo, hi = 1e-3, 1e7
    pick = lambda r: max(ht, lt / r) < 0.9 * max(hh, lh / r)  # noqa: E731
    if not pick(lo) or pick(hi):
        return None
    for _ in range(200):  # monotone in r: transpose at low rates, halo at high ones
        mid = (lo * hi) ** 0.5
        lo, hi = (mid, hi) if pick(mid) else (lo, mid)
    return hi


@dataclass
class _ColSeg:
    """One segment's buffers.  Rank p's column block (width <= b) is cut into `chunks` column
    chunks of width bc; chunk k of every block travels and is reduced on its own, so the
    all-to-alls of one chunk overlap the packing, the round and the unpacking of another.  The
    peer dimension of send / back skips this rank (peer slot of rank p: p, or p - 1 past it)."""
    n: int                  # elements per model
    b: int                  # block width
    blocks: list            # (first column, width) of each rank's block
    chunks: int
    bc: int                 # chunk width (row stride of the work buffers)
    send: torch.Tensor      # [chunks, world-1, own, bc]  my models' chunks, by destination peer
    work_in: torch.Tensor   # [chunks, R, bc]  chunk k of block `rank` of every model (own rows first)
    work_out: torch.Tensor  # [chunks, R, bc]  the round's output for it
    back: torch.Tensor      # [chunks, world-1, own, bc]  my models' output chunks, by source peer

    def chunk_blocks(self, k: int):
        """(first column, width) of chunk k of each rank's block."""
        return [(c0 + k * self.bc, max(0, min(self.bc, w - k * self.bc))) for c0, w in self.blocks]


class TransposedRound:
    """One rank's device-resident round with the transposed exchange (module docstring).  The
    models update in place in pool_a: each column chunk is packed into the send buffer before
    its outputs land (snapshot semantics; chunks touch disjoint columns).

    chunks (default 4): the block is moved and reduced in column chunks,
    pipelined - the forward all-to-all of chunk k+1 and the backward one of chunk k-1 run on
    RCCL's stream while chunk k is reduced - so the local work (pack, K3, unpack) hides under
    the link time.  The int64 segment (tens of elements) moves in one chunk."""

    def __init__(self, layout: StateLayout, orders, weights, rank: int, world: int, device,
                 mode: int = ops.MODE_EXACT, owner: Optional[np.ndarray] = None, group=None,
                 tune: bool = False, transport: str = "device", chunks: Optional[int] = None):
        self.layout = layout
        # "device": torch.distributed all_to_all_single (RCCL); "host": staged through host
        # memory (gloo rehearsal); "cabi": the library's own RCCL communicator (include/tal_agg.h
        # tal_halo_exchange), each all-to-all as one group of per-peer sends / receives
        if transport not in ("device", "host", "cabi"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport
        self.device = torch.device(device)
        self.mode = mode
        self.group = group
        self.rank, self.world = rank, world
        n_dev = len(orders)
        owner = partition_contiguous(n_dev, world) if owner is None else np.asarray(owner, np.int32)
        self.own_by_rank, self.row_base, self.pos = positions_own_first(owner, world, rank)
        self.own = self.own_by_rank[rank]
        self.local_rows = len(self.own)
        self.rows_all = n_dev
        inv = np.empty(n_dev, dtype=np.int64)
        inv[self.pos] = np.arange(n_dev)
        self.orders_pos = [[int(self.pos[j]) for j in orders[int(inv[q])]] for q in range(n_dev)]
        self.weights_pos = [[float(x) for x in weights[int(inv[q])]] for q in range(n_dev)]
        self.pool_a = ModelPool(layout, self.local_rows, self.device)
        self.chunks = max(1, int(chunks if chunks is not None else 4))
        self.segs: Dict[str, _ColSeg] = {}
        for g, n, dt in (("f32", layout.n_f32, torch.float32), ("b16", layout.n_b16, torch.bfloat16),
                         ("i64", layout.n_i64, torch.int64)):
            if not n:
                continue
            b, blocks = column_blocks(n, world)
            c = 1 if g == "i64" else max(1, min(self.chunks, b // 4))
            bc = _round_up(-(-b // c), 4)

            def z(*shape, dt=dt):
                return torch.zeros(*shape, dtype=dt, device=self.device)

            peers = max(1, world - 1)
            self.segs[g] = _ColSeg(n, b, blocks, c, bc, z(c, peers, self.local_rows, bc), z(c, n_dev, bc),
                                   z(c, n_dev, bc), z(c, peers, self.local_rows, bc))
        self.w_me = {g: s.blocks[rank][1] for g, s in self.segs.items()}
        rp, col, w = csr_from_lists(self.orders_pos, self.weights_pos)
        out_rows = np.arange(n_dev, dtype=np.int32)
        tg = tune_segment(layout)
        f = self.segs.get(tg)
        w0 = f.chunk_blocks(0)[rank][1] if f is not None else 0
        if tune and w0:
            self.plan = ops.tune_plan(rp, col, w, out_rows, f.work_in[0], f.work_out[0], n=w0, mode=mode)
        else:
            self.plan = ops.default_plan(rp, col, w, out_rows, bf16=bool(layout.n_b16), mode=mode).to(self.device)
        self.plans = {"round": self.plan}
        self.staged_sources = self.plan.staged_rows()
        self.exchange_kind = "transpose"
        self._events: list = []
        if transport == "cabi":
            from .comm import shared_halo_comm

            self.comm = shared_halo_comm(world, rank, device, group)
            self.comm_stream = torch.cuda.Stream(self.device)
        if dist.is_available() and dist.is_initialized():
            dist.barrier(group=group)

    def _segs_at(self, k: int):
        return [(g, s) for g, s in self.segs.items() if k < s.chunks]

    def peer_slot(self, p: int) -> int:
        """Index of rank p (!= this rank) in the peer dimension of send / back."""
        return p if p < self.rank else p - 1

    def peers(self):
        return [p for p in range(self.world) if p != self.rank]

    def rows_of(self, p: int) -> slice:
        """The work-buffer rows holding rank p's models."""
        return slice(int(self.row_base[p]), int(self.row_base[p]) + len(self.own_by_rank[p]))

    # phases of chunk k: step() pipelines them; the virtual-rank GPU test interleaves ranks
    def pack(self, k: int = 0) -> None:
        """Chunk k of my models: block p into send (peer p), my own block straight into the
        head rows of work_in (it never leaves this GPU)."""
        pools = _pool_segs(self.pool_a)
        own = self.rows_of(self.rank)
        for g, s in self._segs_at(k):
            cb = s.chunk_blocks(k)
            for p in self.peers():
                c0, w = cb[p]
                if w:
                    s.send[k][self.peer_slot(p)][:, :w].copy_(pools[g][: self.local_rows, c0: c0 + w])
            c0, w = cb[self.rank]
            if w:
                s.work_in[k][own, :w].copy_(pools[g][: self.local_rows, c0: c0 + w])

    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        if self.transport == "host":
            o = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_to_all_single(o, inp.reshape(-1).cpu(), out_splits, in_splits, group=self.group)
            out.view(-1).copy_(o)
            return None
        return dist.all_to_all_single(out.view(-1), inp.view(-1), out_splits, in_splits, group=self.group,
                                      async_op=True)

    def _splits(self, per_rank):
        """Split sizes in rank order with 0 for this rank (its block stays local)."""
        return [0 if p == self.rank else int(v) for p, v in enumerate(per_rank)]

    def forward_messages(self, k: int, g: str):
        """The forward all-to-all of chunk k, segment g, as per-peer messages: (sends, recvs),
        entry p = the contiguous tensor going to / coming from rank p (None for this rank):
        my models' chunk of block p, and block `rank`'s chunk of p's models (their work rows)."""
        s = self.segs[g]
        sends, recvs = [None] * self.world, [None] * self.world
        for p in self.peers():
            sends[p] = s.send[k][self.peer_slot(p)]
            recvs[p] = s.work_in[k][self.rows_of(p)]
        return sends, recvs

    def backward_messages(self, k: int, g: str):
        """The backward all-to-all of chunk k, segment g, as per-peer messages: p's models' output
        rows of my block go to p; my models' output chunk of block p comes from p."""
        s = self.segs[g]
        sends, recvs = [None] * self.world, [None] * self.world
        for p in self.peers():
            sends[p] = s.work_out[k][self.rows_of(p)]
            recvs[p] = s.back[k][self.peer_slot(p)]
        return sends, recvs

    def _exchange_cabi(self, k: int, messages) -> list:
        """One RCCL group per segment through the C-ABI (tal_halo_exchange) on the comm stream,
        after everything queued so far on the current stream (the packing, the round that wrote
        the outputs, the unpacking that last read the receive buffers); the compute stream waits
        on the returned request's event."""
        from .distributed import _StreamRequest

        cur = torch.cuda.current_stream(self.device)
        self.comm_stream.wait_stream(cur)
        for g, _ in self._segs_at(k):
            sends, recvs = messages(k, g)
            self.comm.exchange(sends, recvs, self.comm_stream)
        ev = torch.cuda.Event()
        ev.record(self.comm_stream)
        return [_StreamRequest(ev, self.device)]

    def forward_exchange(self, k: int = 0) -> list:
        """Chunk k of block `rank` of every other rank's models into work_in[k] after my own
        rows; returns the pending works (none at world 1: nothing leaves the GPU)."""
        if self.world == 1:
            return []
        if self.transport == "cabi":
            return self._exchange_cabi(k, self.forward_messages)
        works = [self._all_to_all(s.work_in[k][self.local_rows:], s.send[k],
                                  self._splits([len(o) * s.bc for o in self.own_by_rank]),
                                  self._splits([self.local_rows * s.bc] * self.world)) for _, s in self._segs_at(k)]
        return [w for w in works if w is not None]

    def compute(self, k: int = 0) -> None:
        segs = self._segs_at(k)
        run_round_segments(self.layout, {g: s.work_in[k] for g, s in segs}, {g: s.work_out[k] for g, s in segs},
                           self.plan, self.mode, n_of={g: s.chunk_blocks(k)[self.rank][1] for g, s in segs})

    def backward_exchange(self, k: int = 0) -> list:
        """Every other rank's models' output rows back to their owners (my own stay here)."""
        if self.world == 1:
            return []
        if self.transport == "cabi":
            return self._exchange_cabi(k, self.backward_messages)
        works = [self._all_to_all(s.back[k], s.work_out[k][self.local_rows:],
                                  self._splits([self.local_rows * s.bc] * self.world),
                                  self._splits([len(o) * s.bc for o in self.own_by_rank])) for _, s in self._segs_at(k)]
        return [w for w in works if w is not None]

    def unpack(self, k: int = 0) -> None:
        """My models' output chunk k: block p from back (peer p), my own block straight from the
        head rows of work_out."""
        pools = _pool_segs(self.pool_a)
        own = self.rows_of(self.rank)
        for g, s in self._segs_at(k):
            cb = s.chunk_blocks(k)
            for p in self.peers():
                c0, w = cb[p]
                if w:
                    pools[g][: self.local_rows, c0: c0 + w].copy_(s.back[k][self.peer_slot(p)][:, :w])
            c0, w = cb[self.rank]
            if w:
                pools[g][: self.local_rows, c0: c0 + w].copy_(s.work_out[k][own, :w])

    def step(self, timed: bool = False) -> None:
        """One round, chunk-pipelined: pack k+1 and its forward all-to-all are issued before
        chunk k is reduced; chunk k's backward all-to-all runs while k+1 is reduced; each wait()
        only makes the compute stream wait on RCCL's.  With timed=True the K3 launches are
        bracketed by events (kernel_ms(): their sum per step)."""
        C = self.chunks
        ev = [] if timed else None
        fwd, bwd = {}, {}
        self.pack(0)
        fwd[0] = self.forward_exchange(0)
        for k in range(C):
            if k + 1 < C:
                self.pack(k + 1)
                fwd[k + 1] = self.forward_exchange(k + 1)
            for w in fwd.pop(k):
                w.wait()
            if ev is not None:
                ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                ev[-1][0].record()
            self.compute(k)
            if ev is not None:
                ev[-1][1].record()
            bwd[k] = self.backward_exchange(k)
            if k >= 1:
                for w in bwd.pop(k - 1):
                    w.wait()
                self.unpack(k - 1)
        for w in bwd.pop(C - 1):
            w.wait()
        self.unpack(C - 1)
        if ev is not None:
            self._events.append(ev)

    def kernel_ms(self) -> List[float]:
        out = [sum(a.elapsed_time(b) for a, b in e) for e in self._events]
        self._events = []
        return out

    def own_rows(self) -> ModelPool:
        return self.pool_a

    @property
    def own_ids(self) -> List[int]:
        """Global device ids of own_rows()'s rows 0, 1, ..."""
        return self.own

    @property
    def kernel_bytes(self) -> int:
        """Algorithmic HBM bytes of one round's K3 launches (staged sources + written rows)."""
        return sum(_ESIZE[g] * self.w_me[g] for g, _ in float_segments(self.layout)) * (
            self.staged_sources + self.rows_all)

    @property
    def link_bytes(self) -> int:
        """Bytes this rank receives over the links per round (both all-to-alls; its own block
        is copied on the GPU, not sent)."""
        r = 0
        for g, s in self.segs.items():
            r += _ESIZE[g] * s.chunks * s.bc * ((self.rows_all - self.local_rows) + self.local_rows * (self.world - 1))
        return r

    def spot_check(self) -> bool:
        """After a step: the first row of this rank's first column chunk == K1 on its operands'
        chunks (bitwise)."""
        segs = {g: s for g, s in self.segs.items() if g != "i64"}
        ops_ = {g: [s.work_in[0][j] for j in self.orders_pos[0]] for g, s in segs.items()}
        return spot_check_row(self.layout, ops_, self.weights_pos[0], {g: s.work_out[0][0] for g, s in segs.items()},
                              self.mode, n_of={g: s.chunk_blocks(0)[self.rank][1] for g, s in segs.items()})


def make_round(layout: StateLayout, orders, weights, rank: int, world: int, device, exchange: str = "auto",
               mode: int = ops.MODE_EXACT, owner: Optional[np.ndarray] = None, group=None, tune: bool = False,
               transport: str = "device", link_gbps: Optional[float] = None):
    """This rank's sharded round with the given exchange ('halo' | 'transpose' | 'auto');
    transport 'device' = torch.distributed's RCCL, 'host' stages the exchange through host
    memory (gloo rehearsal runs only), 'cabi' moves either exchange through the library's own
    RCCL communicator (tal_comm_* / tal_halo_pack / tal_halo_exchange: per-peer messages in one
    RCCL group; an all-to-all is such a group).  link_gbps: a measured per-pair link rate for
    the 'auto' choice (choose_exchange)."""
    owner = partition_contiguous(len(orders), world) if owner is None else np.asarray(owner, np.int32)
    if transport == "cabi" and world > 1:
        import warnings

        warnings.warn("transport 'cabi' (the library's own RCCL communicator) is experimental across GPUs: "
                      "tested on one rank and on virtual ranks only; no committed multi-GPU run yet",
                      stacklevel=2)
    if exchange == "auto":
        exchange = choose_exchange(orders, owner, world, layout.n_f32, layout.n_i64, layout.n_b16, link_gbps=link_gbps)
    cls = {"halo": ShardedRound, "transpose": TransposedRound}[exchange]
    r = cls(layout, orders, weights, rank, world, device, mode=mode, owner=owner, group=group, tune=tune,
            transport=transport)
    r.exchange_kind = exchange
    return r
