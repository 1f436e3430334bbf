"""Aggregation rounds with the simulated devices sharded over GPUs (one process per GPU).

Partitioning: every rank owns a contiguous block of simulated devices (or any owner map the
caller gives) and keeps their models as rows of a local pool.  A round needs, on rank g, the
models of every remote neighbor of its rows — the halo.  The exchange is point-to-point: for
each ordered pair (g -> h), g sends the unique set of its own rows that h's rows reference,
once, however many of h's rows use it (torch.distributed P2P, i.e. RCCL ncclSend/ncclRecv in
one group over xGMI with the "nccl" backend, gloo on CPU for tests).  There is no all-reduce:
the round is a sparse W·X whose outputs stay sharded.

Overlap: the rows whose operands are all local ("interior") are reduced by the K3 kernel on
the compute stream while the halo is in flight; the remaining ("boundary") rows run after the
receives complete.  Inputs are double-buffered (pool a -> pool b, then swap) so snapshot
semantics hold across the two launches.  Exactness is unchanged: every row still sums its
operands in reference order (neighbors ascending, self last).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .arena import ModelPool, StateLayout
from .round import csr_from_lists


def partition_contiguous(n: int, world: int) -> np.ndarray:
    """owner[i] for n devices over `world` ranks in contiguous, near-equal blocks."""
    return (np.arange(n, dtype=np.int64) * world // n).astype(np.int32)


@dataclass
class ShardSpec:
    rank: int
    world: int
    own: List[int]                      # global ids owned, ascending
    halo: List[int]                     # global ids received, grouped by owner, ascending
    local_of: Dict[int, int]            # global id -> local pool row
    send: Dict[int, List[int]] = field(default_factory=dict)  # peer -> local rows to send
    recv: Dict[int, List[int]] = field(default_factory=dict)  # peer -> local rows to fill
    interior: List[int] = field(default_factory=list)         # own-row indices, all operands local
    boundary: List[int] = field(default_factory=list)
    orders_local: List[List[int]] = field(default_factory=list)  # per own row, local source rows
    weights: List[List[float]] = field(default_factory=list)

    @property
    def rows(self) -> int:
        return len(self.own) + len(self.halo)


def build_shard(orders: Sequence[Sequence[int]], weights: Sequence[Sequence[float]], owner: np.ndarray,
                rank: int, world: Optional[int] = None) -> ShardSpec:
    """Rank `rank`'s part of a round.  orders[i] = operands of device i in reference order."""
    owner = np.asarray(owner)
    if world is None:
        world = int(owner.max()) + 1 if len(owner) else 1
    own = [i for i in range(len(orders)) if owner[i] == rank]
    own_set = set(own)
    need = sorted({j for i in own for j in orders[i] if j not in own_set}, key=lambda j: (owner[j], j))
    local_of = {g: k for k, g in enumerate(own)}
    for k, g in enumerate(need):
        local_of[g] = len(own) + k
    spec = ShardSpec(rank=rank, world=world, own=own, halo=need, local_of=local_of)
    for p in range(world):
        if p == rank:
            continue
        # what p needs from me: my rows referenced by p's rows (same sorted list on both sides)
        p_rows = [i for i in range(len(orders)) if owner[i] == p]
        give = sorted({j for i in p_rows for j in orders[i] if owner[j] == rank})
        if give:
            spec.send[p] = [local_of[j] for j in give]
        take = [j for j in need if owner[j] == p]
        if take:
            spec.recv[p] = [local_of[j] for j in take]
    for k, i in enumerate(own):
        spec.orders_local.append([local_of[j] for j in orders[i]])
        spec.weights.append([float(x) for x in weights[i]])
        (spec.interior if all(owner[j] == rank for j in orders[i]) else spec.boundary).append(k)
    return spec


def recv_range(spec: ShardSpec, peer: int):
    """The halo rows `peer` fills: one contiguous block of local rows (the halo is grouped by
    owner, ascending global id on both sides), or None."""
    rows = spec.recv.get(peer)
    if not rows:
        return None
    r0, r1 = rows[0], rows[-1] + 1
    if r1 - r0 != len(rows):
        raise AssertionError("halo rows of one peer are not contiguous")
    return r0, r1


class HaloPacker:
    """Per-peer send buffers of one pool tensor: the rows a peer needs, in its receive order,
    as ONE contiguous [k, ld] tensor, so a round moves one message per peer per segment
    (instead of one per model row).  Rows that are already consecutive in the pool are sent as
    a view (no copy); otherwise they are gathered into a buffer allocated once."""

    def __init__(self, spec: ShardSpec, t: torch.Tensor):
        self.spec = spec
        self.bufs: Dict[int, torch.Tensor] = {}
        self.idx: Dict[int, torch.Tensor] = {}
        self.idx32: Dict[int, torch.Tensor] = {}
        for peer, rows in spec.send.items():
            if rows == list(range(rows[0], rows[0] + len(rows))):
                continue  # consecutive: sent as t[r0:r1]
            self.idx[peer] = torch.as_tensor(rows, dtype=torch.long, device=t.device)
            self.idx32[peer] = self.idx[peer].to(torch.int32)  # the C-ABI gather's row list
            self.bufs[peer] = torch.empty((len(rows), t.shape[1]), dtype=t.dtype, device=t.device)

    def send_tensor(self, t: torch.Tensor, peer: int) -> torch.Tensor:
        """The message for `peer` from pool tensor t (gathers on the current stream)."""
        rows = self.spec.send[peer]
        if peer not in self.idx:
            return t[rows[0]: rows[0] + len(rows)]
        return torch.index_select(t, 0, self.idx[peer], out=self.bufs[peer])


def post_exchange(spec: ShardSpec, tensors: Sequence[torch.Tensor], group=None,
                  packers: Optional[Sequence[HaloPacker]] = None) -> list:
    """Post the halo sends/receives of one round for each [rows, ld] pool tensor; returns the
    requests (wait on them before reading halo rows).  One message per peer per segment each
    way (HaloPacker), all in one P2P group: RCCL batches it into a single
    ncclGroupStart / ncclSend+ncclRecv per peer / ncclGroupEnd."""
    if packers is None:
        packers = [HaloPacker(spec, t) for t in tensors]
    p2p = []
    for peer in sorted(set(spec.send) | set(spec.recv)):
        for t, pk in zip(tensors, packers):
            if peer in spec.send:
                p2p.append(dist.P2POp(dist.isend, pk.send_tensor(t, peer), peer, group=group))
            rr = recv_range(spec, peer)
            if rr is not None:
                p2p.append(dist.P2POp(dist.irecv, t[rr[0]: rr[1]], peer, group=group))
    if not p2p:
        return []
    return dist.batch_isend_irecv(p2p)


_ESIZE = {"f32": 4, "b16": 2, "i64": 8}


def float_segments(layout: StateLayout):
    """(name, elements) of the layout's non-empty floating-point segments."""
    return [(g, n) for g, n in (("f32", layout.n_f32), ("b16", layout.n_b16)) if n]


def tune_segment(layout: StateLayout) -> str:
    """The segment a round plan is tuned on: bf16 when there is one (its plan forms - sparse,
    narrow - also run fp32 and int64), else fp32."""
    return "b16" if layout.n_b16 else "f32"


def run_round_segments(layout: StateLayout, seg_in: dict, seg_out: dict, plan, mode: int,
                       n_of: Optional[dict] = None) -> None:
    """The K3 round of `plan` on every non-empty segment (seg_*: name -> [rows, ld] tensor;
    n_of: name -> columns, default the layout's elements per model)."""
    for g, n in (("f32", layout.n_f32), ("b16", layout.n_b16), ("i64", layout.n_i64)):
        n = n if n_of is None else n_of.get(g, 0)
        if not n:
            continue
        if g == "f32":
            ops.round_f32(seg_in[g], seg_out[g], plan, n=n, mode=mode)
        elif g == "b16":
            ops.round_bf16(seg_in[g], seg_out[g], plan, n=n, mode=mode)
        else:
            ops.round_i64(seg_in[g], seg_out[g], plan, n=n)


def _pool_segs(pool: ModelPool) -> dict:
    return {"f32": pool.f32, "b16": pool.b16, "i64": pool.i64}


def spot_check_row(layout: StateLayout, operands: dict, weights, got: dict, mode: int, n_of=None) -> bool:
    """K1 on one row's operands (per float segment) == the round's output row, bitwise."""
    for g, n in float_segments(layout):
        n = n if n_of is None else n_of.get(g, 0)
        if not n:
            continue
        dt = torch.float32 if g == "f32" else torch.bfloat16
        chk = torch.empty(n, dtype=dt, device=got[g].device)
        (ops.agg_f32 if g == "f32" else ops.agg_bf16)([x[:n] for x in operands[g]], weights, chk, mode=mode)
        iv = torch.int32 if g == "f32" else torch.int16
        if not torch.equal(chk.view(iv), got[g][:n].contiguous().view(iv)):
            return False
    return True


class _StagedRequests:
    """Requests of a host-staged exchange: wait() completes the receives, then copies the
    received rows into the device pool."""

    def __init__(self, reqs, fills):
        self.reqs, self.fills = reqs, fills

    def wait(self):
        for r in self.reqs:
            r.wait()
        for dst, src in self.fills:
            dst.copy_(src)
        self.reqs, self.fills = [], []


def post_exchange_staged(spec: ShardSpec, tensors: Sequence[torch.Tensor], group=None,
                         packers: Optional[Sequence[HaloPacker]] = None) -> list:
    """post_exchange through host memory, for process groups without device transport (gloo):
    rehearses the multi-GPU path (same packed per-peer messages) with several ranks on one GPU.
    Not a production path."""
    if packers is None:
        packers = [HaloPacker(spec, t) for t in tensors]
    p2p, fills = [], []
    for peer in sorted(set(spec.send) | set(spec.recv)):
        for t, pk in zip(tensors, packers):
            if peer in spec.send:
                p2p.append(dist.P2POp(dist.isend, pk.send_tensor(t, peer).cpu(), peer, group=group))
            rr = recv_range(spec, peer)
            if rr is not None:
                buf = torch.empty((rr[1] - rr[0], t.shape[1]), dtype=t.dtype)
                p2p.append(dist.P2POp(dist.irecv, buf, peer, group=group))
                fills.append((t[rr[0]: rr[1]], buf))
    if not p2p:
        return []
    return [_StagedRequests(dist.batch_isend_irecv(p2p), fills)]


class _StreamRequest:
    """An exchange enqueued on a side stream: wait() makes the current stream wait for it."""

    def __init__(self, event, device):
        self.event, self.device = event, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.event)


def post_exchange_cabi(spec: ShardSpec, tensors: Sequence[torch.Tensor], comm, stream,
                       packers: Sequence[HaloPacker]) -> list:
    """post_exchange through the C-ABI (comm.HaloComm): on `stream`, after the work already
    queued on the current stream, each peer's rows are packed by the library's gather kernel
    and every segment's messages go out in one RCCL group; the returned request makes the
    current stream wait for the receives."""
    cur = torch.cuda.current_stream(comm.device)
    stream.wait_stream(cur)
    world = spec.world
    with torch.cuda.stream(stream):
        for t, pk in zip(tensors, packers):
            sends, recvs = [None] * world, [None] * world
            for peer in spec.send:
                if peer in pk.idx32:
                    sends[peer] = comm.pack(t, pk.idx32[peer], pk.bufs[peer], stream)
                else:
                    rows = spec.send[peer]
                    sends[peer] = t[rows[0]: rows[0] + len(rows)]
            for peer in spec.recv:
                r0, r1 = recv_range(spec, peer)
                recvs[peer] = t[r0:r1]
            comm.exchange(sends, recvs, stream)
    ev = torch.cuda.Event()
    ev.record(stream)
    return [_StreamRequest(ev, comm.device)]


class ShardedRound:
    """One rank's device-resident round over its shard (K3 kernels + halo exchange)."""

    def __init__(self, layout: StateLayout, orders, weights, rank: int, world: int, device,
                 mode: int = ops.MODE_EXACT, owner: Optional[np.ndarray] = None, group=None,
                 exchange: Optional[Callable[["ShardedRound"], list]] = None, tune: bool = False,
                 transport: str = "device"):
        self.layout = layout
        self.device = torch.device(device)
        self.mode = mode
        self.group = group
        # exchange(self) -> requests; default: RCCL/gloo P2P.  Tests may pass an in-process copy.
        # transport "host": the exchange is staged through host memory (gloo rehearsal runs);
        # "cabi": the library's own RCCL communicator and gather kernel (comm.HaloComm) on a
        # side stream, the unique id broadcast through the torch.distributed group (its messages
        # are checked across virtual ranks and through a world-1 communicator on one GPU,
        # tests/test_gpu_comm.py; RCCL refuses two ranks on one GPU)
        if transport not in ("device", "host", "cabi"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport
        if transport == "cabi" and exchange is None:
            from .comm import shared_halo_comm

            self.comm = shared_halo_comm(world, rank, device, group)
            self.comm_stream = torch.cuda.Stream(torch.device(device))
            self._exchange = lambda sr: post_exchange_cabi(sr.spec, [t for _, t, _ in sr.pool_a.segments()],
                                                           sr.comm, sr.comm_stream, sr.packers)
        else:
            post = post_exchange_staged if transport == "host" else post_exchange
            self._exchange = exchange or (lambda sr: post(sr.spec, [t for _, t, _ in sr.pool_a.segments()],
                                                          sr.group, sr.packers))
        owner = partition_contiguous(len(orders), world) if owner is None else np.asarray(owner, np.int32)
        self.spec = build_shard(orders, weights, owner, rank, world)
        self.pool_a = ModelPool(layout, self.spec.rows, self.device)
        self.pool_b = ModelPool(layout, self.spec.rows, self.device)
        # one packer per segment serves both pools (same shape; the row lists do not change)
        self.packers = [HaloPacker(self.spec, t) for _, t, _ in self.pool_a.segments()]
        self.plans = {}
        tg = tune_segment(layout)
        for name, idx in (("interior", self.spec.interior), ("boundary", self.spec.boundary)):
            if idx:
                rp, col, w = csr_from_lists([self.spec.orders_local[k] for k in idx],
                                            [self.spec.weights[k] for k in idx])
                out = np.asarray(idx, np.int32)
                self.plans[name] = (
                    ops.tune_plan(rp, col, w, out, _pool_segs(self.pool_a)[tg], _pool_segs(self.pool_b)[tg],
                                  n=getattr(layout, "n_" + tg), mode=mode)
                    if tune else ops.default_plan(rp, col, w, out, bf16=bool(layout.n_b16), mode=mode).to(self.device))
        if exchange is None and dist.is_available() and dist.is_initialized():
            # a collective over the whole group first: RCCL then builds the communicator with
            # every rank, so the first batched P2P does not depend on which ranks have halos
            dist.barrier(group=group)
        self.local_rows = len(self.spec.own)
        self.halo_rows_in = len(self.spec.halo)
        self.staged_sources = sum(p.staged_rows() for p in self.plans.values())
        self._events: list = []

    def _run(self, name: str, a: ModelPool, b: ModelPool) -> None:
        plan = self.plans.get(name)
        if plan is None:
            return
        run_round_segments(self.layout, _pool_segs(a), _pool_segs(b), plan, self.mode)

    def step(self, timed: bool = False) -> None:
        """One round: halo exchange overlapped with the interior rows, then the boundary rows.
        With timed=True the kernels are bracketed by events (read them with kernel_ms())."""
        a, b = self.pool_a, self.pool_b
        reqs = self._exchange(self)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        if ev:
            ev[0].record()
        self._run("interior", a, b)
        if ev:
            ev[1].record()
        for r in reqs:
            r.wait()
        if ev:
            ev[2].record()
        self._run("boundary", a, b)
        if ev:
            ev[3].record()
            self._events.append(ev)
        self.pool_a, self.pool_b = b, a

    def kernel_ms(self) -> List[float]:
        """Per timed step: interior + boundary kernel time (ms); call after synchronizing."""
        out = [e[0].elapsed_time(e[1]) + e[2].elapsed_time(e[3]) for e in self._events]
        self._events = []
        return out

    def own_rows(self) -> ModelPool:
        """Pool whose rows [0, local_rows) hold this rank's current models."""
        return self.pool_a

    @property
    def own_ids(self) -> List[int]:
        """Global device ids of own_rows()'s rows 0, 1, ..."""
        return self.spec.own

    @property
    def kernel_bytes(self) -> int:
        """Algorithmic HBM bytes of one round's local kernels (staged sources + written rows)."""
        return sum(_ESIZE[g] * n for g, n in float_segments(self.layout)) * (self.staged_sources + self.local_rows)

    @property
    def link_bytes(self) -> int:
        """Bytes this rank receives over the links per round."""
        lay = self.layout
        return self.halo_rows_in * (4 * lay.n_f32 + 2 * lay.n_b16 + 8 * lay.n_i64)

    def spot_check(self) -> bool:
        """After a step: one (boundary if any) row == K1 on its operands as they were received
        (bitwise; the operands are the previous buffer, now pool_b)."""
        k = (self.spec.boundary or self.spec.interior)[0]
        a, b = _pool_segs(self.pool_a), _pool_segs(self.pool_b)
        ops_ = {g: [b[g][j] for j in self.spec.orders_local[k]] for g in ("f32", "b16")}
        return spot_check_row(self.layout, ops_, self.spec.weights[k], {g: a[g][k] for g in a}, self.mode)
