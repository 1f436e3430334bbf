"""The reference's driver on several GPUs of its one process (TAL_GPUS).

The reference runs every aggregation inside one coordinator process (its Parsl thread pool,
/root/reference/src/experiments/parsl_setup.py:75-78; the round driver
/root/reference/src/decentralized_app.py:605-641).  With TAL_GPUS=N that process spreads its
clients over N GPUs: contiguous blocks of clients (distributed.partition_contiguous), one
``ModelPool`` per GPU holding

* the GPU's own clients (rows 0 .. own-1, each client's model bound to its row), then
* ghost rows: every other GPU's client that one of this GPU's clients can draw as a neighbor
  (a non-zero entry of the topology's adjacency row), grouped by owner, ascending,

so every aggregation runs on its client's GPU over rows of one pool (K1 on rows, or the GPU's
share of a K3 round).  A ghost row holds a copy of its owner's row, refreshed when read:

* per call (the reference's form, `aggregate.aggregate_models` / `similarity.cosine_pairs`): the
  operands a call reads from other GPUs are copied into their ghost rows just before the K1
  launch (a device-to-device copy ordered behind both devices' streams), so a call sees the
  neighbor's model as it is at that moment, as the reference's call does;
* per batched round (TAL_BATCHED_ROUND=1): the whole halo - for every ordered GPU pair (h -> g)
  the rows of h that g's ghost block for h holds - moves before the round, by RCCL sends and
  receives between the process's own per-device communicators (tal_comm_init_local /
  tal_halo_exchange_local: one RCCL group, each GPU's messages on its own stream), each
  message packed by tal_halo_pack on the sender and received straight into the receiver's
  contiguous ghost block; each GPU's round kernel then runs on the same stream, so it starts
  only after its own sends (which read the rows it is about to overwrite in place) and receives
  are done.  Pools on one device (virtual GPUs, `TAL_VIRTUAL_GPUS`, for tests on one GPU) use the
  in-process copy transport instead.
"""
from __future__ import annotations

import ctypes
import sys
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .arena import ModelPool, bound_row
from .distributed import partition_contiguous


class LocalComms:
    """n RCCL communicators of this process, rank r on devices[r] (tal_comm_init_local)."""

    def __init__(self, devices: Sequence[int]):
        self.n = len(devices)
        self._comms = (ctypes.c_void_p * self.n)()
        dev = (ctypes.c_int32 * self.n)(*[int(d) for d in devices])
        _lib.check(_lib.load().tal_comm_init_local(self._comms, self.n, dev))

    def exchange(self, sends, recvs, streams) -> None:
        """sends[r][p] / recvs[r][p]: contiguous device tensors (or None) of rank r for peer p;
        streams[r]: rank r's stream.  One RCCL group for all of them."""
        n = self.n
        sb, rb = (ctypes.c_void_p * (n * n))(), (ctypes.c_void_p * (n * n))()
        sn, rn = (ctypes.c_int64 * (n * n))(), (ctypes.c_int64 * (n * n))()
        for r in range(n):
            for p in range(n):
                for t, b, c in ((sends[r][p], sb, sn), (recvs[r][p], rb, rn)):
                    if t is None or t.numel() == 0:
                        continue
                    b[r * n + p] = t.data_ptr()
                    c[r * n + p] = t.numel() * t.element_size()
        st = (ctypes.c_void_p * n)(*[s.cuda_stream for s in streams])
        _lib.check(_lib.load().tal_halo_exchange_local(self._comms, n, sb, sn, rb, rn, st))

    def close(self) -> None:
        L = _lib.load()
        for k in range(self.n):
            if self._comms[k]:
                _lib.check(L.tal_comm_destroy(ctypes.c_void_p(self._comms[k])))
                self._comms[k] = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


class MultiPool:
    """Clients 0..n-1 over `devices` (see the module docstring).  adjacency: the topology's
    [n, n] matrix (non-zero = a neighbor the client can draw); None = every other client.
    transport: 'rccl' (distinct devices; the default there), 'copy' (device-to-device copies;
    the only one for pools sharing a device)."""

    def __init__(self, layout, n: int, devices: Sequence, adjacency=None, transport: str = "auto",
                 make_pool=None):
        self.layout = layout
        self.n = int(n)
        self.devices = [torch.device(d) for d in devices]
        self.world = len(self.devices)
        self.owner = partition_contiguous(self.n, self.world)
        if adjacency is None:
            adj = ~np.eye(self.n, dtype=bool)
        else:
            adj = np.asarray(adjacency) != 0
            if adj.shape != (self.n, self.n):
                raise ValueError(f"adjacency must be [{self.n}, {self.n}]")
        self.own: List[List[int]] = [np.flatnonzero(self.owner == g).tolist() for g in range(self.world)]
        self.halo: List[List[int]] = []
        self.ghost_block: List[Dict[int, Tuple[int, int]]] = []  # g -> {owner h: (first row, rows)}
        self.local: List[Dict[int, int]] = []  # g -> {global id: pool row}
        for g in range(self.world):
            mine = np.zeros(self.n, dtype=bool)
            mine[self.own[g]] = True
            need = adj[mine].any(axis=0) & ~mine
            halo = sorted(np.flatnonzero(need).tolist(), key=lambda j: (int(self.owner[j]), j))
            self.halo.append(halo)
            loc = {j: r for r, j in enumerate(self.own[g])}
            blocks: Dict[int, Tuple[int, int]] = {}
            for k, j in enumerate(halo):
                row = len(self.own[g]) + k
                loc[j] = row
                h = int(self.owner[j])
                first, cnt = blocks.get(h, (row, 0))
                blocks[h] = (first, cnt + 1)
            self.local.append(loc)
            self.ghost_block.append(blocks)
        make = make_pool or (lambda rows, dev: ModelPool(layout, rows, dev))
        self.pools: List[ModelPool] = []
        for g in range(self.world):
            p = make(len(self.own[g]) + len(self.halo[g]), self.devices[g])
            p.multi = (self, g)  # type: ignore[attr-defined]
            self.pools.append(p)
        distinct = len({(d.type, d.index) for d in self.devices}) == self.world
        if transport == "auto":
            transport = "rccl" if distinct and self.world > 1 else "copy"
        if transport == "rccl" and not distinct:
            raise ValueError("the RCCL transport takes one rank per device; pools sharing a device use 'copy'")
        self.transport = transport
        self._comms: Optional[LocalComms] = None
        # rows each owner sends to each peer (its ghost block there, in order), on the owner's device
        self._send_rows: Dict[Tuple[int, int], torch.Tensor] = {}
        for g in range(self.world):
            for h, (first, cnt) in self.ghost_block[g].items():
                ids = self.halo[g][first - len(self.own[g]): first - len(self.own[g]) + cnt]
                rows = [self.local[h][j] for j in ids]
                self._send_rows[(h, g)] = torch.tensor(rows, dtype=torch.int32, device=self.devices[h])

    # ---- placement ------------------------------------------------------------------------
    def home(self, gid: int) -> Tuple[int, int]:
        """(GPU, pool row) of client gid's own row."""
        g = int(self.owner[gid])
        return g, self.local[g][gid]

    def global_id(self, pool: ModelPool, row: int) -> int:
        g = pool.multi[1]  # type: ignore[attr-defined]
        if row >= len(self.own[g]):
            raise ValueError("a model bound to a ghost row")
        return self.own[g][row]

    def bind(self, module, gid: int):
        g, r = self.home(gid)
        module.to(self.devices[g])
        return self.pools[g].bind(module, r)

    def member(self, pool) -> Optional[int]:
        """GPU index of `pool` if it is one of this MultiPool's pools."""
        m = getattr(pool, "multi", None)
        return m[1] if m is not None and m[0] is self else None

    # ---- per-call reads ---------------------------------------------------------------------
    def rows_for(self, g: int, bounds: Sequence[Tuple[ModelPool, int]]) -> List[int]:
        """Rows of pool g holding the models bound at `bounds` ((pool, row) of this MultiPool),
        the remote ones copied into their ghost rows first (all segments, ordered behind the
        owner's and this device's current streams)."""
        out = []
        dst = self.pools[g]
        for pool, r in bounds:
            h = self.member(pool)
            if h is None:
                raise ValueError("a model outside this MultiPool")
            if h == g:
                out.append(r)
                continue
            gid = self.global_id(pool, r)
            gr = self.local[g].get(gid)
            if gr is None:
                raise ValueError(f"client {gid} is not a neighbor of any client on GPU {g} in the topology")
            for (_, t_dst, _), (_, t_src, _) in zip(dst.segments(), pool.segments()):
                t_dst[gr].copy_(t_src[r])
            out.append(gr)
        return out

    # ---- batched round ----------------------------------------------------------------------
    def exchange_halo(self) -> None:
        """Every ghost row of every pool refreshed from its owner's row (the whole halo)."""
        if self.world == 1:
            return
        if self.transport == "copy":
            for g in range(self.world):
                for h, (first, cnt) in self.ghost_block[g].items():
                    src_rows = self._send_rows[(h, g)].long()
                    for (_, t_dst, _), (_, t_src, _) in zip(self.pools[g].segments(), self.pools[h].segments()):
                        t_dst[first: first + cnt].copy_(t_src.index_select(0, src_rows))
            return
        from .comm import HaloComm

        if self._comms is None:
            self._comms = LocalComms([d.index for d in self.devices])
        streams = [torch.cuda.current_stream(d) for d in self.devices]
        segs = [p.segments() for p in self.pools]
        for k in range(len(segs[0])):  # one RCCL group per segment (f32, b16, i64)
            sends = [[None] * self.world for _ in range(self.world)]
            recvs = [[None] * self.world for _ in range(self.world)]
            keep = []
            for g in range(self.world):
                for h, (first, cnt) in self.ghost_block[g].items():
                    t_src = segs[h][k][1]
                    with torch.cuda.device(self.devices[h]):
                        buf = torch.empty((cnt, t_src.shape[1]), dtype=t_src.dtype, device=self.devices[h])
                        HaloComm.pack(t_src, self._send_rows[(h, g)], buf, stream=streams[h])
                    keep.append(buf)
                    sends[h][g] = buf
                    recvs[g][h] = segs[g][k][1][first: first + cnt]
            self._comms.exchange(sends, recvs, streams)
            del keep  # the caching allocator reuses them only behind the exchange on their stream

    def halo_bytes(self) -> Dict[str, int]:
        """Bytes one full halo exchange moves: total and the busiest ordered GPU pair."""
        row = sum(t.shape[1] * t.element_size() for _, t, _ in self.pools[0].segments())
        per = [cnt * row for g in range(self.world) for _, (_, cnt) in self.ghost_block[g].items()]
        return dict(total=int(sum(per)), busiest_pair=int(max(per or [0])))

    def close(self) -> None:
        if self._comms is not None:
            self._comms.close()
            self._comms = None


def devices_from_env() -> Optional[List[torch.device]]:
    """TAL_GPUS=N (N >= 2): GPUs 0..N-1 of this process; TAL_VIRTUAL_GPUS=N: N pools on the
    current GPU (one-GPU tests of the same code, copy transport).  None: one pool (default)."""
    import os

    v = os.environ.get("TAL_VIRTUAL_GPUS", "")
    if v and int(v) >= 2:
        return [torch.device("cuda", torch.cuda.current_device())] * int(v)
    n = os.environ.get("TAL_GPUS", "")
    if n and int(n) >= 2:
        if int(n) > torch.cuda.device_count():
            raise ValueError(f"TAL_GPUS={n} but {torch.cuda.device_count()} GPUs are visible")
        return [torch.device("cuda", k) for k in range(int(n))]
    return None
