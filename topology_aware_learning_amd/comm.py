"""The halo exchange through the C-ABI (include/tal_agg.h, halo section): one RCCL communicator
per process, a gather kernel that packs the rows a peer needs into one contiguous message, and
one RCCL group of per-peer sends / receives.

This is the binding a host without torch.distributed would use;
`ShardedRound(transport="cabi")` runs a sharded round through it.  The default multi-GPU path
(`distributed.post_exchange`) moves the same per-peer messages with torch.distributed's RCCL.
"""
from __future__ import annotations

import ctypes
import sys
from typing import Optional, Sequence

import torch

from . import _lib


def _check(rc: int) -> None:
    _lib.check(rc)


class HaloComm:
    """An RCCL communicator of `world` ranks made by the C-ABI on `device`.

    uid: the TAL_COMM_ID_BYTES bytes of HaloComm.unique_id() made once by rank 0 and shared by
    the caller with every rank (torch.distributed.broadcast_object_list, a file, ...)."""

    def __init__(self, world: int, rank: int, uid: bytes, device):
        if len(uid) != _lib.TAL_COMM_ID_BYTES:
            raise ValueError(f"the unique id is {_lib.TAL_COMM_ID_BYTES} bytes")
        self.world, self.rank = int(world), int(rank)
        self.device = torch.device(device)
        if self.device.index is None:  # "cuda": the current device
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._comm = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(bytes(uid), len(uid))
        _check(_lib.load().tal_comm_init(ctypes.byref(self._comm), self.world, self.rank, idbuf,
                                         self.device.index))

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(_lib.TAL_COMM_ID_BYTES)
        _check(_lib.load().tal_comm_unique_id(buf))
        return buf.raw

    def close(self) -> None:
        if self._comm:
            _check(_lib.load().tal_comm_destroy(self._comm))
            self._comm = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter teardown order
        # at interpreter exit the HIP runtime may already be torn down: leave the communicator
        # to the process exit instead of calling into RCCL
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def pack(seg: torch.Tensor, rows: torch.Tensor, out: torch.Tensor,
             stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        """out[k] = seg[rows[k]] for a [pool_rows, ld] segment and device int32 `rows` (the rows
        a peer needs, in its receive order); out is [len(rows), ld]."""
        if rows.dtype != torch.int32 or rows.device != seg.device or out.device != seg.device:
            raise ValueError("rows must be a device int32 tensor on the pool's device")
        if seg.dim() != 2 or not seg.is_contiguous() or out.shape != (rows.numel(), seg.shape[1]) \
                or out.dtype != seg.dtype or not out.is_contiguous():
            raise ValueError("seg [rows, ld] contiguous and out [len(rows), ld] of its dtype")
        es = seg.element_size()
        s = (stream or torch.cuda.current_stream(seg.device)).cuda_stream
        _check(_lib.load().tal_halo_pack(seg.data_ptr(), seg.stride(0) * es, seg.shape[0], rows.data_ptr(),
                                         rows.numel(), seg.shape[1] * es, out.data_ptr(), s))
        return out

    def exchange(self, sends: Sequence[Optional[torch.Tensor]], recvs: Sequence[Optional[torch.Tensor]],
                 stream: Optional[torch.cuda.Stream] = None) -> None:
        """One RCCL group: sends[p] to peer p and recvs[p] from peer p (None: nothing), each a
        contiguous device tensor on this communicator's device, enqueued on `stream`."""
        if len(sends) != self.world or len(recvs) != self.world:
            raise ValueError("one send and one receive entry per rank")
        sb = (ctypes.c_void_p * self.world)()
        rb = (ctypes.c_void_p * self.world)()
        sn = (ctypes.c_int64 * self.world)()
        rn = (ctypes.c_int64 * self.world)()
        for p in range(self.world):
            for t, b, n in ((sends[p], sb, sn), (recvs[p], rb, rn)):
                if t is None or t.numel() == 0:
                    continue
                if not t.is_contiguous() or t.device != self.device:
                    raise ValueError("exchange buffers are contiguous tensors on the communicator's device")
                b[p] = t.data_ptr()
                n[p] = t.numel() * t.element_size()
        s = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        _check(_lib.load().tal_halo_exchange(self._comm, self.world, sb, sn, rb, rn, s))


def shared_halo_comm(world: int, rank: int, device, group=None) -> HaloComm:
    """A HaloComm over the ranks of an initialised torch.distributed group: the group's first
    member makes the unique id and broadcasts it through the group.

    `rank` is the shard rank the communicator uses; who creates the id and where the broadcast
    comes from are decided by group membership (a group need not contain global rank 0, and a
    shard rank need not equal the group rank)."""
    import torch.distributed as dist

    grank = dist.get_rank(group) if group is not None else dist.get_rank()
    src = dist.get_global_rank(group, 0) if group is not None else 0
    obj = [HaloComm.unique_id() if grank == 0 else None]
    dist.broadcast_object_list(obj, src=src, group=group)
    return HaloComm(world, rank, obj[0], device)
