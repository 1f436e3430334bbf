"""Checkpoints written from / read into the device model pool.

The reference saves {"client_state_dicts": [model.state_dict() for each client],
"round_idx": r, "client_results": [...]} with torch.save (reference src/utils.py:19-38) and
restores with load_state_dict per client (:41-56).  With the models living as rows of a
ModelPool in HBM, the whole checkpoint is one device-to-host copy per segment (per run of
consecutive rows) into pinned memory; the per-client state dicts are views into that host buffer (torch.save stores
the shared storage once), so the file has the reference's structure, keys, dtypes and shapes
and the reference's loader reads it unchanged.  Restoring is one host-to-device copy.
"""
from __future__ import annotations

import pathlib
from collections import OrderedDict
from typing import List, Optional, Sequence

import torch

from .arena import ModelPool


def pool_state_dicts_host(pool: ModelPool, rows: Sequence[int]) -> List["OrderedDict[str, torch.Tensor]"]:
    """State dicts of pool rows `rows` (in that order) as CPU tensors, copied with one D2H per
    segment (fp32, bf16, int64) through pinned memory."""
    rows = [int(r) for r in rows]
    lay = pool.layout
    pin = pool.device.type == "cuda"
    host = {id(t): torch.empty((len(rows), t.shape[1]), dtype=t.dtype, pin_memory=pin)
            for t in (pool.f32, pool.i64, pool.b16)}
    for _, src, _ in pool.segments():
        dst = host[id(src)]
        for a, b, r0 in _runs(rows):  # consecutive pool rows move as one copy (no device temp)
            dst[a:b].copy_(src[r0: r0 + b - a], non_blocking=pin)
    if pin:
        torch.cuda.current_stream(pool.device).synchronize()
    f32, i64, b16 = host[id(pool.f32)], host[id(pool.i64)], host[id(pool.b16)]
    return [lay.views(f32[k], i64[k], b16[k]) for k in range(len(rows))]


def _runs(rows):
    """(dst_begin, dst_end, first pool row) for each run of consecutive pool rows."""
    out, a = [], 0
    for k in range(1, len(rows) + 1):
        if k == len(rows) or rows[k] != rows[k - 1] + 1:
            out.append((a, k, rows[a]))
            a = k
    return out


def save_pool_checkpoint(path, round_idx: int, pool: ModelPool, rows: Sequence[int], client_results) -> None:
    """Write the reference's checkpoint format from pool rows (one D2H per run of consecutive
    rows: a single copy per segment for the usual rows 0..n-1)."""
    sds = pool_state_dicts_host(pool, rows)
    torch.save({"client_state_dicts": sds, "round_idx": round_idx, "client_results": client_results},
               pathlib.Path(path))


def load_state_dicts_into_pool(pool: ModelPool, rows: Sequence[int], state_dicts) -> None:
    """Flatten state dicts (reference checkpoint entries) into pool rows: host staging, then
    one H2D per segment."""
    lay = pool.layout
    pin = pool.device.type == "cuda"
    host = {id(t): torch.zeros((len(rows), t.shape[1]), dtype=t.dtype, pin_memory=pin)
            for t in (pool.f32, pool.i64, pool.b16)}
    f32, i64, b16 = host[id(pool.f32)], host[id(pool.i64)], host[id(pool.b16)]
    for k, sd in enumerate(state_dicts):
        lay.check_compatible(sd, "checkpoint state_dict")
        lay.flatten_into(sd, f32[k], i64[k], b16=b16[k])
    rows = [int(r) for r in rows]
    for _, dst, _ in pool.segments():
        src = host[id(dst)]
        for a, b, r0 in _runs(rows):
            dst[r0: r0 + b - a].copy_(src[a:b], non_blocking=pin)
    if pin:  # the pinned staging buffers must outlive the copies
        torch.cuda.current_stream(pool.device).synchronize()


def load_pool_checkpoint(path, pool: ModelPool, rows: Optional[Sequence[int]] = None):
    """Read a checkpoint (this framework's or the reference's) into pool rows (default
    0..len-1); returns (round_idx, client_results).  The file holds result dicts with
    datetimes, so it is loaded as a full pickle: only load checkpoints you wrote."""
    ckpt = torch.load(pathlib.Path(path), map_location="cpu", weights_only=False)
    sds = ckpt["client_state_dicts"]
    rows = list(range(len(sds))) if rows is None else list(rows)
    load_state_dicts_into_pool(pool, rows, sds)
    return ckpt["round_idx"], ckpt["client_results"]


def common_pool(models) -> Optional[tuple]:
    """(pool, rows) when every model is bound to rows of one ModelPool, else None."""
    from .arena import bound_row

    pool, rows = None, []
    for m in models:
        b = bound_row(m)
        if b is None or (pool is not None and b[0] is not pool):
            return None
        pool = b[0]
        rows.append(b[1])
    return (pool, rows) if pool is not None else None
