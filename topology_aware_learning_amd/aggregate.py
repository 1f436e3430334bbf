"""One aggregation call on the GPU: the body the reference's apps share
(src/decentralized_client.py:399-413), i.e.

    avg = sum_i w_i * state_dict(model_i)      (fp32 mul + fp32 add per operand, in order)
    target.load_state_dict(avg)                (int64 buffers truncated)

Operands and target may be
  * pool-bound models (``arena.ModelPool.bind``): zero copies, the kernel reads the operand
    rows and writes the target row in place (the target is normally the last operand itself);
  * any other models (CPU — as the reference leaves them after training, tasks.py:342 — or
    GPU): their state is packed into one pinned host buffer, copied H2D once, aggregated, and
    the result copied back into the target's own tensors, as load_state_dict would.
There is no CPU arithmetic path.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import ops
from .arena import StateLayout, bound_row

_tls = threading.local()
_layout_cache: dict = {}


def layout_of_module(model: nn.Module) -> StateLayout:
    sd = model.state_dict()
    key = tuple((k, tuple(v.shape), v.dtype) for k, v in sd.items())
    lay = _layout_cache.get(key)
    if lay is None:
        lay = StateLayout.from_state_dict(sd)
        _layout_cache[key] = lay
    return lay


def _device_for(models: Sequence[nn.Module]) -> torch.device:
    for m in models:
        b = bound_row(m)
        if b is not None:
            return b[0].device
    for m in models:
        for t in m.state_dict().values():
            if t.device.type == "cuda":
                return t.device
            break
    if not torch.cuda.is_available():
        raise RuntimeError("aggregation runs on the GPU (HIP library); no GPU is visible to this process")
    return torch.device("cuda", torch.cuda.current_device())


def _pinned(nbytes: int, tag: str) -> torch.Tensor:
    """Per-thread pinned staging buffer; waits until the last async copy that used it is done."""
    bufs = getattr(_tls, "pinned", None)
    if bufs is None:
        bufs = _tls.pinned = {}
        _tls.events = {}
    ev = _tls.events.get(tag)
    if ev is not None:
        ev.synchronize()
    b = bufs.get(tag)
    if b is None or b.numel() < nbytes:
        b = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
        bufs[tag] = b
    return b[:nbytes]


def _mark_used(tag: str, device) -> None:
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(device))
    _tls.events[tag] = ev


def _stage(models: Sequence[nn.Module], layout: StateLayout, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Pack non-bound models' f32 / i64 segments into [k, n] device tensors.

    Models already on `device` are packed there; the others go through one pinned host buffer
    and a single H2D copy per segment (the host-memory path of the reference's CPU models)."""
    k = len(models)
    nf, ni = layout.n_f32, layout.n_i64
    df = torch.empty(k, nf, dtype=torch.float32, device=device)
    di = torch.empty(k, max(ni, 1), dtype=torch.int64, device=device)
    host_rows = []
    sds = []
    for j, m in enumerate(models):
        sd = m.state_dict()
        layout.check_compatible(sd, f"operand {j}")
        sds.append(sd)
        if all(t.device == device for t in sd.values()):
            fl = layout.flatten_cat(sd, "f32")
            if fl:
                torch.cat(fl, out=df[j])
            il = layout.flatten_cat(sd, "i64")
            if il:
                torch.cat(il, out=di[j, :ni])
        else:
            host_rows.append(j)
    if host_rows:
        h = len(host_rows)
        hf = _pinned(4 * h * max(nf, 1), "in_f32").view(torch.float32).view(h, max(nf, 1))
        hi = _pinned(8 * h * max(ni, 1), "in_i64").view(torch.int64).view(h, max(ni, 1))
        for q, j in enumerate(host_rows):
            fl = layout.flatten_cat(sds[j], "f32")
            if fl:
                torch.cat([t.detach().to("cpu") for t in fl], out=hf[q, :nf])
            il = layout.flatten_cat(sds[j], "i64")
            if il:
                torch.cat([t.detach().to("cpu") for t in il], out=hi[q, :ni])
        idx = torch.tensor(host_rows, dtype=torch.long, device=device)
        if nf:
            df.index_copy_(0, idx, hf[:, :nf].to(device, non_blocking=True))
        if ni:
            di.index_copy_(0, idx, hi.to(device, non_blocking=True))
        _mark_used("in_f32", device)
        _mark_used("in_i64", device)
    return df, di


def aggregate_models(operands: Sequence[nn.Module], weights: Sequence[float], target: nn.Module,
                     mode: int = ops.MODE_EXACT) -> nn.Module:
    """target <- sum_i weights[i] * operands[i] (state_dict-wise), reference semantics."""
    if len(operands) == 0:
        raise ValueError("no operands")
    if len(weights) != len(operands):
        raise ValueError("one weight per operand is required")
    layout = layout_of_module(target)
    device = _device_for(list(operands) + [target])

    f32_ptrs: List[Optional[torch.Tensor]] = [None] * len(operands)
    i64_ptrs: List[Optional[torch.Tensor]] = [None] * len(operands)
    unbound = []
    for j, m in enumerate(operands):
        b = bound_row(m)
        if b is not None and b[0].device == device and b[0].layout == layout:
            pool, r = b
            f32_ptrs[j] = pool.row_f32(r)
            i64_ptrs[j] = pool.row_i64(r)
        else:
            unbound.append(j)
    if unbound:
        df, di = _stage([operands[j] for j in unbound], layout, device)
        for k, j in enumerate(unbound):
            f32_ptrs[j] = df[k]
            i64_ptrs[j] = di[k, : layout.n_i64]

    tb = bound_row(target)
    if tb is not None and tb[0].device == device and tb[0].layout == layout:
        out_f = tb[0].row_f32(tb[1])
        out_i = tb[0].row_i64(tb[1])
        in_place = True
    else:
        out_f = torch.empty(layout.n_f32, dtype=torch.float32, device=device)
        out_i = torch.empty(layout.n_i64, dtype=torch.int64, device=device)
        in_place = False

    w = [float(x) for x in weights]
    if layout.n_f32:
        ops.agg_f32(f32_ptrs, w, out_f, mode=mode)
    if layout.n_i64:
        ops.agg_i64(i64_ptrs, w, out_i)

    if not in_place:
        _write_back(target, layout, out_f, out_i)
    return target


def _write_back(target: nn.Module, layout: StateLayout, out_f: torch.Tensor, out_i: torch.Tensor) -> None:
    """load_state_dict(avg) equivalent: copy_ into the target's existing tensors."""
    sd = target.state_dict()
    on_gpu = [t.device.type == "cuda" for t in sd.values()]
    if all(on_gpu):
        views = layout.views(out_f, out_i)
        with torch.no_grad():
            for name, t in sd.items():
                t.copy_(views[name])
        return
    hf = _pinned(4 * max(layout.n_f32, 1), "out_f32").view(torch.float32)[: layout.n_f32]
    hi = _pinned(8 * max(layout.n_i64, 1), "out_i64").view(torch.int64)[: layout.n_i64]
    hf.copy_(out_f, non_blocking=True)
    hi.copy_(out_i, non_blocking=True)
    torch.cuda.current_stream(out_f.device).synchronize()  # host reads hf / hi next
    views = layout.views(hf, hi)
    with torch.no_grad():
        for name, t in sd.items():
            t.copy_(views[name])
