"""One aggregation call on the GPU: the body the reference's apps share
(src/decentralized_client.py:399-413), i.e.

    avg = sum_i w_i * state_dict(model_i)      (fp32 mul + fp32 add per operand, in order;
                                                bf16 entries rounded to bf16 after each op)
    target.load_state_dict(avg)                (int64 buffers truncated)

Operands and target may be
  * pool-bound models (``arena.ModelPool.bind``): zero copies, the kernel reads the operand
    rows and writes the target row in place (the target is normally the last operand itself);
  * any other models (CPU — as the reference leaves them after training, tasks.py:342 — or
    GPU): their state is packed into one pinned host buffer, copied H2D once, aggregated, and
    the result copied back into the target's own tensors, as load_state_dict would.
A process that sees no GPU (BASELINE config 1: the reference's driver on CPU models, no GPU)
runs the library's host reduction instead (tal_host_agg_*, native code with the kernels'
arithmetic); with a GPU visible every call runs the HIP kernels.  Without the library either
way raises TalLibraryError.
"""
from __future__ import annotations

import os
import threading
import weakref
from collections import OrderedDict
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import ops
from .arena import ModelPool, StateLayout, bound_row

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
        if b is not None and b[0].device.type == "cuda":  # (pinned host rows: TAL_HOST_PIN)
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


_SEG_DTYPE = {"f32": torch.float32, "b16": torch.bfloat16, "i64": torch.int64}
_D2H_CHUNK = 16 << 20  # bytes per write-back chunk


def _seg_sizes(layout: StateLayout):
    return {"f32": layout.n_f32, "b16": layout.n_b16, "i64": layout.n_i64}


class _OperandCache:
    """Opt-in (TAL_HOST_CACHE_GB > 0) device copies of host-memory operand models.

    In a round of the reference's per-call apps on CPU models every model is an operand of up
    to M calls, and each call would copy it host -> device again.  An entry is reused only while
    the model object is alive (weak reference) and every state tensor has the data pointer and
    version counter it had when it was copied: training steps, load_state_dict, this module's
    own write-back and module.to() all change one of them.  What it cannot see is an in-place
    write through `tensor.data` (a detached alias with its own version counter), hence opt-in.
    The aggregating model's result is kept as its entry after the write-back, so a later call
    that reads it as a neighbor copies nothing."""

    def __init__(self, cap_bytes: int):
        self.cap = cap_bytes
        self.used = 0
        # re-entrant: put() allocates under the lock, which can run cyclic GC, whose collection
        # of a cached model calls _drop on this same thread
        self.lock = threading.RLock()
        self.entries: "OrderedDict[int, tuple]" = OrderedDict()  # id -> (wref, sig, device, segs, nbytes)
        self.hits = self.misses = 0

    @staticmethod
    def signature(sd) -> tuple:
        return tuple((t.data_ptr(), t._version) for t in sd.values())

    def get(self, model: nn.Module, sig: tuple, device):
        with self.lock:
            ent = self.entries.get(id(model))
            if ent is not None and ent[0]() is model and ent[1] == sig and ent[2] == device:
                self.entries.move_to_end(id(model))
                self.hits += 1
                return ent[3]
            self.misses += 1
            return None

    def put(self, model: nn.Module, sig: tuple, device, segs: dict) -> None:
        nbytes = sum(t.numel() * t.element_size() for t in segs.values())
        if nbytes > self.cap:
            return
        with self.lock:
            old = self.entries.pop(id(model), None)
            if old is not None:
                self.used -= old[4]
            while self.entries and self.used + nbytes > self.cap:
                self.used -= self.entries.popitem(last=False)[1][4]
            key = id(model)
            wref = weakref.ref(model, lambda _r, k=key: self._drop(k, _r))
            self.entries[key] = (wref, sig, device, segs, nbytes)
            self.used += nbytes

    def _drop(self, key: int, wref) -> None:
        with self.lock:
            ent = self.entries.get(key)
            if ent is not None and ent[0] is wref:
                self.used -= ent[4]
                del self.entries[key]


def _host_cache() -> Optional[_OperandCache]:
    global _CACHE
    gb = float(os.environ.get("TAL_HOST_CACHE_GB", "0") or 0)
    if gb <= 0:
        return None
    if _CACHE is None or _CACHE.cap != int(gb * (1 << 30)):
        _CACHE = _OperandCache(int(gb * (1 << 30)))
    return _CACHE


_CACHE: Optional[_OperandCache] = None


def _pipe_enabled() -> bool:
    """The chunked H2D / K1 / D2H pipeline for all-pinned host calls (TAL_HOST_PIPE=0: one
    stream, whole segments)."""
    return os.environ.get("TAL_HOST_PIPE", "1") not in ("", "0")


def _pin_enabled() -> bool:
    """Pinned binding of CPU models is the default since round 4 (TAL_HOST_PIN=0 opts out)."""
    return os.environ.get("TAL_HOST_PIN", "1") not in ("", "0")


def _host_binding(model: nn.Module, layout: StateLayout) -> Optional[Tuple[ModelPool, int]]:
    """(pool, row) of a model whose state lives in a pinned host row, or None.

    By default (TAL_HOST_PIN unset or 1; 0 opts out) a model whose state is on the CPU and not
    bound anywhere is bound first: its state is copied once into a pinned one-row host pool and
    its parameters / buffers become views of that row (ModelPool.bind, as for device pools).
    The call then moves its operands host -> device and its result device -> host as one DMA
    per segment straight from / into the row - no packing of 320 tensors into a staging buffer
    and no unpacking copy afterwards (round 3: 25.5 ms per config-3 call packing, the PCIe
    floor ~17 ms).  A model whose tensors are replaced later (module.to(), load_state_dict
    into new tensors) fails the binding check and is bound again on its next call; if pinned
    memory cannot be allocated the call packs as before."""
    b = bound_row(model)
    if b is not None:
        return b if b[0].device.type == "cpu" and b[0].layout == layout else None
    if not _pin_enabled():
        return None
    with _bind_lock:  # the reference runs two app calls at once; bind a shared operand once
        b = bound_row(model)
        if b is not None:
            return b if b[0].device.type == "cpu" and b[0].layout == layout else None
        return _bind_pinned(model, layout)


# re-entrant: a pool freed by garbage collection while this thread binds (weakref.finalize ->
# _pin_release) takes it again on the same thread
_bind_lock = threading.RLock()
_PIN = {"used": 0, "budget": None}


def _pin_budget() -> int:
    """Bytes of page-locked host memory the pinned bindings may hold at once: TAL_HOST_PIN_GB,
    else a quarter of the host memory available when the first model is bound (page-locked
    memory cannot be swapped or reclaimed, so tens of ViT-sized models must not take it all).
    Past the budget a model is packed per call as with TAL_HOST_PIN=0."""
    gb = os.environ.get("TAL_HOST_PIN_GB", "")
    if gb:
        return int(float(gb) * (1 << 30))
    if _PIN["budget"] is None:
        avail = 0
        try:
            with open("/proc/meminfo") as f:
                for line in f:
                    if line.startswith("MemAvailable:"):
                        avail = int(line.split()[1]) * 1024
                        break
        except OSError:
            pass
        _PIN["budget"] = avail // 4 if avail else 16 << 30
    return int(_PIN["budget"])


def _pin_release(nbytes: int) -> None:
    # weakref.finalize runs on whichever thread collects the pool: the same lock as the binder's
    with _bind_lock:
        _PIN["used"] -= nbytes


def _bind_pinned(model: nn.Module, layout: StateLayout) -> Optional[Tuple[ModelPool, int]]:
    sd = model.state_dict()
    if not sd or any(t.device.type != "cpu" for t in sd.values()):
        return None
    try:
        layout.check_compatible(sd, "model")
    except ValueError:
        return None
    nbytes = 4 * layout.ld_f32 + 8 * layout.ld_i64 + 2 * layout.ld_b16
    if _PIN["used"] + nbytes > _pin_budget():
        return None

    def pinned(rows_ld, dtype):
        return torch.empty((1, rows_ld), dtype=dtype, pin_memory=rows_ld > 0)

    try:
        pool = ModelPool(layout, 1, "cpu", f32=pinned(layout.ld_f32, torch.float32),
                         i64=pinned(layout.ld_i64, torch.int64), b16=pinned(layout.ld_b16, torch.bfloat16))
    except RuntimeError:  # no pinned memory to be had (locked-memory limit): pack instead
        return None
    _PIN["used"] += nbytes
    weakref.finalize(pool, _pin_release, nbytes)  # the row lives as long as the model bound to it
    pool.bind(model, 0)
    return pool, 0


def _pinned_signature(model: nn.Module, pool: ModelPool) -> tuple:
    """Cache signature of a pinned-bound model: its row (binding already checked by bound_row)
    and the version counter of every bound tensor (training steps bump them)."""
    return (pool.f32.data_ptr(),) + tuple(table[attr]._version for table, attr in model._tal_slots)


def _row_segments(pool: ModelPool, r: int, sizes) -> dict:
    rows = {"f32": pool.row_f32, "b16": pool.row_b16, "i64": pool.row_i64}
    return {g: rows[g](r) for g in sizes}


def _stage(models: Sequence[nn.Module], layout: StateLayout, device) -> List[dict]:
    """Each non-bound model's segments as flat device tensors ({segment: [n]} per model).

    Models already on `device` are packed there; the others are packed into one pinned host
    buffer per segment, each operand's H2D copy issued as soon as that operand is packed so the
    copy overlaps packing the next one (the host-memory path of the reference's CPU models);
    with TAL_HOST_CACHE_GB set, an unchanged host model copied before is not copied again."""
    sizes = {g: n for g, n in _seg_sizes(layout).items() if n}
    cache = _host_cache()
    out: List[dict] = [None] * len(models)  # type: ignore[list-item]
    host_rows, sds, sigs = [], [], []
    for j, m in enumerate(models):
        hb = _host_binding(m, layout)
        if hb is not None:  # pinned row: one H2D per segment straight from it
            sig = _pinned_signature(m, hb[0]) if cache is not None else None
            hit = cache.get(m, sig, device) if cache is not None else None
            if hit is not None:
                out[j] = hit
                continue
            src = _row_segments(hb[0], hb[1], sizes)
            out[j] = {g: torch.empty(n, dtype=_SEG_DTYPE[g], device=device) for g, n in sizes.items()}
            for g in sizes:
                out[j][g].copy_(src[g], non_blocking=True)
            if cache is not None:
                cache.put(m, sig, device, out[j])
            sds.append(None)
            sigs.append(None)
            continue
        sd = m.state_dict()
        layout.check_compatible(sd, f"operand {j}")
        sds.append(sd)
        sigs.append(None)
        if all(t.device == device for t in sd.values()):
            out[j] = {g: torch.cat(layout.flatten_cat(sd, g)) for g in sizes}
            continue
        if cache is not None:
            sigs[j] = _OperandCache.signature(sd)
            hit = cache.get(m, sigs[j], device)
            if hit is not None:
                out[j] = hit
                continue
        host_rows.append(j)
    if host_rows:
        h = len(host_rows)
        for j in host_rows:
            out[j] = {g: torch.empty(n, dtype=_SEG_DTYPE[g], device=device) for g, n in sizes.items()}
        for g, n in sizes.items():
            esz = torch.empty((), dtype=_SEG_DTYPE[g]).element_size()
            hb = _pinned(esz * h * n, "in_" + g).view(_SEG_DTYPE[g]).view(h, n)
            for q, j in enumerate(host_rows):
                torch.cat([t.detach().to("cpu") for t in layout.flatten_cat(sds[j], g)], out=hb[q])
                out[j][g].copy_(hb[q], non_blocking=True)  # in flight while the next one packs
            _mark_used("in_" + g, device)
        if cache is not None:
            for j in host_rows:
                cache.put(models[j], sigs[j], device, out[j])
    return out


# The host-memory call (every model in a pinned host row) as a pipeline over column chunks:
# chunk c's operand H2Ds, its K1 and its result's D2H run on three streams, so the D2H of one
# chunk and the K1 of another overlap the H2D of the next (PCIe is full duplex).  The
# unpipelined form queues all H2Ds, then K1, then the D2H on one stream.
_PIPE_CHUNK = 4 << 20  # elements per chunk of a float segment (16 MiB fp32)
_PIPE_STREAMS: dict = {}


def _pipe_streams(device: torch.device):
    key = (device.index, threading.get_ident())  # per thread: the reference runs two calls at once
    st = _PIPE_STREAMS.get(key)
    if st is None:
        st = _PIPE_STREAMS[key] = tuple(torch.cuda.Stream(device) for _ in range(3))
    return st


def _k1(g: str, xs, w, out, mode, stream) -> None:
    if g == "i64":
        ops.agg_i64(xs, w, out, stream=stream)
    elif g == "b16":
        ops.agg_bf16(xs, w, out, mode=mode, stream=stream)
    else:
        ops.agg_f32(xs, w, out, mode=mode, stream=stream)


def _pipelined_host_call(hbs, target_hb, layout: StateLayout, w: List[float], mode: int, device) -> None:
    """target's row <- sum_i w_i * row of hbs[i], every model a pinned host row (the reference's
    CPU models after their first call): per segment, column chunks flow H2D -> K1 -> D2H on three
    streams.  K1 on a chunk is the same per-element arithmetic as on the whole segment."""
    sizes = {g: n for g, n in _seg_sizes(layout).items() if n}
    h2d, comp, d2h = _pipe_streams(device)
    start = torch.cuda.Event()
    start.record(torch.cuda.current_stream(device))
    for st in (h2d, comp, d2h):
        st.wait_event(start)
    m = len(hbs)
    src = [_row_segments(hb[0], hb[1], sizes) for hb in hbs]
    dst = _row_segments(target_hb[0], target_hb[1], sizes)
    keep = []
    try:
        for g, n in sizes.items():
            ld = (n + 63) // 64 * 64  # 256-B aligned operand rows: chunks keep K1's vector path
            dev = torch.empty((m, ld), dtype=_SEG_DTYPE[g], device=device)
            out = torch.empty(ld, dtype=_SEG_DTYPE[g], device=device)
            keep += [dev, out]
            step = n if g == "i64" else _PIPE_CHUNK
            for a in range(0, n, step):
                b = min(n, a + step)
                with torch.cuda.stream(h2d):
                    for j in range(m):
                        dev[j, a:b].copy_(src[j][g][a:b], non_blocking=True)
                landed = torch.cuda.Event()
                landed.record(h2d)
                comp.wait_event(landed)
                _k1(g, [dev[j, a:b] for j in range(m)], w, out[a:b], mode, comp)
                done = torch.cuda.Event()
                done.record(comp)
                d2h.wait_event(done)
                with torch.cuda.stream(d2h):
                    dst[g][a:b].copy_(out[a:b], non_blocking=True)
    finally:
        # the call returns with the model written, as the reference's load_state_dict; and if a
        # launch or copy raised part way, no queued copy may still touch `keep` (allocated on the
        # caller's stream, used on the three side streams) once the allocator gets it back
        for st in (h2d, comp, d2h):
            st.synchronize()
        del keep


_AGG = {"f32": lambda xs, w, out, mode: ops.agg_f32(xs, w, out, mode=mode),
        "b16": lambda xs, w, out, mode: ops.agg_bf16(xs, w, out, mode=mode),
        "i64": lambda xs, w, out, mode: ops.agg_i64(xs, w, out)}


def aggregate_models(operands: Sequence[nn.Module], weights: Sequence[float], target: nn.Module,
                     mode: int = ops.MODE_EXACT) -> nn.Module:
    """target <- sum_i weights[i] * operands[i] (state_dict-wise), reference semantics (bf16
    entries: the reference's ops on bf16 tensors in MODE_EXACT)."""
    if len(operands) == 0:
        raise ValueError("no operands")
    if len(weights) != len(operands):
        raise ValueError("one weight per operand is required")
    if not torch.cuda.is_available():
        return _aggregate_host(operands, weights, target, mode)
    # pool-bound models are checked once each (bound_row: every entry still a view of its
    # row); the target's pool then gives the layout without rebuilding its state_dict
    tb = bound_row(target)
    bounds = [bound_row(m) for m in operands]
    mp = getattr(tb[0], "multi", None) if tb is not None else None
    if mp is not None and all(b is not None and mp[0].member(b[0]) is not None for b in bounds):
        # the driver's clients over several GPUs (multipool.MultiPool, TAL_GPUS): the operands
        # other GPUs own are copied into this GPU's ghost rows, then K1 on rows of one pool
        with torch.cuda.device(tb[0].device):
            rows = mp[0].rows_for(mp[1], bounds)
            ops.agg_pool_rows(tb[0], rows, [float(x) for x in weights], tb[1], mode)
        return target
    if tb is not None and tb[0].device.type == "cuda" and all(b is not None and b[0] is tb[0] for b in bounds):
        # every model a row of one device pool (the driver's binding): K1 on the rows in place,
        # addresses from the pool instead of a view per row and segment
        ops.agg_pool_rows(tb[0], [b[1] for b in bounds], [float(x) for x in weights], tb[1], mode)
        return target
    layout = tb[0].layout if tb is not None else layout_of_module(target)
    device = next((b[0].device for b in [tb, *bounds] if b is not None and b[0].device.type == "cuda"), None)
    if device is None:
        device = _device_for(list(operands) + [target])
    host_target = _host_binding(target, layout) if tb is None or tb[0].device.type == "cpu" else None
    sizes = {g: n for g, n in _seg_sizes(layout).items() if n}
    if host_target is not None and _host_cache() is None and _pipe_enabled():
        hbs = [_host_binding(m, layout) for m in operands]
        if all(h is not None for h in hbs):  # every model in a pinned host row
            _pipelined_host_call(hbs, host_target, layout, [float(x) for x in weights], mode, device)
            return target

    ptrs: dict = {g: [None] * len(operands) for g in sizes}
    unbound = []
    for j, m in enumerate(operands):
        b = bounds[j]
        if b is not None and b[0].device == device and b[0].layout == layout:  # device pool row
            pool, r = b
            rows = {"f32": pool.row_f32, "b16": pool.row_b16, "i64": pool.row_i64}
            for g in sizes:
                ptrs[g][j] = rows[g](r)
        else:
            unbound.append(j)
    if unbound:
        staged = _stage([operands[j] for j in unbound], layout, device)
        for k, j in enumerate(unbound):
            for g in sizes:
                ptrs[g][j] = staged[k][g]

    if tb is not None and tb[0].device == device and tb[0].layout == layout:
        rows = {"f32": tb[0].row_f32, "b16": tb[0].row_b16, "i64": tb[0].row_i64}
        outs = {g: rows[g](tb[1]) for g in sizes}
        in_place = True
    else:
        outs = {g: torch.empty(n, dtype=_SEG_DTYPE[g], device=device) for g, n in sizes.items()}
        in_place = False

    w = [float(x) for x in weights]
    if set(sizes) == {"f32", "i64"}:  # a ResNet-like model: both segments in one launch
        ops.agg_model_f32(ptrs["f32"], ptrs["i64"], w, outs["f32"], outs["i64"], mode)
    else:
        for g in sizes:
            _AGG[g](ptrs[g], w, outs[g], mode)

    synced = False
    if host_target is not None:  # pinned row: one D2H per segment straight into it
        dst = _row_segments(host_target[0], host_target[1], sizes)
        for g in sizes:
            dst[g].copy_(outs[g], non_blocking=True)
        torch.cuda.current_stream(device).synchronize()
        synced = True
        cache = _host_cache()
        if cache is not None:
            cache.put(target, _pinned_signature(target, host_target[0]), device, outs)
    elif not in_place:
        _write_back(target, layout, outs)
        cache = _host_cache()
        if cache is not None:  # the target's new state is this output: its next use copies nothing
            sd = target.state_dict()
            if not all(t.device == device for t in sd.values()):
                cache.put(target, _OperandCache.signature(sd), device, outs)
    if unbound and not synced and _pin_enabled():
        # H2D copies straight from pinned rows (live model storage) may still be in flight: the
        # caller may train that model as soon as this returns, whatever the target's placement
        torch.cuda.current_stream(device).synchronize()
    return target


def _write_back(target: nn.Module, layout: StateLayout, outs: dict) -> None:
    """load_state_dict(avg) equivalent: copy_ into the target's existing tensors."""
    sd = target.state_dict()
    empty = {g: torch.empty(0, dtype=_SEG_DTYPE[g]) for g in _SEG_DTYPE}
    on_gpu = [t.device.type == "cuda" for t in sd.values()]
    if all(on_gpu):
        segs = {g: outs.get(g, empty[g]) for g in _SEG_DTYPE}
        views = layout.views(segs["f32"], segs["i64"], segs["b16"])
        with torch.no_grad():
            for name, t in sd.items():
                t.copy_(views[name])
        return
    # D2H in chunks of whole entries (~_D2H_CHUNK bytes), each with its own event: the host
    # copies a chunk's entries into the model while later chunks are still in flight
    host = dict(empty)
    pending = []  # (event, entry names)
    for g, o in outs.items():
        esz = o.element_size()
        host[g] = _pinned(esz * max(o.numel(), 1), "out_" + g).view(o.dtype)[: o.numel()]
        stream = torch.cuda.current_stream(o.device)
        ents = [e for e in layout.entries if e.seg == g and e.alias_of is None]
        names, start = [], 0
        for k, e in enumerate(ents):
            names.append(e.name)
            end = e.offset + e.numel
            if (end - start) * esz >= _D2H_CHUNK or k == len(ents) - 1:
                host[g][start:end].copy_(o[start:end], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(stream)
                pending.append((ev, names))
                names, start = [], end
    views = layout.views(host["f32"], host["i64"], host["b16"])
    with torch.no_grad():
        for ev, names in pending:
            ev.synchronize()
            for name in names:
                sd[name].copy_(views[name])
        for e in layout.entries:  # tied keys share storage; copy_ as load_state_dict would
            if e.alias_of is not None:
                sd[e.name].copy_(views[e.name])


def _aggregate_host(operands: Sequence[nn.Module], weights: Sequence[float], target: nn.Module,
                    mode: int) -> nn.Module:
    """No GPU visible: each operand's segments packed into flat CPU tensors, the library's host
    reduction (ops.host_agg), and the result copied into the target's own tensors as
    load_state_dict(avg) would (decentralized_client.py:399-413 on CPU models)."""
    layout = layout_of_module(target)
    sizes = {g: n for g, n in _seg_sizes(layout).items() if n}
    flats = []
    for j, m in enumerate(operands):
        sd = m.state_dict()
        layout.check_compatible(sd, f"operand {j}")
        if any(t.device.type != "cpu" for t in sd.values()):
            raise RuntimeError("no GPU is visible, but an operand has tensors off the CPU")
        flats.append({g: torch.cat([t.detach() for t in layout.flatten_cat(sd, g)]) for g in sizes})
    w = [float(x) for x in weights]
    outs = {g: torch.empty(n, dtype=_SEG_DTYPE[g]) for g, n in sizes.items()}
    for g in sizes:
        ops.host_agg([f[g] for f in flats], w, outs[g], mode)
    empty = {g: torch.empty(0, dtype=_SEG_DTYPE[g]) for g in _SEG_DTYPE}
    views = layout.views(outs.get("f32", empty["f32"]), outs.get("i64", empty["i64"]), outs.get("b16", empty["b16"]))
    sd = target.state_dict()
    with torch.no_grad():
        for name, t in sd.items():
            t.copy_(views[name])
    return target
