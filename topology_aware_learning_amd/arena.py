"""Flattened state_dict layout and the device-resident model pool.

A model's state_dict is split into flat segments: every fp32 entry back to back (the "f32
segment", where the kernels stream), every bf16 entry (the "b16 segment", bf16 models) and every
int64 entry (the "i64 segment", num_batches_tracked counters).  A ``ModelPool`` holds many
models of one layout as rows of 2-D device tensors ``f32[rows, ld_f32]`` / ``b16[rows, ld_b16]``
/ ``i64[rows, ld_i64]`` (fp32 rows 256-B aligned, bf16 rows 128-B aligned), and can
rebind an ``nn.Module``'s parameters and buffers to views of a row — so training, optimizers and
the aggregation kernels all work on the same HBM bytes, with no pack/unpack per call
(SURVEY §7 "state_dict flattening without re-packing every call", §8(f) rank 1).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Callable, Dict, List, Mapping, Optional, Sequence, Tuple

import torch
import torch.nn as nn

SUPPORTED = {torch.float32: "f32", torch.int64: "i64", torch.bfloat16: "b16"}
ROW_ALIGN = 64  # elements: 256 B for fp32 rows, 128 B for bf16 rows


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


@dataclass(frozen=True)
class Entry:
    name: str
    shape: Tuple[int, ...]
    dtype: torch.dtype
    seg: str          # "f32" | "b16" | "i64"
    offset: int       # element offset inside its segment
    numel: int
    alias_of: Optional[str] = None  # tied entry (same storage as an earlier key)


class StateLayout:
    """Segments of a state_dict (entry order = state_dict order)."""

    def __init__(self, entries: Sequence[Entry]):
        self.entries: List[Entry] = list(entries)
        self.by_name: Dict[str, Entry] = {e.name: e for e in self.entries}
        self.n_f32 = sum(e.numel for e in self.entries if e.seg == "f32" and e.alias_of is None)
        self.n_i64 = sum(e.numel for e in self.entries if e.seg == "i64" and e.alias_of is None)
        self.n_b16 = sum(e.numel for e in self.entries if e.seg == "b16" and e.alias_of is None)
        self.ld_f32 = max(_round_up(self.n_f32, ROW_ALIGN), ROW_ALIGN)
        self.ld_i64 = max(_round_up(self.n_i64, 8), 8)
        self.ld_b16 = max(_round_up(self.n_b16, ROW_ALIGN), ROW_ALIGN)
        self.key = tuple((e.name, e.shape, str(e.dtype), e.alias_of) for e in self.entries)

    def __eq__(self, other) -> bool:
        return isinstance(other, StateLayout) and self.key == other.key

    def __hash__(self) -> int:
        return hash(self.key)

    @classmethod
    def from_state_dict(cls, sd: Mapping[str, torch.Tensor]) -> "StateLayout":
        entries: List[Entry] = []
        off = {"f32": 0, "i64": 0, "b16": 0}
        seen: Dict[Tuple[int, int, Tuple[int, ...]], str] = {}
        for name, t in sd.items():
            if t.dtype not in SUPPORTED:
                raise NotImplementedError(
                    f"state_dict entry {name!r} has dtype {t.dtype}; the aggregation kernels handle "
                    "float32, bfloat16 and int64 entries")
            seg = SUPPORTED[t.dtype]
            key = (t.data_ptr(), t.storage_offset(), tuple(t.shape)) if t.numel() else None
            if key is not None and key in seen and t.is_contiguous():
                entries.append(Entry(name, tuple(t.shape), t.dtype, seg, by_name_offset(entries, seen[key]),
                                     t.numel(), alias_of=seen[key]))
                continue
            entries.append(Entry(name, tuple(t.shape), t.dtype, seg, off[seg], t.numel()))
            off[seg] += t.numel()
            if key is not None:
                seen[key] = name
        return cls(entries)

    @classmethod
    def from_layout(cls, layout: Sequence[Tuple[str, Sequence[int], str]]) -> "StateLayout":
        dt = {"float32": torch.float32, "int64": torch.int64, "bfloat16": torch.bfloat16}
        sd = OrderedDict((n, torch.empty(tuple(s), dtype=dt[d], device="meta")) for n, s, d in layout)
        entries: List[Entry] = []
        off = {"f32": 0, "i64": 0, "b16": 0}
        for name, t in sd.items():
            seg = SUPPORTED[t.dtype]
            n = 1
            for s in t.shape:
                n *= int(s)
            entries.append(Entry(name, tuple(t.shape), t.dtype, seg, off[seg], n))
            off[seg] += n
        return cls(entries)

    def check_compatible(self, sd: Mapping[str, torch.Tensor], what: str = "state_dict") -> None:
        """Same keys / shapes / dtypes as this layout (the reference would fail in `+=` or in
        load_state_dict(strict=True) otherwise)."""
        if len(sd) != len(self.entries):
            raise RuntimeError(f"{what}: {len(sd)} entries, expected {len(self.entries)}")
        for (name, t), e in zip(sd.items(), self.entries):
            if name != e.name or tuple(t.shape) != e.shape or t.dtype != e.dtype:
                raise RuntimeError(f"{what}: entry {name!r} {tuple(t.shape)} {t.dtype} does not match "
                                   f"{e.name!r} {e.shape} {e.dtype}")

    # ---------------------------------------------------------------------------------------
    def views(self, f32: torch.Tensor, i64: torch.Tensor,
              b16: Optional[torch.Tensor] = None) -> "OrderedDict[str, torch.Tensor]":
        out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        segs = {"f32": f32, "i64": i64, "b16": b16}
        for e in self.entries:
            out[e.name] = segs[e.seg][e.offset: e.offset + e.numel].view(e.shape)
        return out

    def flatten_into(self, sd: Mapping[str, torch.Tensor], f32: torch.Tensor, i64: torch.Tensor,
                     non_blocking: bool = False, b16: Optional[torch.Tensor] = None) -> None:
        """Copy a state_dict's values into flat segment tensors (any devices)."""
        segs = {"f32": f32, "i64": i64, "b16": b16}
        for e in self.entries:
            if e.alias_of is not None:
                continue
            segs[e.seg][e.offset: e.offset + e.numel].copy_(sd[e.name].reshape(-1), non_blocking=non_blocking)

    def flatten_cat(self, sd: Mapping[str, torch.Tensor], seg: str) -> List[torch.Tensor]:
        return [sd[e.name].reshape(-1) for e in self.entries if e.seg == seg and e.alias_of is None]

    def param_segments(self, param_names: Sequence[str]) -> List[Tuple[int, int, int, int]]:
        """(offset, A, I, B) of each parameter for the cosine kernel: nn.CosineSimilarity(dim=1)
        on the tensor, 1-D tensors unsqueezed to [n, 1] (decentralized_client.py:674-678)."""
        segs = []
        for name in param_names:
            e = self.by_name[name]
            if e.seg != "f32":
                raise NotImplementedError(f"parameter {name} is not fp32")
            s = e.shape
            if len(s) < 2:
                A, I, B = max(e.numel, 1), 1, 1
            else:
                A, I = s[0], s[1]
                B = 1
                for x in s[2:]:
                    B *= x
            segs.append((e.offset, int(A), int(I), int(B)))
        return segs


def by_name_offset(entries: Sequence[Entry], name: str) -> int:
    for e in entries:
        if e.name == name:
            return e.offset
    raise KeyError(name)


# Binding generation.  A bound module's state can stop being its pool row only by being
# re-pointed: Module._apply (module.to() / .cuda() / .float() / ..., on it or on any submodule),
# registering a parameter / buffer / submodule (setattr, register_buffer, load_state_dict
# (assign=True)), or assigning `.data` directly.  Hooks installed with the first bind bump this
# counter on each of them (torch's global registration hooks, a wrapper around Module._apply,
# and a `data` property on nn.Parameter whose setter bumps it); a binding verified entry by
# entry at generation g stays valid while the counter is still g, so the per-call check is O(1)
# (plus one data_ptr of the first entry) instead of one data_ptr per entry (ResNet-50: 320,
# ~70 us per model, ten models per call).  Not hooked: `buf.data = x` on a plain-tensor buffer
# (torch.Tensor itself is left alone); it is seen at the next full check, after any hook event.
_GEN = [0]
_HOOKS: list = []      # registration-hook handles
_RESTORE: list = []    # (owner, attribute, original) of every patched attribute


def _invalidate(*_args, **_kw) -> None:
    _GEN[0] += 1


def _install_hooks() -> None:
    if _HOOKS:
        return
    from torch.nn.modules import module as _m

    _HOOKS.append(_m.register_module_parameter_registration_hook(_invalidate))
    _HOOKS.append(_m.register_module_buffer_registration_hook(_invalidate))
    _HOOKS.append(_m.register_module_module_registration_hook(_invalidate))
    orig = nn.Module._apply

    def _apply(self, *args, **kwargs):
        _invalidate()
        return orig(self, *args, **kwargs)

    _RESTORE.append((nn.Module, "_apply", orig))
    nn.Module._apply = _apply  # type: ignore[method-assign]
    for name in ("register_parameter", "register_buffer", "__delattr__"):  # (set to None, del)
        def wrapped(self, *args, _orig=getattr(nn.Module, name), **kwargs):
            _invalidate()
            return _orig(self, *args, **kwargs)

        _RESTORE.append((nn.Module, name, getattr(nn.Module, name)))
        setattr(nn.Module, name, wrapped)
    base = torch._C.TensorBase.data

    def _set_data(self, value):
        _invalidate()
        base.__set__(self, value)

    _RESTORE.append((nn.Parameter, "data", nn.Parameter.__dict__.get("data")))
    nn.Parameter.data = property(base.__get__, _set_data, doc=base.__doc__)  # type: ignore[assignment]


def uninstall_hooks() -> None:
    """Undo what the first bind() installed on torch (registration hooks, the Module._apply /
    register_* / __delattr__ wrappers, the Parameter.data property).  Bindings stay usable:
    without the hooks every binding check is the full per-entry one.  bind() installs them
    again."""
    for h in _HOOKS:
        h.remove()
    _HOOKS.clear()
    for owner, attr, orig in reversed(_RESTORE):
        if orig is None:
            delattr(owner, attr)
        else:
            setattr(owner, attr, orig)
    _RESTORE.clear()
    _invalidate()


def _resolve(module: nn.Module, name: str) -> Tuple[nn.Module, str]:
    parts = name.split(".")
    mod = module
    for p in parts[:-1]:
        mod = getattr(mod, p)
    return mod, parts[-1]


class ModelPool:
    """Rows of flat model state on one GPU: f32[rows, ld_f32], b16[rows, ld_b16], i64[rows, ld_i64]."""

    def __init__(self, layout: StateLayout, rows: int, device, f32: Optional[torch.Tensor] = None,
                 i64: Optional[torch.Tensor] = None, b16: Optional[torch.Tensor] = None):
        self.layout = layout
        self.rows = rows
        self.device = torch.device(device)
        self.f32 = f32 if f32 is not None else torch.zeros(rows, layout.ld_f32, dtype=torch.float32, device=self.device)
        self.i64 = i64 if i64 is not None else torch.zeros(rows, layout.ld_i64, dtype=torch.int64, device=self.device)
        self.b16 = b16 if b16 is not None else torch.zeros(rows, layout.ld_b16, dtype=torch.bfloat16, device=self.device)
        self._bound: Dict[int, int] = {}  # id(module) -> row

    def row_f32(self, r: int) -> torch.Tensor:
        return self.f32[r, : self.layout.n_f32]

    def row_i64(self, r: int) -> torch.Tensor:
        return self.i64[r, : self.layout.n_i64]

    def row_b16(self, r: int) -> torch.Tensor:
        return self.b16[r, : self.layout.n_b16]

    def row_ptrs(self, seg: str, rows: Sequence[int]) -> List[int]:
        """Addresses of segment `seg` ("f32", "b16", "i64") of each of `rows`, without building
        a tensor view per row (the per-call path: ten operands per app call)."""
        t = getattr(self, seg)
        base, step = t.data_ptr(), t.stride(0) * t.element_size()
        return [base + step * r for r in rows]

    def segments(self):
        """(name, pool tensor, elements per row) of the layout's non-empty segments."""
        lay = self.layout
        return [(k, t, n) for k, t, n in (("f32", self.f32, lay.n_f32), ("b16", self.b16, lay.n_b16),
                                          ("i64", self.i64, lay.n_i64)) if n]

    def load_row(self, r: int, sd: Mapping[str, torch.Tensor]) -> None:
        self.layout.check_compatible(sd)
        self.layout.flatten_into(sd, self.f32[r], self.i64[r], b16=self.b16[r])

    def state_dict(self, r: int) -> "OrderedDict[str, torch.Tensor]":
        return self.layout.views(self.f32[r], self.i64[r], self.b16[r])

    def bind(self, module: nn.Module, r: int) -> nn.Module:
        """Copy `module`'s state into row r and make its parameters / buffers views of that row.

        Parameter objects keep their identity (``param.data`` is re-pointed) so optimizers built
        before or after binding keep working; buffers are re-registered as views.  The first
        bind installs torch hooks that make the binding check O(1) (_GEN; uninstall_hooks()
        removes them).  Re-pointing a bound tensor by a path no hook sees - ``Tensor.set_``,
        ``torch.utils.swap_tensors``, ``.data =`` on a plain-tensor buffer - is caught by the
        O(1) check only for the first and the last state entry; for the others it is seen at
        the next full check (after any hooked event), so do not use those paths on bound
        models (module.to(), load_state_dict, optimizer steps and in-place updates are safe)."""
        sd = module.state_dict()
        self.layout.check_compatible(sd, "module")
        with torch.no_grad():
            self.layout.flatten_into(sd, self.f32[r], self.i64[r], b16=self.b16[r])
        views = self.state_dict(r)
        slots = []  # (owning module, its _parameters or _buffers dict, attribute, row view's data_ptr)
        for e in self.layout.entries:
            mod, attr = _resolve(module, e.name)
            v = views[e.name]
            if attr in mod._parameters and mod._parameters[attr] is not None:
                table = mod._parameters
                if e.alias_of is None:
                    table[attr].data = v
            elif attr in mod._buffers:
                table = mod._buffers
                if e.alias_of is None:
                    table[attr] = v
            else:  # pragma: no cover - state_dict keys always resolve to a param or buffer
                raise KeyError(e.name)
            slots.append((table, attr, e.seg, v.data_ptr() - getattr(self, e.seg).data_ptr()))
        _install_hooks()
        module._tal_pool = self  # type: ignore[attr-defined]
        module._tal_row = r  # type: ignore[attr-defined]
        module._tal_gen = _GEN[0]  # type: ignore[attr-defined]
        module._tal_slots = [(table, attr) for table, attr, _, _ in slots]  # type: ignore[attr-defined]
        # each entry's byte offset from its segment's base: the base moves when a double-buffered
        # round exchanges the pool's storage (swap_storage), the offsets do not
        module._tal_segs = [seg for _, _, seg, _ in slots]  # type: ignore[attr-defined]
        module._tal_offs = [off for _, _, _, off in slots]  # type: ignore[attr-defined]
        self._bound[id(module)] = r
        return module

    def swap_with(self, other: "ModelPool") -> None:
        """Exchange this pool's memory with `other`'s (same layout, rows and device), segment by
        segment: every view of either pool - the bound models' parameters and buffers included -
        then reads the other's bytes.  No data moves (swap_storage)."""
        if other.layout != self.layout or other.rows != self.rows or other.device != self.device:
            raise ValueError("swap_with: pools differ in layout, rows or device")
        if not (self.whole_storage() and other.whole_storage()):
            raise ValueError("swap_with: a pool segment that is not a whole storage")
        for k in ("f32", "b16", "i64"):
            swap_storage(getattr(self, k), getattr(other, k))

    def whole_storage(self) -> bool:
        """Every segment tensor is its storage, whole (what swap_with exchanges)."""
        return all(not t.storage_offset() and t.untyped_storage().nbytes() == t.numel() * t.element_size()
                   for t in (self.f32, self.b16, self.i64))

    def row_of(self, module: nn.Module) -> Optional[int]:
        """Row the module is bound to, if its state still lives there: O(1) while no re-pointing
        hook fired since its last full check (_GEN), else checked per entry."""
        if getattr(module, "_tal_pool", None) is not self:
            return None
        r = module._tal_row  # type: ignore[attr-defined]
        slots = module._tal_slots  # type: ignore[attr-defined]
        if _HOOKS and module._tal_gen == _GEN[0]:  # type: ignore[attr-defined]
            # no re-pointing hook fired since the last full check (see _GEN); the first and
            # the last entry are compared as well (unhooked re-pointing of either is seen)
            segs, offs = module._tal_segs, module._tal_offs  # type: ignore[attr-defined]
            for k in (0, len(slots) - 1):
                table, attr = slots[k]
                t = table.get(attr)
                if t is None or t.data_ptr() - getattr(self, segs[k]).data_ptr() != offs[k]:
                    return None
            return r
        # after a hook event: every state entry, resolved by name again (a replaced submodule
        # keeps its old tables), must still be the row view bound to it
        gen = _GEN[0]
        fresh = []
        mods = dict(module.named_modules(remove_duplicate=False))
        try:
            for e in self.layout.entries:
                path, _, attr = e.name.rpartition(".")
                mod = mods[path]
                table = mod._parameters if attr in mod._parameters else mod._buffers
                fresh.append((table, attr))
            base = {k: getattr(self, k).data_ptr() for k in ("f32", "b16", "i64")}
            offs = [table[attr].data_ptr() - base[k] for (table, attr), k in zip(fresh, module._tal_segs)]
        except (KeyError, AttributeError):  # an entry removed or set to None
            return None
        if offs != module._tal_offs:  # type: ignore[attr-defined]
            return None
        table, attr = fresh[0]
        if table[attr].device != self.device:
            return None
        module._tal_slots = fresh  # type: ignore[attr-defined]
        module._tal_gen = gen  # type: ignore[attr-defined]
        return r


def bound_row(module: nn.Module) -> Optional[Tuple[ModelPool, int]]:
    pool = getattr(module, "_tal_pool", None)
    if pool is None:
        return None
    r = pool.row_of(module)
    return None if r is None else (pool, r)


_SWAP: list = []  # the loaded libtal_swap.so


def swap_storage(a: torch.Tensor, b: torch.Tensor) -> None:
    """Exchange the memory behind the storages of `a` and `b` (same size and device): every view
    of either then reads the other's bytes (csrc/storage_swap.cpp, built by build.build_swap)."""
    import ctypes

    if not _SWAP:
        from .build import SWAP_LIB

        if not SWAP_LIB.exists():
            raise RuntimeError(f"{SWAP_LIB} is missing: run __graft_entry__.build() (double-buffered rounds "
                               "exchange pool storages through it)")
        lib = ctypes.CDLL(str(SWAP_LIB))
        lib.tal_swap_storage.restype = ctypes.c_int32
        lib.tal_swap_storage.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _SWAP.append(lib)
    rc = _SWAP[0].tal_swap_storage(a.untyped_storage()._cdata, b.untyped_storage()._cdata)
    if rc:
        raise ValueError("swap_storage: " + ("the same storage" if rc == 1 else "sizes or devices differ"))


def select_pool_pair(make_pool: Callable[[], "ModelPool"], score: Callable[["ModelPool", "ModelPool"], float],
                     trials: int):
    """Placement calibration for a double-buffered device-resident round.

    Where a pool lands in HBM changes the round kernel's time bimodally - on config 3 the same
    plan over the same strides runs 2.0 or 2.45 ms depending on the physical placement of the
    pool it WRITES (tools/placement_probe.py, DESIGN.md §5: the slow allocations show the same
    TLB hit/miss counts and the same sequential-fill rate as the fast ones, but 1.5-2x the
    memory-side write-credit stalls and 2-3x the L2 tag stalls, i.e. DRAM-side contention of
    the concurrent row streams, not translation) - and a placement is fixed for the pool's
    lifetime, i.e. for every round of a training run.  So the arena allocates `trials` pools
    once, times a round INTO each (`score(src, dst)`, src = the next pool), then every ordered
    pair among the three fastest destinations, keeps the pair with the fastest round trip (the
    double-buffered round runs a -> b and b -> a in turn; the first two allocations are a
    candidate pair as well, and are kept unless another pair is more than 2 % faster; pairs are
    timed twice, interleaved, best of two) and frees the others: at most trials + 16 timed
    rounds instead of every ordered pair.  Returns (a, b, report); report["first_pair_ms"] is
    what the first two allocations run (both directions)."""
    pools = [make_pool() for _ in range(max(2, trials))]
    k = len(pools)
    ms = [float(score(pools[(j + 1) % k], pools[j])) for j in range(k)]
    order = sorted(range(k), key=lambda j: ms[j])
    # the SOURCE's placement counts too (a pair kept by destination times alone ran 8 % slower
    # than its calibration on one board, profiles/r02/final6): among the best three destinations
    # every ordered pair is timed and the pair with the fastest round trip a -> b, b -> a is kept
    top = sorted(order[:3])
    pairs = sorted({(i, j) for i in top for j in top if i < j} | {(0, 1)})  # the first two allocations too
    pair_ms = {}
    for _ in range(2):  # two passes, interleaved: the lower of two times per direction
        for i, j in pairs:
            for a, b in ((i, j), (j, i)):
                t = float(score(pools[a], pools[b]))
                pair_ms[(a, b)] = min(t, pair_ms.get((a, b), t))
    best = min(pairs, key=lambda q: pair_ms[q] + pair_ms[q[::-1]])
    # keep the first two allocations unless another pair is clearly faster: on a vector-ALU-bound
    # round every placement runs alike and the minimum is noise (config 4 once kept a pair
    # slower than the first)
    rt = {q: pair_ms[q] + pair_ms[q[::-1]] for q in pairs}
    if rt[best] > 0.98 * rt[(0, 1)]:
        best = (0, 1)
    a, b = pools[best[0]], pools[best[1]]
    first = (pair_ms[(0, 1)] + pair_ms[(1, 0)]) / 2
    report = dict(pools=k, dest_ms=[round(v, 3) for v in ms], chosen=list(best),
                  pair_ms={f"{i}->{j}": round(v, 3) for (i, j), v in pair_ms.items()},
                  first_pair_ms=round(first, 3),
                  chosen_pair_ms=round((pair_ms[best] + pair_ms[best[::-1]]) / 2, 3))
    del pools
    torch.cuda.empty_cache()
    return a, b, report
