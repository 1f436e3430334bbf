"""Device operations: thin, checked wrappers over the C-ABI (include/tal_agg.h).

Every function takes torch tensors that already live on the GPU and launches on the current
torch stream of their device.  Nothing here falls back to the CPU: without the HIP library
the first call raises ``TalLibraryError``; with a CPU tensor it raises ``ValueError``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import RoundPlanInfo, check

MODE_EXACT = _lib.TAL_MODE_EXACT
MODE_FMA = _lib.TAL_MODE_FMA


def _stream(device: torch.device, stream: Optional[torch.cuda.Stream] = None) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def _require_gpu(t: torch.Tensor, name: str, dtype: torch.dtype) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a GPU tensor (got {t.device}); the aggregation has no CPU path")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _ptrs_and_weights(xs, weights, n, dtype, out):
    if len(xs) == 0:
        raise ValueError("at least one operand is required")
    if len(weights) != len(xs):
        raise ValueError(f"{len(xs)} operands but {len(weights)} weights")
    for i, x in enumerate(xs):
        _require_gpu(x, f"operand {i}", dtype)
        if x.numel() != n:
            raise ValueError(f"operand {i} has {x.numel()} elements, expected {n}")
        if x.device != out.device:
            raise ValueError(f"operand {i} is on {x.device}, out on {out.device}")
    return _lib.ptr_array([x.data_ptr() for x in xs]), _lib.double_array(weights)


def agg_f32(xs: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor,
            mode: int = MODE_EXACT, stream=None) -> torch.Tensor:
    """K1: out = sum_i fp32(w_i) * xs[i] (reference order; decentralized_client.py:399-411)."""
    _require_gpu(out, "out", torch.float32)
    n = out.numel()
    P, W = _ptrs_and_weights(xs, weights, n, torch.float32, out)
    L = _lib.load()
    check(L.tal_agg_f32(P, W, len(xs), ctypes.c_void_p(out.data_ptr()), n, int(mode),
                        _stream(out.device, stream)))
    return out


def agg_i64(xs: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor,
            stream=None) -> torch.Tensor:
    """K1 on int64 buffers: fp32 accumulate, truncation (decentralized_client.py:407-413)."""
    _require_gpu(out, "out", torch.int64)
    n = out.numel()
    P, W = _ptrs_and_weights(xs, weights, n, torch.int64, out)
    L = _lib.load()
    check(L.tal_agg_i64(P, W, len(xs), ctypes.c_void_p(out.data_ptr()), n, _stream(out.device, stream)))
    return out


def agg_model_f32(xs: Sequence[torch.Tensor], xis: Sequence[torch.Tensor], weights: Sequence[float],
                  out: torch.Tensor, out_i: torch.Tensor, mode: int = MODE_EXACT, stream=None) -> None:
    """K1 over a whole model in one launch: out = sum_i fp32(w_i) * xs[i] (fp32 segment) and
    out_i = trunc(sum_i fp32(w_i) * fp32(xis[i])) (int64 segment), the arithmetic of agg_f32 and
    agg_i64 bit for bit (decentralized_client.py:406-413 over every state_dict entry)."""
    _require_gpu(out, "out", torch.float32)
    _require_gpu(out_i, "out_i", torch.int64)
    n, n_i = out.numel(), out_i.numel()
    P, W = _ptrs_and_weights(xs, weights, n, torch.float32, out)
    PI, _ = _ptrs_and_weights(xis, weights, n_i, torch.int64, out)
    L = _lib.load()
    check(L.tal_agg_model_f32(P, PI, W, len(xs), ctypes.c_void_p(out.data_ptr()), n,
                              ctypes.c_void_p(out_i.data_ptr()), n_i, int(mode), _stream(out.device, stream)))


def agg_pool_rows(pool, rows: Sequence[int], weights: Sequence[float], out_row: int,
                  mode: int = MODE_EXACT, stream=None) -> None:
    """K1 on rows of one device-resident ModelPool: row out_row <- sum_i fp32(w_i) * row rows[i],
    every segment of the layout (fp32 + int64 in one launch, as agg_model_f32; otherwise one
    launch per segment), out_row may be one of the operands (the app's own model, in place).
    The arithmetic of agg_model_f32 / agg_f32 / agg_bf16 / agg_i64 on the rows' views, with the
    operand addresses computed from the pool (the pool's tensors are checked once per call, not
    each row view): the per-call app path on pool-bound models (decentralized_client.py:399-413)."""
    if pool.device.type != "cuda":
        raise ValueError(f"agg_pool_rows needs a device pool (got {pool.device}); the aggregation has no CPU path")
    m = len(rows)
    if m == 0:
        raise ValueError("at least one operand is required")
    if len(weights) != m:
        raise ValueError(f"{m} operands but {len(weights)} weights")
    for r in (*rows, out_row):
        if not 0 <= int(r) < pool.rows:
            raise IndexError(f"row {r} outside the pool's {pool.rows} rows")
    lay = pool.layout
    for seg, t, n in pool.segments():
        if t.dim() != 2 or t.stride(1) != 1 or t.shape[1] < n:
            raise ValueError(f"pool segment {seg} must be [rows, ld] with unit column stride")
    W = _lib.double_array(weights)
    s = _stream(pool.device, stream)
    L = _lib.load()
    rows = [int(r) for r in rows]
    if lay.n_f32 and lay.n_i64 and not lay.n_b16:
        check(L.tal_agg_model_f32(_lib.ptr_array(pool.row_ptrs("f32", rows)), _lib.ptr_array(pool.row_ptrs("i64", rows)),
                                  W, m, ctypes.c_void_p(pool.row_ptrs("f32", [out_row])[0]), lay.n_f32,
                                  ctypes.c_void_p(pool.row_ptrs("i64", [out_row])[0]), lay.n_i64, int(mode), s))
        return
    for seg, n in (("f32", lay.n_f32), ("b16", lay.n_b16), ("i64", lay.n_i64)):
        if not n:
            continue
        P = _lib.ptr_array(pool.row_ptrs(seg, rows))
        out = ctypes.c_void_p(pool.row_ptrs(seg, [out_row])[0])
        if seg == "i64":
            check(L.tal_agg_i64(P, W, m, out, n, s))
        else:
            fn = L.tal_agg_f32 if seg == "f32" else L.tal_agg_bf16
            check(fn(P, W, m, out, n, int(mode), s))


def agg_bf16(xs: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor,
             mode: int = MODE_EXACT, stream=None) -> torch.Tensor:
    """K1 on bf16 buffers.  MODE_EXACT: the reference's torch ops on bf16 tensors (every product
    and partial sum rounded to bf16; decentralized_client.py:407-411); MODE_FMA: fp32 fused
    accumulation rounded once."""
    _require_gpu(out, "out", torch.bfloat16)
    n = out.numel()
    P, W = _ptrs_and_weights(xs, weights, n, torch.bfloat16, out)
    L = _lib.load()
    check(L.tal_agg_bf16(P, W, len(xs), ctypes.c_void_p(out.data_ptr()), n, int(mode),
                         _stream(out.device, stream)))
    return out


# ------------------------------------------------------------------------------------------
# Host reduction (a process that sees no GPU: BASELINE config 1)
# ------------------------------------------------------------------------------------------
_HOST_FN = {torch.float32: "tal_host_agg_f32", torch.int64: "tal_host_agg_i64",
            torch.bfloat16: "tal_host_agg_bf16"}


def host_agg(xs: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor,
             mode: int = MODE_EXACT) -> torch.Tensor:
    """The library's host reduction (tal_host_agg_*) on contiguous CPU tensors of one dtype:
    out = sum_i fp32(w_i) * xs[i] with the kernels' arithmetic (fp32 / int64 / bf16, modes as
    agg_f32 / agg_i64 / agg_bf16).  For processes without a GPU only (aggregate.py dispatches
    on torch.cuda.is_available()); GPU tensors are refused."""
    if out.device.type != "cpu" or not out.is_contiguous() or out.dtype not in _HOST_FN:
        raise ValueError("host_agg: out must be a contiguous CPU float32 / int64 / bfloat16 tensor")
    if len(xs) == 0 or len(weights) != len(xs):
        raise ValueError("host_agg: one weight per operand, at least one operand")
    n = out.numel()
    for i, x in enumerate(xs):
        if x.device.type != "cpu" or x.dtype != out.dtype or not x.is_contiguous() or x.numel() != n:
            raise ValueError(f"host_agg: operand {i} must be a contiguous CPU {out.dtype} tensor of {n} elements")
    L = _lib.load()
    P, W = _lib.ptr_array([x.data_ptr() for x in xs]), _lib.double_array(weights)
    args = [P, W, len(xs), ctypes.c_void_p(out.data_ptr()), n]
    if out.dtype != torch.int64:
        args.append(int(mode))
    check(getattr(L, _HOST_FN[out.dtype])(*args))
    return out


# ------------------------------------------------------------------------------------------
# K3 round plans
# ------------------------------------------------------------------------------------------
LDS_BUDGET = 80 * 1024  # two workgroups per CU overlap one's HBM staging with the other's math
LDS_BUDGETS = (80 * 1024, 160 * 1024)  # candidates: 2 workgroups / CU, or 1 with bigger groups
TILE_WIDTHS = (64, 128, 32, 16)  # float4 per staged source per tile (ties keep the earlier)
# the narrow kernel's broadcast form (build_plan(bcast=...)): (c4, wavefronts per workgroup,
# workgroups per CU) of the forms that won a measured round - per-operand weights on a
# community graph (config 5 degree-centrality: fp32 16/8/2, bf16 32/16/1 and 16/16/2).
# The form is a candidate only for rounds with per-operand weights: on uniform-weight rows it
# never won (config 3: 6.2-9.9 ms against 2.0 in BENCH_r05; config 5 bf16 unweighted: 23.6-103
# against 22.3, profiles/r06/r06a)
BCAST_CANDIDATES = ((16, 8, 2), (16, 16, 2), (32, 16, 1), (32, 8, 2))
TUNE_DROP = 1.5  # a candidate whose first timed run exceeds the default's by this factor is dropped


@dataclass
class RoundPlan:
    info: RoundPlanInfo
    host: np.ndarray           # int32 blob
    device: Optional[torch.Tensor] = None
    rows: int = 0
    nnz: int = 0
    tuned_ms: Optional[float] = None
    candidates: Optional[list] = None  # tune_plan's measured candidates
    spec: Optional[dict] = None        # how it was built (plan_from_spec rebuilds it)

    @property
    def single_group(self) -> bool:
        return self.info.n_groups == 1

    def to(self, device) -> "RoundPlan":
        self.device = torch.from_numpy(self.host).to(device, non_blocking=False)
        return self

    def staged_rows(self) -> int:
        """Source rows read from HBM per column tile (sum over groups)."""
        return int(self.info.total_src)


@dataclass
class RowCallPlan:
    """A round as one K1 call per row, out of place (snapshot semantics): the fallback for a
    round with a row of more distinct sources than any LDS-tiled form stages in one tile
    (> ~620 at c4 = 16) on a bf16 pool, where the streamed form (fp32 only) cannot take it
    either - e.g. the reference's `unweighted_fl` strategy (every other client a neighbor,
    decentralized_app.py:386-389) with many clients under the batched round.  K1 chains any
    operand count in reference order, so every row is bitwise its per-call aggregation."""
    row_ptr: np.ndarray
    col: np.ndarray
    w: np.ndarray
    out_row: np.ndarray
    device: Optional[torch.device] = None
    tuned_ms: Optional[float] = None
    candidates: Optional[list] = None
    spec: Optional[dict] = None

    @property
    def rows(self) -> int:
        return len(self.out_row)

    @property
    def single_group(self) -> bool:
        return False  # rows read other rows' pre-round values: never in place

    def staged_rows(self) -> int:
        """Source rows read from HBM per column: every operand of every row."""
        return int(len(self.col))

    def to(self, device) -> "RowCallPlan":
        self.device = torch.device(device)
        return self


def row_call_plan(row_ptr, col, w, out_row) -> RowCallPlan:
    rp, cl, ww, orow = _csr(row_ptr, col, w, out_row)
    return RowCallPlan(rp, cl, ww, orow, spec={"rows_k1": 1})


def _round_rows(pool_in, pool_out, plan: RowCallPlan, n, dtype, mode, stream):
    _require_gpu(pool_in, "pool_in", dtype)
    _require_gpu(pool_out, "pool_out", dtype)
    if pool_in.dim() != 2 or pool_out.dim() != 2:
        raise ValueError("pools must be 2-D [models, ld]")
    if pool_in.data_ptr() == pool_out.data_ptr():
        raise ValueError("a per-row round runs out of place (snapshot semantics)")
    n = pool_in.shape[1] if n is None else int(n)
    if plan.col.max(initial=-1) >= pool_in.shape[0] or plan.out_row.max(initial=-1) >= pool_out.shape[0]:
        raise ValueError("plan rows beyond the pools")
    for r in range(plan.rows):
        a, b = int(plan.row_ptr[r]), int(plan.row_ptr[r + 1])
        xs = [pool_in[int(j), :n] for j in plan.col[a:b]]
        out = pool_out[int(plan.out_row[r]), :n]
        ws = plan.w[a:b].tolist()
        if dtype == torch.int64:
            agg_i64(xs, ws, out, stream=stream)
        elif dtype == torch.bfloat16:
            agg_bf16(xs, ws, out, mode=mode, stream=stream)
        else:
            agg_f32(xs, ws, out, mode=mode, stream=stream)
    return pool_out


def build_plan(row_ptr, col, w, out_row, c4: int = 0, lds_bytes: int = 0, dense: int = 0,
               bcast: int = 0, bcast_wg: int = 2) -> RoundPlan:
    """Tile plan for a round given as CSR (row r: operands col[row_ptr[r]:row_ptr[r+1]] with
    float64 weights w, written to pool row out_row[r]).

    c4 = 0 / lds_bytes = 0 search the float4 tile width (16, 32, 64 or 128 float4 per source;
    16 / 32 are the narrow-tile kernel: up to 256 / 128 sources in one group, sparse form) and
    the LDS budget (LDS_BUDGETS) for the plan with the lowest estimated time per element:
      HBM  = 4 B x (staged sources + rows)                     at ~5.5 TB/s
      LDS  = 4 B x operands (one LDS read per operand)         at ~150 TB/s x eff(workgroups/CU)
    (eff = 0.33 / 0.6 / 0.8 for 1 / 2 / >= 3 resident workgroups, halved at c4 = 64; fitted to
    tools/tune/round_variants.hip on MI355X); ties go to more resident workgroups.
    dense: 0 (default) = the sparse form; 8 requests dense row blocks; -1 lets the library
    pick dense when one LDS read serves >= 4 operands on average.  The dense form lost every
    measured A/B outside cliques (config 3: 6.2 vs 2.45 ms, config 5: 171 vs 83 ms; round-1
    tuner candidates), and clique rounds take the K3c plan (default_plan).
    bcast = 8 / 16: the narrow kernel's broadcast form (tal_round_plan_build_bcast) with that
    many wavefronts per workgroup: per-lane operand records in VGPRs, handed to a row's lanes
    by DPP row broadcasts, so per-operand weights cost no LDS reads (c4 16 / 32 only);
    bcast_wg = resident workgroups per CU it is compiled for (1: 128 VGPRs at 1024 threads and
    8 LDS reads in flight per wavefront; 2: 64 VGPRs, two groups' tiles per CU)."""
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
    col = np.ascontiguousarray(col, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    out_row = np.ascontiguousarray(out_row, dtype=np.int32)
    rows = len(out_row)
    if len(row_ptr) != rows + 1 or row_ptr[-1] != len(col) or len(w) != len(col):
        raise ValueError("inconsistent CSR arrays")
    L = _lib.load()
    cap = L.tal_round_plan_words(rows, len(col))
    best = None
    last_err = None
    widths = [c4] if c4 else ((16, 32) if bcast else TILE_WIDTHS)
    cands = [(c, b) for b in ([lds_bytes] if lds_bytes else LDS_BUDGETS) for c in widths]
    for cand, budget in cands:
        info = RoundPlanInfo()
        P32 = ctypes.POINTER(ctypes.c_int32)
        size = cap
        for _ in range(2):  # the dense tables' size is known only after grouping: retry once
            blob = np.zeros(size, dtype=np.int32)
            args = (rows, row_ptr.ctypes.data_as(P32), col.ctypes.data_as(P32),
                    w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out_row.ctypes.data_as(P32), cand, int(budget))
            if bcast:
                rc = L.tal_round_plan_build_bcast(*args, int(bcast), int(bcast_wg), blob.ctypes.data_as(P32), size,
                                                  ctypes.byref(info))
            else:
                rc = L.tal_round_plan_build(*args, int(dense), blob.ctypes.data_as(P32), size, ctypes.byref(info))
            if rc == _lib.TAL_ERR_CAPACITY and info.words > size:
                size = int(info.words)
                continue
            break
        if rc != _lib.TAL_OK:
            last_err = _lib.TalError(rc, L.tal_last_error().decode())
            continue
        spec = dict(c4=int(cand), lds=int(budget), dense=int(dense))
        if bcast:
            spec["bcast"] = int(bcast)
            spec["bcwg"] = int(bcast_wg)
        plan = RoundPlan(info=info, host=blob[: info.words].copy(), rows=rows, nnz=len(col), spec=spec)
        key = (_plan_cost(plan.info), -_blocks_per_cu(plan.info))
        if best is None or key < best[0]:
            best = (key, plan)
    if best is None:
        raise last_err
    return best[1]


CLIQUE_MAX = 64
CLIQUE_EXTRA = 4          # attached rows per clique block
CLIQUE_EXTRA_WORDS = 12
CLIQUE_WORDS = 4 + 2 * CLIQUE_MAX + CLIQUE_EXTRA * CLIQUE_EXTRA_WORDS  # TAL_CLIQUE_WORDS (180)
CLIQUE_MIN_ROWS = 8       # smaller blocks stay in the regular plan
CLIQUE_MIN_SHARED = 8     # an attached row takes at least this many operands from the block


def find_cliques(row_ptr, col, w, out_row, min_rows: int = CLIQUE_MIN_ROWS):
    """Uniform-weight clique blocks of a round (the K3c kernel's rows, tal_agg.h): rows whose
    operands are strictly ascending sources and then their own model (not among them), all with
    one finite fp32 weight, grouped by (operand set, weight); a group of >= min_rows rows with
    distinct own models and <= 64 sources is a clique block.  Other such rows that take at
    least CLIQUE_MIN_SHARED neighbors from a block and have at most two more are attached to it
    (up to CLIQUE_EXTRA per block).  Returns (cliques, rest): cliques = [(sources ascending, fp32
    weight, {member index: out_row}, [attached row records])], rest = the other row indices."""
    row_ptr, col, w, out_row = _csr(row_ptr, col, w, out_row)
    groups: dict = {}
    for r in range(len(out_row)):
        ops_ = col[row_ptr[r]: row_ptr[r + 1]]
        m = len(ops_)
        if m < 2 or m > CLIQUE_MAX:
            continue
        w32 = w[row_ptr[r]: row_ptr[r + 1]].astype(np.float32)
        if not np.isfinite(w32[0]) or np.any(w32.view(np.uint32) != w32[:1].view(np.uint32)):
            continue
        rest, own = ops_[:-1], int(ops_[-1])
        if np.any(np.diff(rest) <= 0) or own in rest:
            continue
        groups.setdefault((tuple(sorted(ops_.tolist())), int(w32[:1].view(np.uint32)[0])), []).append(r)
    cliques, used = [], set()
    for (srcs, wbits), rows in groups.items():
        owns = [int(col[row_ptr[r + 1] - 1]) for r in rows]
        if len(rows) < min_rows or len(set(owns)) != len(rows):
            continue
        idx = {s: i for i, s in enumerate(srcs)}
        cliques.append((list(srcs), np.array([wbits], np.uint32).view(np.float32)[0],
                        {idx[o]: int(out_row[r]) for o, r in zip(owns, rows)}, []))
        used.update(rows)
    # attached rows: uniform-weight rows in reference order that take most operands from one
    # block (a barbell's bridge nodes) - at most two other neighbors, own model anywhere
    for r in range(len(out_row)):
        if r in used or not cliques:
            continue
        ops_ = col[row_ptr[r]: row_ptr[r + 1]]
        w32 = w[row_ptr[r]: row_ptr[r + 1]].astype(np.float32)
        if len(ops_) < 2 or not np.isfinite(w32[0]) or np.any(w32.view(np.uint32) != w32[:1].view(np.uint32)):
            continue
        nb, own = ops_[:-1], int(ops_[-1])
        if np.any(np.diff(nb) <= 0) or own in nb:
            continue
        best = max(range(len(cliques)), key=lambda c: len(set(cliques[c][0]).intersection(nb.tolist())))
        srcs, _, _, att = cliques[best]
        idx = {s: i for i, s in enumerate(srcs)}
        mem = [int(x) for x in nb if int(x) in idx]
        ext = [int(x) for x in nb if int(x) not in idx]
        if len(mem) < CLIQUE_MIN_SHARED or len(ext) > 2 or len(att) >= CLIQUE_EXTRA:
            continue
        mask = 0
        for x in mem:
            mask |= 1 << idx[x]
        att.append(dict(out=int(out_row[r]), w=w32[0], mask=mask, self_member=idx.get(own, -1),
                        self_row=-1 if own in idx else own,
                        ext=[(x, sum(1 for s_ in srcs if s_ < x)) for x in ext]))
        used.add(r)
    return cliques, [r for r in range(len(out_row)) if r not in used]


@dataclass
class CliquePlan:
    """A round split into clique blocks (K3c, one launch) and the remaining rows (a regular
    RoundPlan, None if there are none).  `full` is a sparse plan over all rows, used for the
    int64 and bf16 segments (the clique kernel is fp32)."""
    table: np.ndarray
    n_cliques: int
    mmax: int
    clique_sources: int
    clique_rows: int
    rest: Optional[RoundPlan]
    full: RoundPlan
    rows: int
    rest_rows: Optional[list] = None
    device: Optional[torch.Tensor] = None
    tuned_ms: Optional[float] = None
    candidates: Optional[list] = None
    spec: Optional[dict] = None

    @property
    def info(self) -> RoundPlanInfo:
        return self.full.info

    @property
    def single_group(self) -> bool:
        return False  # clique blocks read other blocks' sources: never in place

    def staged_rows(self) -> int:
        """Source rows read from HBM per column (clique sources + the rest plan's)."""
        return self.clique_sources + (self.rest.staged_rows() if self.rest is not None else 0)

    def to(self, device) -> "CliquePlan":
        self.device = torch.from_numpy(self.table).to(device)
        if self.rest is not None:
            self.rest.to(device)
        self.full.to(device)
        return self


def build_clique_plan(row_ptr, col, w, out_row, min_rows: int = CLIQUE_MIN_ROWS,
                      rest_spec: Optional[dict] = None) -> Optional[CliquePlan]:
    """CliquePlan of a round, or None when it has no clique block (find_cliques)."""
    row_ptr, col, w, out_row = _csr(row_ptr, col, w, out_row)
    cliques, rest = find_cliques(row_ptr, col, w, out_row, min_rows)
    if not cliques:
        return None
    table = np.zeros((len(cliques), CLIQUE_WORDS), np.int32)
    n_ext_loads = 0
    for k, (srcs, w32, outs, att) in enumerate(cliques):
        table[k, 0] = len(srcs)
        table[k, 1] = np.array([w32], np.float32).view(np.int32)[0]
        table[k, 2] = len(att)
        table[k, 4: 4 + len(srcs)] = srcs
        table[k, 4 + CLIQUE_MAX: 4 + 2 * CLIQUE_MAX] = -1
        for i, o in outs.items():
            table[k, 4 + CLIQUE_MAX + i] = o
        for q, a in enumerate(att):
            rec = table[k, 4 + 2 * CLIQUE_MAX + q * CLIQUE_EXTRA_WORDS:][:CLIQUE_EXTRA_WORDS]
            rec[0] = a["out"]
            rec[1] = np.array([a["w"]], np.float32).view(np.int32)[0]
            rec[2:4] = np.array([a["mask"] & 0xFFFFFFFF, a["mask"] >> 32], np.uint32).view(np.int32)
            rec[4], rec[5], rec[6] = a["self_member"], a["self_row"], len(a["ext"])
            for e_, (row, pos) in enumerate(a["ext"]):
                rec[7 + e_], rec[9 + e_] = row, pos
            n_ext_loads += len(a["ext"]) + (a["self_row"] >= 0)
    rest_plan = None
    if rest:
        sub = _sub_csr(row_ptr, col, w, out_row, rest)
        rest_plan = plan_from_spec(*sub, rest_spec) if rest_spec else build_plan(*sub)
    mmax = max(len(c[0]) for c in cliques)
    return CliquePlan(table=table.reshape(-1), n_cliques=len(cliques), mmax=mmax,
                      clique_sources=sum(len(c[0]) for c in cliques) + n_ext_loads,
                      clique_rows=sum(len(c[2]) + len(c[3]) for c in cliques), rest=rest_plan,
                      full=build_plan(row_ptr, col, w, out_row, dense=0), rows=len(out_row), rest_rows=rest)


REG_MAX_SRC = 64   # sources per register group (v[32:160): 64 x 2 fp32 per lane)
REG_WINDOW = 64    # rows considered when growing a group


@dataclass
class RegPlan:
    """A round as register-resident source groups (K3r, tal_agg_round_reg): rows grouped so that
    each group's operands are <= max_src distinct sources, a group's rows run in pairs whose
    operands come in trip records of four per row.  `full` is a sparse plan over all rows for
    the int64 segment (and bf16 EXACT, which K3r does not take)."""
    table: np.ndarray
    n_groups: int
    off_src: int
    off_pairs: int
    off_rec: int
    max_src: int
    group_sources: int   # sum over groups of their sources (L2 reads per column)
    full: RoundPlan
    rows: int
    trips: int = 0       # trip records (16 dwords each; 8 operand slots, padding included)
    device: Optional[torch.Tensor] = None
    tuned_ms: Optional[float] = None
    candidates: Optional[list] = None
    spec: Optional[dict] = None

    @property
    def info(self) -> RoundPlanInfo:
        return self.full.info

    @property
    def single_group(self) -> bool:
        return False  # groups read other groups' output rows: never in place

    def staged_rows(self) -> int:
        """Distinct sources read per column: every source once (the groups sharing a source
        are served by L2 on the XCD their piece runs on)."""
        return int(len(np.unique(self.table[self.off_src: self.off_pairs])))

    def pair_records(self) -> np.ndarray:
        """[P, 4] {out row A, out row B or -1, trips, byte offset of the first trip record}."""
        return self.table[self.off_pairs: self.off_rec].reshape(-1, 4)[:self.n_pairs]

    @property
    def n_pairs(self) -> int:
        g = self.table[: 4 * self.n_groups].reshape(-1, 4)
        return int(g[:, 3].sum())

    def to(self, device) -> "RegPlan":
        self.device = torch.from_numpy(self.table).to(device)
        self.full.to(device)
        self._src_off = {}
        return self

    def src_offsets(self, pitch_bytes: int, device) -> torch.Tensor:
        """Device int64 byte offsets (row x pitch) of the source list's entries, once per pool
        pitch: the kernel adds them to the piece's base instead of multiplying per source."""
        cache = self.__dict__.setdefault("_src_off", {})
        key = (int(pitch_bytes), str(device))
        t = cache.get(key)
        if t is None:
            rows = self.table[self.off_src: self.off_src + 16 * ((self.max_src + 15) // 16) * self.n_groups]
            t = cache[key] = torch.from_numpy(rows.astype(np.int64) * int(pitch_bytes)).to(device)
        return t


REG_TRIP = 4        # operands of each row per trip record
REG_REC_WORDS = 16  # {A idx x4, B idx x4, A w x4, B w x4}


def reg_groups(row_ptr, col, max_src: int = REG_MAX_SRC, window: int = REG_WINDOW):
    """Rows grouped greedily: a group starts at the first unassigned row and repeatedly takes,
    among the next `window` unassigned rows, the one adding the fewest new sources while the
    union stays <= max_src.  Returns [(rows, sources ascending)]."""
    n = len(row_ptr) - 1
    ops_ = [set(col[row_ptr[r]: row_ptr[r + 1]].tolist()) for r in range(n)]
    left = list(range(n))
    groups = []
    while left:
        r0 = left.pop(0)
        if len(ops_[r0]) > max_src:
            raise ValueError(f"row {r0} has {len(ops_[r0])} distinct sources > {max_src}")
        cur, src = [r0], set(ops_[r0])
        while True:
            best = None
            for r in left[:window]:
                add = len(ops_[r] - src)
                if len(src) + add <= max_src and (best is None or add < best[0]):
                    best = (add, r)
            if best is None:
                break
            left.remove(best[1])
            cur.append(best[1])
            src |= ops_[best[1]]
        groups.append((cur, sorted(src)))
    return groups


def build_reg_plan(row_ptr, col, w, out_row, max_src: int = REG_MAX_SRC) -> Optional[RegPlan]:
    """RegPlan of a round (table layout: tal_agg.h K3r), or None when a row has more than
    max_src distinct sources.  Inside a group the rows are ordered by operand count
    (descending) and paired in that order, so a pair's rows need about the same number of
    trips; the shorter row (and a lone last row's partner) is padded with the neutral operand
    (register offset 32 x NB, weight +0.0)."""
    row_ptr, col, w = row_ptr.astype(np.int32), col.astype(np.int32), np.asarray(w, np.float64)
    row_ptr, col, w, out_row = _csr(row_ptr, col, w, out_row)
    try:
        groups = reg_groups(row_ptr, col, max_src)
    except ValueError:
        return None
    G = len(groups)
    nb = (max(len(s_) for _, s_ in groups) + 15) // 16
    span, neutral = 16 * nb, 32 * nb
    w32all = w.astype(np.float32).view(np.uint32)
    src_list, pairs, recs = [], [], []
    grp = np.zeros((G, 4), np.int32)

    def lists(r, slot):
        if r is None:
            return [], []
        q0, q1 = int(row_ptr[r]), int(row_ptr[r + 1])
        return [2 * slot[int(c)] for c in col[q0:q1]], [int(x) for x in w32all[q0:q1]]

    for g, (rows, srcs) in enumerate(groups):
        slot = {s_: k for k, s_ in enumerate(srcs)}
        rows = sorted(rows, key=lambda r: -(row_ptr[r + 1] - row_ptr[r]))
        grp[g] = (len(src_list), len(srcs), len(pairs), (len(rows) + 1) // 2)
        src_list.extend(srcs + [srcs[0]] * (span - len(srcs)))  # padding reloads the first source
        for k in range(0, len(rows), 2):
            ra, rb = rows[k], rows[k + 1] if k + 1 < len(rows) else None
            ia, wa = lists(ra, slot)
            ib, wb = lists(rb, slot)
            trips = (max(len(ia), len(ib)) + REG_TRIP - 1) // REG_TRIP
            pad = REG_TRIP * trips
            ia, wa = ia + [neutral] * (pad - len(ia)), wa + [0] * (pad - len(wa))
            ib, wb = ib + [neutral] * (pad - len(ib)), wb + [0] * (pad - len(wb))
            pairs.append([int(out_row[ra]), -1 if rb is None else int(out_row[rb]), trips, len(recs)])
            for t in range(trips):
                sl = slice(REG_TRIP * t, REG_TRIP * (t + 1))
                recs.append(ia[sl] + ib[sl] + wa[sl] + wb[sl])
    off_src = 4 * G
    off_pairs = (off_src + len(src_list) + 3) // 4 * 4
    off_rec = (off_pairs + 4 * len(pairs) + 15) // 16 * 16
    words = off_rec + REG_REC_WORDS * (len(recs) + 1)  # + one record read ahead by the loop
    table = np.zeros(words, np.int32)
    table[:off_src] = grp.reshape(-1)
    table[off_src: off_src + len(src_list)] = src_list
    pr = np.asarray(pairs, np.int64)
    pr[:, 3] = 4 * (off_rec + REG_REC_WORDS * pr[:, 3])  # byte offsets from the table base
    table[off_pairs: off_pairs + 4 * len(pairs)] = pr.astype(np.int32).reshape(-1)
    table[off_rec: off_rec + REG_REC_WORDS * len(recs)] = \
        np.asarray(recs, np.uint32).view(np.int32).reshape(-1)
    return RegPlan(table=table, n_groups=G, off_src=off_src, off_pairs=off_pairs, off_rec=off_rec,
                   max_src=max(len(s_) for _, s_ in groups), group_sources=sum(len(s_) for _, s_ in groups),
                   full=build_plan(row_ptr, col, w, out_row, dense=0), rows=len(out_row), trips=len(recs))


def _round_reg(pool_in, pool_out, plan: RegPlan, n, dtype, mode, stream):
    _require_gpu(pool_in, "pool_in", dtype)
    _require_gpu(pool_out, "pool_out", dtype)
    if pool_in.dim() != 2 or pool_out.dim() != 2:
        raise ValueError("pools must be 2-D [models, ld]")
    if pool_in.device != pool_out.device:
        raise ValueError("pools on different devices")
    if pool_in.data_ptr() == pool_out.data_ptr():
        raise ValueError("a register round runs out of place (snapshot semantics)")
    n = pool_in.shape[1] if n is None else int(n)
    bf16 = dtype == torch.bfloat16
    esz = pool_in.element_size()
    pad = n + (n & 1)
    if (bf16 and mode == MODE_EXACT) or pool_in.stride(0) % 2 or pool_out.stride(0) % 2 \
            or pool_in.shape[1] < pad or pool_out.shape[1] < pad \
            or (pool_in.data_ptr() | pool_out.data_ptr()) % (2 * esz):
        # K3r reads and writes 2-element pairs and runs bf16 in FMA mode only: other pools and
        # bf16 EXACT take the full plan
        return _round(pool_in, pool_out, plan.full, n, dtype, mode, stream)
    if plan.device is None or plan.device.device != pool_in.device:
        plan.to(pool_in.device)
    t = plan.table
    if t[plan.off_src: plan.off_pairs].max(initial=-1) >= pool_in.shape[0]:
        raise ValueError("plan reads a pool row beyond pool_in")
    if plan.pair_records()[:, :2].max(initial=-1) >= pool_out.shape[0]:
        raise ValueError("plan writes a pool row beyond pool_out")
    L = _lib.load()
    offs = plan.src_offsets(pool_in.stride(0) * esz, pool_in.device)
    check(L.tal_agg_round_reg(ctypes.c_void_p(pool_in.data_ptr()), pool_in.stride(0),
                              ctypes.c_void_p(pool_out.data_ptr()), pool_out.stride(0), n, int(bf16),
                              ctypes.c_void_p(plan.device.data_ptr()), ctypes.c_void_p(offs.data_ptr()),
                              plan.n_groups, plan.off_src,
                              plan.off_pairs, plan.off_rec, plan.max_src, int(mode),
                              _stream(pool_in.device, stream)))
    return pool_out


def _sub_csr(row_ptr, col, w, out_row, rows):
    """The CSR of a subset of a round's rows."""
    rp = np.concatenate([[0], np.cumsum([row_ptr[r + 1] - row_ptr[r] for r in rows])]).astype(np.int32)
    sel = np.concatenate([np.arange(row_ptr[r], row_ptr[r + 1]) for r in rows])
    return rp, col[sel], w[sel], np.asarray(out_row)[rows]




def _csr(row_ptr, col, w, out_row):
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
    col = np.ascontiguousarray(col, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    out_row = np.ascontiguousarray(out_row, dtype=np.int32)
    if len(row_ptr) != len(out_row) + 1 or row_ptr[-1] != len(col) or len(w) != len(col):
        raise ValueError("inconsistent CSR arrays")
    return row_ptr, col, w, out_row


def build_stream_plan(row_ptr, col, w, out_row, max_group_rows: int = 64, max_group_src: int = 0) -> RoundPlan:
    """Streamed-form plan (tal_round_plan_build_stream): groups of <= max_group_rows
    consecutive rows (and <= max_group_src distinct sources if > 0) whose sources stream through
    an LDS ring, so cliques and other dense neighborhoods of any size run without the LDS bound
    of build_plan.  Needs every row in reference order (sorted neighbors, then self)."""
    row_ptr, col, w, out_row = _csr(row_ptr, col, w, out_row)
    rows = len(out_row)
    L = _lib.load()
    P32 = ctypes.POINTER(ctypes.c_int32)
    size = L.tal_round_plan_words(rows, len(col))
    info = RoundPlanInfo()
    for _ in range(2):
        blob = np.zeros(size, dtype=np.int32)
        rc = L.tal_round_plan_build_stream(rows, row_ptr.ctypes.data_as(P32), col.ctypes.data_as(P32),
                                           w.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                           out_row.ctypes.data_as(P32), int(max_group_rows),
                                           int(max_group_src), blob.ctypes.data_as(P32), size,
                                           ctypes.byref(info))
        if rc == _lib.TAL_ERR_CAPACITY and info.words > size:
            size = int(info.words)
            continue
        break
    check(rc)
    return RoundPlan(info=info, host=blob[: info.words].copy(), rows=rows, nnz=len(col))


def rows_uniform(row_ptr, w) -> bool:
    """Every row's operands share one fp32 weight (unweighted_module_avg, scale_agg): the
    narrow plans' row-weight form, on which the broadcast form never won."""
    w32 = np.asarray(w, dtype=np.float64).astype(np.float32)
    rp = np.asarray(row_ptr)
    first = np.repeat(w32[rp[:-1]], np.diff(rp))
    return bool(np.array_equal(w32, first))


def tune_candidates(row_ptr, col, w, out_row, bf16: bool = False, mode: int = MODE_EXACT):
    """tune_plan's candidates [(key, plan)], the default plan first (host-side plans)."""
    base = default_plan(row_ptr, col, w, out_row, bf16=bf16, mode=mode)
    if base.spec is None:
        base.spec = {}
    cands = [(("default",), base)]
    sparse = []
    for c4 in TILE_WIDTHS:
        for budget in LDS_BUDGETS:
            try:
                p = build_plan(row_ptr, col, w, out_row, c4=c4, lds_bytes=budget, dense=0)
            except _lib.TalError:
                continue
            sparse.append(p)
    if sparse:
        fewest = min(p.staged_rows() for p in sparse)
        for p in sparse:
            key = (p.info.c4, p.info.n_groups, p.info.total_src, p.info.max_src)
            if p.staged_rows() <= 1.25 * fewest and all(key != k for k, _ in cands) and p.spec != base.spec:
                cands.append((key, p))
    for c4, waves, wg in (BCAST_CANDIDATES if not rows_uniform(row_ptr, w) else ()):
        try:
            p = build_plan(row_ptr, col, w, out_row, c4=c4, lds_bytes=LDS_BUDGETS[-1], bcast=waves, bcast_wg=wg)
        except _lib.TalError:
            continue
        key = ("bcast", c4, waves, wg)
        if all(key != k for k, _ in cands) and p.spec != base.spec:
            cands.append((key, p))
    if not bf16 and not isinstance(base, CliquePlan):
        cp = build_clique_plan(row_ptr, col, w, out_row)
        if cp is not None:
            cp.spec = dict(clique=1, rest=cp.rest.spec if cp.rest is not None else None)
            cands.append((("clique",), cp))
    return cands


def tune_plan(row_ptr, col, w, out_row, pool_in: torch.Tensor, pool_out: torch.Tensor,
              n: Optional[int] = None, reps: int = 5, mode: int = MODE_EXACT,
              margin: float = 0.01) -> RoundPlan:
    """Pick the plan by measurement, anchored on the untimed default (default_plan).

    Candidates are the forms that have won a measured round on some BASELINE config (DESIGN §4
    "Plan forms and their selection"): the sparse form at every tile width and LDS budget whose
    staging stays within 1.25 x the fewest staged sources of any candidate (multi-group plans
    that re-read sources - config 3's 80 KiB c4 = 128 plan stages 3.7x - never won), the
    broadcast forms that won (BCAST_CANDIDATES) on rounds with per-operand weights, and the
    clique plan (tune_candidates).  Dense row blocks, the streamed form and the
    register-resident groups lost every measured A/B outside their probes (BENCH_r04: 5.9, 7.0
    and 8.5-16 ms against 2.0 ms on config 3) and are built only on request (plan_from_spec).

    Each candidate runs `reps` times, interleaved rep by rep with the others, and is judged by
    its median; one slower than TUNE_DROP x the default on its first timed run is not timed
    again (its median comes from that run).  A candidate replaces the default only when its
    median beats the default's by more than `margin` (round 4: the tuner's single short timings
    once kept a plan slower than the default - 23.74 vs 22.89 ms).  pool_out must not alias
    pool_in."""
    if pool_in.data_ptr() == pool_out.data_ptr():
        raise ValueError("tune_plan needs distinct input / output pools")
    bf16 = pool_in.dtype == torch.bfloat16  # bf16 rounds: sparse and narrow plans only
    run = round_bf16 if bf16 else round_f32
    cands = tune_candidates(row_ptr, col, w, out_row, bf16=bf16, mode=mode)
    base = cands[0][1]
    if isinstance(base, CliquePlan) and base.rest is not None:  # the rows outside the cliques: tuned too
        r_rp, r_col, r_w, r_out = _sub_csr(row_ptr, col, w, out_row, base.rest_rows)
        base.rest = tune_plan(r_rp, r_col, r_w, r_out, pool_in, pool_out, n=n, reps=reps, mode=mode, margin=margin)
        base.spec = dict(clique=1, rest=base.rest.spec)
    if len(cands) == 1:
        return base.to(pool_in.device)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _, p in cands:
        p.to(pool_in.device)
        run(pool_in, pool_out, p, n=n, mode=mode)  # warm (LDS attribute, code load)
    # candidates interleaved rep by rep, so a clock or thermal drift during tuning does not
    # favour the ones timed first
    ts = [[] for _ in cands]
    live = list(range(len(cands)))
    for rep in range(reps):
        for k in live:
            s.record()
            run(pool_in, pool_out, cands[k][1], n=n, mode=mode)
            e.record()
            e.synchronize()
            ts[k].append(s.elapsed_time(e))
        if rep == 0:  # far slower than the default on its first timed run: not timed again
            live = [k for k in live if k == 0 or ts[k][0] <= TUNE_DROP * ts[0][0]]
    med = [float(np.median(tk)) for tk in ts]
    timings = [{"form": "/".join(map(str, key)), "ms": round(t, 4), "all_ms": [round(x, 4) for x in tk], "spec": p.spec}
               for (key, p), t, tk in zip(cands, med, ts)]
    k_best = int(np.argmin(med))
    if med[k_best] >= (1.0 - margin) * med[0]:
        k_best = 0  # not clearly faster than the default: keep the default
    best = cands[k_best][1]
    best.tuned_ms = med[k_best]
    best.candidates = timings
    return best


def plan_from_spec(row_ptr, col, w, out_row, spec: dict) -> RoundPlan:
    """Rebuild a plan tune_plan chose (its `spec`): profiling runs then time the same plan
    without re-tuning."""
    if spec.get("clique"):
        p = build_clique_plan(row_ptr, col, w, out_row, rest_spec=spec.get("rest"))
        if p is None:
            raise ValueError("plan spec asks for clique blocks but the round has none")
        p.spec = dict(spec)
        return p
    if spec.get("reg"):
        p = build_reg_plan(row_ptr, col, w, out_row, int(spec.get("max_src", REG_MAX_SRC)))
        if p is None:
            raise ValueError("plan spec asks for register groups but a row has too many sources")
        p.spec = dict(spec)
        return p
    if "rows_k1" in spec:
        return row_call_plan(row_ptr, col, w, out_row)
    if "stream_rows" in spec:
        p = build_stream_plan(row_ptr, col, w, out_row, int(spec["stream_rows"]), int(spec["stream_src"]))
    else:
        p = build_plan(row_ptr, col, w, out_row, c4=int(spec["c4"]), lds_bytes=int(spec["lds"]),
                       dense=int(spec["dense"]), bcast=int(spec.get("bcast", 0)), bcast_wg=int(spec.get("bcwg", 2)))
    p.spec = dict(spec)
    return p


def default_plan(row_ptr, col, w, out_row, bf16: bool = False, mode: int = MODE_EXACT):
    """The plan the round components build when they do not time candidates (tune=False):
    the round's uniform-weight clique blocks by K3c when it has any (fp32 pools; the other rows
    by their own sparse plan), else build_plan's sparse form at the tile width and LDS budget
    its cost model picks.  On the round-1 A/B tables this is the measured winner's form for
    configs 2-5 (tests/test_host_logic.py::test_default_plan_forms).  One exception, from
    round 4's measurements: a round whose narrow plan needs per-operand weights (the pairs
    form: centrality weights on a graph whose degrees differ) runs the narrow kernel's
    broadcast form with the whole source set in one LDS tile — for bf16 in FMA mode the
    two-chunk form (c4 = 32, 16 wavefronts, one workgroup per CU; config 5 with
    degree-centrality weights: 23.0-23.3 ms against 23.7-24.4 for the 16 x 2 form, 32.1-32.6 for
    the pairs form and 29.8-30.1 for the register-resident K3r, which round 3 picked;
    profiles/r04/r04j, profiles/r04/pmc), for fp32 8 wavefronts x 2 (38.2-42.2 ms against 46.0
    for the cost model's two-group pairs plan; profiles/r04/r04f).  The broadcast plan is taken
    only when it has no more groups than the sparse plan; RoundExecutor runs a single-group
    plan (config 5's: every source in one tile) in place and a multi-group one through its
    scratch pool.  A round with a row of more distinct sources than one LDS tile holds (e.g.
    `unweighted_fl` over > ~620 clients) gets a streamed plan - the fp32 streamed kernel, or for
    bf16 pools the wide-row kernel - or, rows out of reference order, one K1 call per row
    (RowCallPlan)."""
    try:
        if not bf16:
            cp = build_clique_plan(row_ptr, col, w, out_row)
            if cp is not None:
                cp.spec = dict(clique=1, rest=cp.rest.spec if cp.rest is not None else None)
                return cp
        p = build_plan(row_ptr, col, w, out_row, dense=0)
    except _lib.TalError as exc:
        if exc.code != _lib.TAL_ERR_CAPACITY:
            raise
        # a row with more distinct sources than one LDS tile holds: fp32 rounds stream their
        # sources through an LDS ring (k_round_stream), bf16 rounds through LDS chunks in groups
        # of 16 rows (k_round_wide); rows in reference order either way; other operand orders
        # run one K1 call per row
        try:  # fp32: the streamed kernel's groups of 64 rows; bf16: the wide-row form's 16
            rows = 64 if not bf16 else WIDE_ROWS
            p = build_stream_plan(row_ptr, col, w, out_row, max_group_rows=rows)
            p.spec = {"stream_rows": rows, "stream_src": 0}
            return p
        except _lib.TalError:
            pass
        return row_call_plan(row_ptr, col, w, out_row)
    if p.info.c4 < 64 and not p.info.narrow_roww and (not bf16 or mode == MODE_FMA):
        # per-operand weights on a narrow plan: the broadcast form with every source in one LDS
        # tile - bf16 FMA: the two-chunk form (c4 = 32, one workgroup per CU) when its 512-B
        # tiles hold the group, else 16 wavefronts x 2; fp32: 8 wavefronts x 2 (its 1024-thread
        # two-workgroup form spills; the two-chunk form ran alike)
        forms = [(32, 16, 1), (16, 16, 2)] if bf16 else [(16, 8, 2)]
        for c4, waves, wg in forms:
            try:
                bp = build_plan(row_ptr, col, w, out_row, c4=c4, lds_bytes=LDS_BUDGETS[-1], bcast=waves, bcast_wg=wg)
            except _lib.TalError:  # a row past 128 / waves records: no broadcast form
                continue
            if bp.info.n_groups <= p.info.n_groups:
                return bp
    return p


WIDE_ROWS = 16  # rows per group of the bf16 wide-row form (k_round_wide, kWideRows)


def round_kernel_name(plan, bf16: bool = False) -> str:
    """Which K3 kernel tal_agg_round_f32 (bf16: tal_agg_round_bf16) launches for this plan or plan
    info (mirrors launch_round_vec); clique plans name the K3c kernel (their rest rows run a
    second one)."""
    if isinstance(plan, CliquePlan):
        return "k_round_clique"
    if isinstance(plan, RegPlan):
        return "k_round_reg"
    if isinstance(plan, RowCallPlan):
        return "k_agg (one call per row)"
    info = plan.info if isinstance(plan, RoundPlan) else plan
    if info.stream_cs:
        return "k_round_wide" if bf16 else "k_round_stream"
    if info.c4 < 64:
        return "k_round_f32_narrow"
    threads = 1024 if info.c4 == 64 else 512
    j_max = 20 if threads <= 512 else 8
    loads = info.max_src * info.c4
    return "k_round_f32_persistent" if loads <= j_max * threads else "k_round_f32_tiled"


def _blocks_per_cu(info: RoundPlanInfo) -> int:
    if info.c4 < 64:  # narrow kernel: 1024 threads, data tile + plan slice
        return max(1, min(2, (160 * 1024) // max(1, info.lds_bytes)))
    lds = max(1, info.max_src * info.c4 * 16)
    return max(1, min(4, (160 * 1024) // lds))


def _plan_cost(info: RoundPlanInfo) -> float:
    """Estimated seconds per element column of the round (see build_plan)."""
    eff = {1: 0.33, 2: 0.6}.get(_blocks_per_cu(info), 0.8)
    if info.c4 <= 64:
        eff *= 0.5  # one float4 column per lane: half the LDS reads in flight of the c4=128 form
    hbm = 4.0 * (info.total_src + info.rows) / 5.5e12
    lds = 4.0 * info.dense_reads / (150e12 * eff)
    return max(hbm, lds)


def round_f32(pool_in: torch.Tensor, pool_out: torch.Tensor, plan, n: Optional[int] = None,
              mode: int = MODE_EXACT, stream=None) -> torch.Tensor:
    """K3 on [models, ld] fp32 pools (snapshot semantics; see tal_agg.h).  A CliquePlan runs
    its clique blocks with K3c and its other rows with their regular plan (out of place)."""
    if isinstance(plan, CliquePlan):
        return _round_clique(pool_in, pool_out, plan, n, mode, stream)
    if isinstance(plan, RegPlan):
        return _round_reg(pool_in, pool_out, plan, n, torch.float32, mode, stream)
    if isinstance(plan, RowCallPlan):
        return _round_rows(pool_in, pool_out, plan, n, torch.float32, mode, stream)
    return _round(pool_in, pool_out, plan, n, torch.float32, mode, stream)


def _round_clique(pool_in, pool_out, plan: CliquePlan, n, mode, stream):
    _require_gpu(pool_in, "pool_in", torch.float32)
    _require_gpu(pool_out, "pool_out", torch.float32)
    if pool_in.dim() != 2 or pool_out.dim() != 2:
        raise ValueError("pools must be 2-D [models, ld]")
    if pool_in.device != pool_out.device:
        raise ValueError("pools on different devices")
    if pool_in.data_ptr() == pool_out.data_ptr():
        raise ValueError("a clique round runs out of place (snapshot semantics)")
    if plan.device is None or plan.device.device != pool_in.device:
        plan.to(pool_in.device)
    n = pool_in.shape[1] if n is None else int(n)
    if (pool_in.stride(0) | pool_out.stride(0)) % 2 or (pool_in.data_ptr() | pool_out.data_ptr()) % 8:
        # K3c reads and writes 8-B column pairs: rows that are not 8-B aligned take the full plan
        return _round(pool_in, pool_out, plan.full, n, torch.float32, mode, stream)
    t = plan.table.reshape(plan.n_cliques, CLIQUE_WORDS)
    att = t[:, 4 + 2 * CLIQUE_MAX:].reshape(plan.n_cliques, CLIQUE_EXTRA, CLIQUE_EXTRA_WORDS)
    used = np.arange(CLIQUE_EXTRA)[None, :] < t[:, 2:3]  # attached records in use
    if max(t[:, 4: 4 + CLIQUE_MAX].max(), att[used][:, [5, 7, 8]].max(initial=-1)) >= pool_in.shape[0]:
        raise ValueError("plan reads a pool row beyond pool_in")
    if max(t[:, 4 + CLIQUE_MAX: 4 + 2 * CLIQUE_MAX].max(), att[used][:, 0].max(initial=-1)) >= pool_out.shape[0]:
        raise ValueError("plan writes a pool row beyond pool_out")
    L = _lib.load()
    check(L.tal_agg_round_clique_f32(ctypes.c_void_p(pool_in.data_ptr()), pool_in.stride(0),
                                     ctypes.c_void_p(pool_out.data_ptr()), pool_out.stride(0), n,
                                     ctypes.c_void_p(plan.device.data_ptr()), plan.n_cliques, plan.mmax,
                                     int(mode), _stream(pool_in.device, stream)))
    if plan.rest is not None:
        _round(pool_in, pool_out, plan.rest, n, torch.float32, mode, stream)
    return pool_out


def round_i64(pool_in: torch.Tensor, pool_out: torch.Tensor, plan: RoundPlan, n: Optional[int] = None,
              stream=None) -> torch.Tensor:
    if isinstance(plan, (CliquePlan, RegPlan)):
        plan = plan.full
    if isinstance(plan, RowCallPlan):
        return _round_rows(pool_in, pool_out, plan, n, torch.int64, MODE_EXACT, stream)
    return _round(pool_in, pool_out, plan, n, torch.int64, MODE_EXACT, stream)


def round_bf16(pool_in: torch.Tensor, pool_out: torch.Tensor, plan: RoundPlan, n: Optional[int] = None,
               mode: int = MODE_EXACT, stream=None) -> torch.Tensor:
    """K3 on [models, ld] bf16 pools (sparse, narrow or - rows wider than one LDS tile - streamed
    plans of at most 16 rows per group, the wide-row kernel; modes as agg_bf16)."""
    if isinstance(plan, CliquePlan):
        plan = plan.full
    if isinstance(plan, RegPlan):
        return _round_reg(pool_in, pool_out, plan, n, torch.bfloat16, mode, stream)
    if isinstance(plan, RowCallPlan):
        return _round_rows(pool_in, pool_out, plan, n, torch.bfloat16, mode, stream)
    return _round(pool_in, pool_out, plan, n, torch.bfloat16, mode, stream)


_ROUND_FN = {torch.float32: "tal_agg_round_f32", torch.int64: "tal_agg_round_i64",
             torch.bfloat16: "tal_agg_round_bf16"}


def _round(pool_in, pool_out, plan, n, dtype, mode, stream):
    _require_gpu(pool_in, "pool_in", dtype)
    _require_gpu(pool_out, "pool_out", dtype)
    if pool_in.dim() != 2 or pool_out.dim() != 2:
        raise ValueError("pools must be 2-D [models, ld]")
    if pool_in.device != pool_out.device:
        raise ValueError("pools on different devices")
    if plan.device is None or plan.device.device != pool_in.device:
        plan.to(pool_in.device)
    n = pool_in.shape[1] if n is None else int(n)
    rows_in = pool_in.shape[0]
    rows_out = pool_out.shape[0]
    h = plan.host
    i = plan.info
    if h[i.off_src_row: i.off_src_row + i.total_src].max(initial=-1) >= rows_in:
        raise ValueError("plan reads a pool row beyond pool_in")
    if h[i.off_out_row: i.off_out_row + i.rows].max(initial=-1) >= rows_out:
        raise ValueError("plan writes a pool row beyond pool_out")
    L = _lib.load()
    fn = getattr(L, _ROUND_FN[dtype])
    args = [ctypes.c_void_p(pool_in.data_ptr()), pool_in.stride(0), ctypes.c_void_p(pool_out.data_ptr()),
            pool_out.stride(0), n, ctypes.c_void_p(plan.device.data_ptr()), ctypes.byref(plan.info)]
    if dtype != torch.int64:
        args.append(int(mode))
    args.append(_stream(pool_in.device, stream))
    check(fn(*args))
    return pool_out


# ------------------------------------------------------------------------------------------
# K2 cosine similarity
# ------------------------------------------------------------------------------------------
@dataclass
class CosinePlan:
    n_seg: int
    n_chunks: int
    host: np.ndarray
    device: Optional[torch.Tensor] = None
    threads: int = 1


def build_cosine_plan(segments: Sequence[Sequence[int]], threads: int = 1) -> CosinePlan:
    """segments: (offset, A, I, B) per parameter tensor (see tal_agg.h K2).  threads: the torch
    intra-op thread count whose reduction order a tensor mean over >= 32768 outputs follows
    (the reference's process's torch.get_num_threads(); 1 = torch's serial order)."""
    seg = np.ascontiguousarray(np.asarray(segments, dtype=np.int64).reshape(-1, 4))
    L = _lib.load()
    P64 = ctypes.POINTER(ctypes.c_int64)
    words = L.tal_cosine_plan_words(seg.ctypes.data_as(P64), len(seg))
    if words < 0:
        raise ValueError("bad cosine segments")
    blob = np.zeros(words, dtype=np.int64)
    nch = ctypes.c_int32()
    check(L.tal_cosine_plan_build(seg.ctypes.data_as(P64), len(seg), blob.ctypes.data_as(P64), words,
                                  ctypes.byref(nch)))
    check(L.tal_cosine_plan_set_threads(blob.ctypes.data_as(P64), int(threads)))
    return CosinePlan(n_seg=len(seg), n_chunks=nch.value, host=blob, threads=int(threads))


def cosine(a_list: Sequence[torch.Tensor], b_list: Sequence[torch.Tensor], plan: CosinePlan,
           stream=None) -> torch.Tensor:
    """K2: cosine_similarity(a_j, b_j) for every pair (flat fp32 parameter arenas), the
    reference's fp32 value bit for bit."""
    if len(a_list) != len(b_list) or not a_list:
        raise ValueError("need matching, non-empty a/b lists")
    dev = a_list[0].device
    for i, t in enumerate(list(a_list) + list(b_list)):
        _require_gpu(t, f"model {i}", torch.float32)
        if t.device != dev:
            raise ValueError("models on different devices")
    if plan.device is None or plan.device.device != dev:
        plan.device = torch.from_numpy(plan.host).to(dev)
    L = _lib.load()
    P64 = ctypes.POINTER(ctypes.c_int64)
    hp = plan.host.ctypes.data_as(P64)
    scratch = torch.empty(int(L.tal_cosine_scratch_bytes(hp, len(a_list))), dtype=torch.uint8, device=dev)
    out = torch.empty(len(a_list), dtype=torch.float32, device=dev)
    check(L.tal_cosine_params(_lib.ptr_array([t.data_ptr() for t in a_list]),
                              _lib.ptr_array([t.data_ptr() for t in b_list]), len(a_list),
                              ctypes.c_void_p(plan.device.data_ptr()), hp, plan.n_chunks,
                              ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                              _stream(dev, stream)))
    return out


def host_cosine(a_list: Sequence[torch.Tensor], b_list: Sequence[torch.Tensor], plan: CosinePlan) -> torch.Tensor:
    """K2's arithmetic on the host (tal_host_cosine): cosine_similarity(a_j, b_j) for flat
    contiguous CPU fp32 parameter arenas, the reference's fp32 value bit for bit, in a process
    that sees no GPU (similarity.cosine_pairs dispatches on torch.cuda.is_available())."""
    if len(a_list) != len(b_list) or not a_list:
        raise ValueError("need matching, non-empty a/b lists")
    for i, t in enumerate(list(a_list) + list(b_list)):
        if t.device.type != "cpu" or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"host_cosine: model {i} must be a contiguous CPU float32 tensor")
    out = torch.empty(len(a_list), dtype=torch.float32)
    L = _lib.load()
    check(L.tal_host_cosine(_lib.ptr_array([t.data_ptr() for t in a_list]), _lib.ptr_array([t.data_ptr() for t in b_list]),
                            len(a_list), plan.host.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                            ctypes.c_void_p(out.data_ptr())))
    return out


# ------------------------------------------------------------------------------------------
# Synthetic pool rows (benchmark / full-size test inputs)
# ------------------------------------------------------------------------------------------
_FILL_TORCH = {0: torch.float32, 1: torch.bfloat16, 2: torch.int64}


def fill_counter(seg: torch.Tensor, table: np.ndarray, dtype_code: int, stream=None) -> torch.Tensor:
    """tal_fill_counter: rows 0..n_rows-1 of the [rows, ld] segment `seg` = synth's counter
    generator per `table` (synth.fill_table), one launch for all rows."""
    if seg.device.type != "cuda" or seg.dtype != _FILL_TORCH[int(dtype_code)]:
        raise ValueError(f"fill_counter needs a GPU {_FILL_TORCH[int(dtype_code)]} segment (got {seg.device} {seg.dtype})")
    tab = np.ascontiguousarray(table, dtype=np.int64)
    n_rows, n = int(tab[0]), int(tab[1])
    if seg.dim() != 2 or seg.stride(1) != 1 or seg.shape[0] < n_rows or seg.shape[1] < n:
        raise ValueError(f"seg must be [>= {n_rows}, >= {n}] with unit column stride (got {tuple(seg.shape)})")
    dev_tab = torch.from_numpy(tab).to(seg.device)
    L = _lib.load()
    check(L.tal_fill_counter(ctypes.c_void_p(seg.data_ptr()), seg.stride(0), int(dtype_code),
                             ctypes.c_void_p(dev_tab.data_ptr()), tab.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                             _stream(seg.device, stream)))
    return seg
