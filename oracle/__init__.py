"""TEST INFRASTRUCTURE — the CPU oracle for the aggregation hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / the timed CPU baseline: the product (topology_aware_learning_amd,
src/) never imports it and has no CPU fallback.

Contents
  cosine_oracle.c          the reference's model cosine similarity in torch's exact CPU
                           reduction order (`cosine_model`, bitwise; decentralized_client.py:661-681)
  agg_oracle.c / Makefile  plain-C restatement of the reference arithmetic
                           (src/decentralized_client.py:399-413) — `agg_f32`, `agg_i64`,
                           `round_f32`, `round_i64`, and for bf16 tensors `agg_bf16`,
                           `round_bf16` (uint16 bit patterns) below are its numpy wrappers
  reference_alg.py         numpy restatement of the host-side logic on the path: weight
                           vectors of every app, cosine similarity, round semantics
  torch_path.py            the reference loop restated with the same torch CPU ops
                           (clone / mul / add_ / load_state_dict) — bench.py's cpu_baseline

Pinning: tests/test_oracle_golden.py checks all of it against golden vectors generated from
the reference itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle_agg.so"


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        srcs = [HERE / "agg_oracle.c", HERE / "cosine_oracle.c"]
        if not LIB.exists() or any(LIB.stat().st_mtime < s.stat().st_mtime for s in srcs):
            build()
        L = ctypes.CDLL(str(LIB))
        P = ctypes.c_void_p
        L.oracle_agg_f32.argtypes = [P, P, ctypes.c_int32, P, ctypes.c_int64]
        L.oracle_agg_i64.argtypes = [P, P, ctypes.c_int32, P, ctypes.c_int64]
        rargs = [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, P, P, P, P]
        L.oracle_round_f32.argtypes = rargs
        L.oracle_round_i64.argtypes = rargs
        L.oracle_agg_bf16.argtypes = [P, P, ctypes.c_int32, P, ctypes.c_int64, ctypes.c_int32]
        L.oracle_round_bf16.argtypes = rargs + [ctypes.c_int32]
        L.oracle_f32_to_bf16.argtypes = [P, P, ctypes.c_int64]
        L.oracle_cosine_scratch.argtypes = [P, ctypes.c_int32]
        L.oracle_cosine_scratch.restype = ctypes.c_int64
        L.oracle_cosine_model.argtypes = [P, P, P, ctypes.c_int32, P, P]
        L.oracle_cosine_model.restype = ctypes.c_float
        L.oracle_cosine_model_t.argtypes = [P, P, P, ctypes.c_int32, ctypes.c_int32, P, P]
        L.oracle_cosine_model_t.restype = ctypes.c_float
        L.oracle_cosine_outputs.argtypes = [P, P, P, ctypes.c_int32, P, P, P]
        _lib = L
    return _lib


def _ptrs(arrs):
    a = (ctypes.c_void_p * len(arrs))()
    for i, x in enumerate(arrs):
        a[i] = x.ctypes.data
    return a


def agg_f32(xs, w) -> np.ndarray:
    """One call, fp32 operands (list of equal-length 1-D arrays), float64 weights."""
    xs = [np.ascontiguousarray(x, dtype=np.float32).reshape(-1) for x in xs]
    w = np.ascontiguousarray(w, dtype=np.float64)
    out = np.empty_like(xs[0])
    lib().oracle_agg_f32(_ptrs(xs), w.ctypes.data, len(xs), out.ctypes.data, out.size)
    return out


def agg_i64(xs, w) -> np.ndarray:
    xs = [np.ascontiguousarray(x, dtype=np.int64).reshape(-1) for x in xs]
    w = np.ascontiguousarray(w, dtype=np.float64)
    out = np.empty_like(xs[0])
    lib().oracle_agg_i64(_ptrs(xs), w.ctypes.data, len(xs), out.ctypes.data, out.size)
    return out


def _round(fn, pool_in, row_ptr, col, w, out_row, pool_out):
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
    col = np.ascontiguousarray(col, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    out_row = np.ascontiguousarray(out_row, dtype=np.int32)
    assert pool_in.flags.c_contiguous and pool_out.flags.c_contiguous
    fn(pool_in.ctypes.data, pool_in.shape[1], pool_out.ctypes.data, pool_out.shape[1], pool_in.shape[1],
       len(out_row), row_ptr.ctypes.data, col.ctypes.data, w.ctypes.data, out_row.ctypes.data)
    return pool_out


def round_f32(pool_in, row_ptr, col, w, out_row, pool_out=None) -> np.ndarray:
    """Snapshot round over a [models, n] fp32 pool (pool_out defaults to a copy of pool_in)."""
    pool_in = np.ascontiguousarray(pool_in, dtype=np.float32)
    if pool_out is None:
        pool_out = pool_in.copy()
    return _round(lib().oracle_round_f32, pool_in, row_ptr, col, w, out_row, pool_out)


def round_i64(pool_in, row_ptr, col, w, out_row, pool_out=None) -> np.ndarray:
    pool_in = np.ascontiguousarray(pool_in, dtype=np.int64)
    if pool_out is None:
        pool_out = pool_in.copy()
    return _round(lib().oracle_round_i64, pool_in, row_ptr, col, w, out_row, pool_out)


# ---- bf16 (numpy has no bf16: arrays of uint16 bit patterns) -------------------------------
def f32_to_bf16(x) -> np.ndarray:
    """fp32 -> bf16 bits, round to nearest even, NaN -> 0xFFFF (torch's vectorized conversion)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.shape, dtype=np.uint16)
    lib().oracle_f32_to_bf16(x.ctypes.data, out.ctypes.data, x.size)
    return out


def bf16_to_f32(b) -> np.ndarray:
    b = np.ascontiguousarray(b, dtype=np.uint16)
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)


def agg_bf16(xs, w, exact: bool = True) -> np.ndarray:
    """One call on bf16 operands.  exact: the reference's torch ops on bf16 tensors (every
    product and partial sum rounded to bf16); else fp32 fused accumulation, one rounding."""
    xs = [np.ascontiguousarray(x, dtype=np.uint16).reshape(-1) for x in xs]
    w = np.ascontiguousarray(w, dtype=np.float64)
    out = np.empty_like(xs[0])
    lib().oracle_agg_bf16(_ptrs(xs), w.ctypes.data, len(xs), out.ctypes.data, out.size, int(bool(exact)))
    return out


def round_bf16(pool_in, row_ptr, col, w, out_row, pool_out=None, exact: bool = True) -> np.ndarray:
    pool_in = np.ascontiguousarray(pool_in, dtype=np.uint16)
    if pool_out is None:
        pool_out = pool_in.copy()
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
    col = np.ascontiguousarray(col, dtype=np.int32)
    w = np.ascontiguousarray(w, dtype=np.float64)
    out_row = np.ascontiguousarray(out_row, dtype=np.int32)
    lib().oracle_round_bf16(pool_in.ctypes.data, pool_in.shape[1], pool_out.ctypes.data, pool_out.shape[1],
                            pool_in.shape[1], len(out_row), row_ptr.ctypes.data, col.ctypes.data, w.ctypes.data,
                            out_row.ctypes.data, int(bool(exact)))
    return pool_out


def cosine_model(a, b, segments, per_tensor: bool = False, threads: int = 1):
    """The reference's cosine_similarity(model_1, model_2) of two flat fp32 parameter rows,
    bit for bit (torch's CPU reduction order; cosine_oracle.c).  segments: (offset, A, I, B)
    per parameter in named_parameters order (arena.StateLayout.param_segments).  threads: the
    torch intra-op thread count of the reference's process (matters for tensor means over
    >= 32768 outputs only)."""
    if not 1 <= int(threads) <= 1024:  # cosine_oracle.c MAX_THREADS (the library's limit too)
        raise ValueError(f"threads must be in 1..1024, got {threads}")
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    seg = np.ascontiguousarray(np.asarray(segments, dtype=np.int64).reshape(-1, 4))
    L = lib()
    scratch = np.empty(max(1, L.oracle_cosine_scratch(seg.ctypes.data, len(seg))), np.float32)
    per = np.empty(len(seg), np.float32)
    v = L.oracle_cosine_model_t(a.ctypes.data, b.ctypes.data, seg.ctypes.data, len(seg), int(threads),
                                scratch.ctypes.data, per.ctypes.data)
    v = np.float32(v)
    return (v, per) if per_tensor else v


def cosine_outputs(a, b, segments):
    """Debug view of cosine_model: (per-output values s of every tensor, per-tensor means)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    seg = np.ascontiguousarray(np.asarray(segments, dtype=np.int64).reshape(-1, 4))
    L = lib()
    scratch = np.empty(max(1, L.oracle_cosine_scratch(seg.ctypes.data, len(seg))), np.float32)
    n_out = int(sum(int(r[1]) * int(r[3]) for r in seg))
    s = np.empty(n_out, np.float32)
    means = np.empty(len(seg), np.float32)
    L.oracle_cosine_outputs(a.ctypes.data, b.ctypes.data, seg.ctypes.data, len(seg), scratch.ctypes.data,
                            s.ctypes.data, means.ctypes.data)
    return s, means
