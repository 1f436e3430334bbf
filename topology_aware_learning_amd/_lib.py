"""ctypes binding of the gfx950 C-ABI library (include/tal_agg.h).

This is the only way the package reaches the device: there is no CPU fallback.  If the
library is missing or fails to load, every operation raises ``TalLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

# torch ships its own libamdhip64.so (soname libamdhip64.so.7, ROCm 7.0).  Loading torch first
# makes the dynamic linker resolve our library's libamdhip64.so.7 dependency to that same
# runtime, so torch's streams and device pointers are valid in our calls.
import torch  # noqa: F401  (import order matters, see above)

# TAL_LIB_PATH: an alternative build of the same library (A/B probes under tools/); default the
# in-tree product build
LIB_PATH = Path(os.environ.get("TAL_LIB_PATH") or Path(__file__).resolve().parent / "libtal_agg.so")

TAL_OK = 0
TAL_ERR_INVALID = 1
TAL_ERR_HIP = 2
TAL_ERR_CAPACITY = 3
TAL_ERR_COMM = 4
TAL_COMM_ID_BYTES = 128
TAL_MODE_FMA = 0
TAL_MODE_EXACT = 1
ABI_VERSION = 25

EXPORTED = (
    "tal_last_error",
    "tal_abi_version",
    "tal_agg_f32",
    "tal_agg_i64",
    "tal_agg_model_f32",
    "tal_agg_bf16",
    "tal_round_plan_words",
    "tal_round_plan_build",
    "tal_round_plan_build_bcast",
    "tal_round_bcast_max_loads",
    "tal_round_plan_build_stream",
    "tal_agg_round_f32",
    "tal_agg_round_i64",
    "tal_agg_round_bf16",
    "tal_agg_round_clique_f32",
    "tal_agg_round_reg",
    "tal_cosine_plan_words",
    "tal_cosine_plan_build",
    "tal_cosine_plan_set_threads",
    "tal_cosine_scratch_bytes",
    "tal_cosine_params",
    "tal_prox_plan_words",
    "tal_prox_plan_build",
    "tal_prox_scratch_bytes",
    "tal_prox_norms",
    "tal_prox_grad",
    "tal_comm_unique_id",
    "tal_comm_init",
    "tal_comm_destroy",
    "tal_halo_pack",
    "tal_halo_exchange",
    "tal_comm_init_local",
    "tal_halo_exchange_local",
    "tal_fill_counter",
    "tal_host_agg_f32",
    "tal_host_agg_i64",
    "tal_host_agg_bf16",
    "tal_host_cosine",
)


class TalLibraryError(RuntimeError):
    """The HIP library is unavailable (not built / not loadable)."""


class TalError(RuntimeError):
    """A C-ABI call returned a non-zero status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[tal status {code}] {msg}")
        self.code = code


class RoundPlanInfo(ctypes.Structure):
    _fields_ = [
        ("rows", ctypes.c_int32),
        ("nnz", ctypes.c_int32),
        ("n_groups", ctypes.c_int32),
        ("total_src", ctypes.c_int32),
        ("max_src", ctypes.c_int32),
        ("max_rows", ctypes.c_int32),
        ("max_nnz", ctypes.c_int32),
        ("c4", ctypes.c_int32),
        ("lds_bytes", ctypes.c_int32),
        ("off_grp_row_ptr", ctypes.c_int32),
        ("off_grp_src_ptr", ctypes.c_int32),
        ("off_src_row", ctypes.c_int32),
        ("off_row_ptr", ctypes.c_int32),
        ("off_op_slot", ctypes.c_int32),
        ("off_op_w", ctypes.c_int32),
        ("off_out_row", ctypes.c_int32),
        ("words", ctypes.c_int32),
        ("dense_rb", ctypes.c_int32),
        ("n_blocks", ctypes.c_int32),
        ("off_grp_blk_ptr", ctypes.c_int32),
        ("off_blk_tab", ctypes.c_int32),
        ("off_dense", ctypes.c_int32),
        ("dense_reads", ctypes.c_int32),
        ("stream_cs", ctypes.c_int32),
        ("off_nrow_ptr", ctypes.c_int32),
        ("off_npairs", ctypes.c_int32),
        ("npairs", ctypes.c_int32),
        ("max_npairs", ctypes.c_int32),
        ("narrow_roww", ctypes.c_int32),
        ("off_nrow_w", ctypes.c_int32),
        ("scalar_lds_bytes", ctypes.c_int32),
        ("narrow_bcast", ctypes.c_int32),
        ("bc_rec_max", ctypes.c_int32),
        ("off_bc_prog", ctypes.c_int32),
        ("bc_records", ctypes.c_int32),
        ("bc_wg_per_cu", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_PP = ctypes.POINTER(ctypes.c_void_p)
_PD = ctypes.POINTER(ctypes.c_double)
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PI64 = ctypes.POINTER(ctypes.c_int64)

_SIGS = {
    "tal_last_error": (ctypes.c_char_p, []),
    "tal_abi_version": (_I32, []),
    "tal_agg_f32": (_I32, [_PP, _PD, _I32, _P, _I64, _I32, _P]),
    "tal_agg_i64": (_I32, [_PP, _PD, _I32, _P, _I64, _P]),
    "tal_agg_model_f32": (_I32, [_PP, _PP, _PD, _I32, _P, _I64, _P, _I64, _I32, _P]),
    "tal_agg_bf16": (_I32, [_PP, _PD, _I32, _P, _I64, _I32, _P]),
    "tal_round_plan_words": (_I64, [_I32, _I64]),
    "tal_round_plan_build": (
        _I32,
        [_I32, _PI32, _PI32, _PD, _PI32, _I32, _I32, _I32, _PI32, _I64, ctypes.POINTER(RoundPlanInfo)],
    ),
    "tal_round_plan_build_bcast": (
        _I32,
        [_I32, _PI32, _PI32, _PD, _PI32, _I32, _I32, _I32, _I32, _PI32, _I64, ctypes.POINTER(RoundPlanInfo)],
    ),
    "tal_round_bcast_max_loads": (_I64, [_I32, _I32, _I32]),
    "tal_round_plan_build_stream": (
        _I32,
        [_I32, _PI32, _PI32, _PD, _PI32, _I32, _I32, _PI32, _I64, ctypes.POINTER(RoundPlanInfo)],
    ),
    "tal_agg_round_f32": (_I32, [_P, _I64, _P, _I64, _I64, _P, ctypes.POINTER(RoundPlanInfo), _I32, _P]),
    "tal_agg_round_i64": (_I32, [_P, _I64, _P, _I64, _I64, _P, ctypes.POINTER(RoundPlanInfo), _P]),
    "tal_agg_round_bf16": (_I32, [_P, _I64, _P, _I64, _I64, _P, ctypes.POINTER(RoundPlanInfo), _I32, _P]),
    "tal_agg_round_clique_f32": (_I32, [_P, _I64, _P, _I64, _I64, _P, _I32, _I32, _I32, _P]),
    "tal_agg_round_reg": (_I32, [_P, _I64, _P, _I64, _I64, _I32, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    "tal_cosine_plan_words": (_I64, [_PI64, _I32]),
    "tal_cosine_plan_build": (_I32, [_PI64, _I32, _PI64, _I64, _PI32]),
    "tal_cosine_plan_set_threads": (_I32, [_PI64, _I32]),
    "tal_cosine_scratch_bytes": (_I64, [_PI64, _I32]),
    "tal_cosine_params": (_I32, [_PP, _PP, _I32, _P, _PI64, _I32, _P, _P, _P]),
    "tal_prox_plan_words": (_I64, [_PI64, _I32]),
    "tal_prox_plan_build": (_I32, [_PI64, _I32, _PI64, _I64, _PI32]),
    "tal_prox_scratch_bytes": (_I64, [_I32, _I32]),
    "tal_prox_norms": (_I32, [_P, _PP, _I32, _P, _I32, _I32, _P, _P, _P]),
    "tal_prox_grad": (_I32, [_P, _PP, _I32, _P, _I32, _I32, _P, _P, _P, _PP, _P]),
    "tal_comm_unique_id": (_I32, [_P]),
    "tal_comm_init": (_I32, [_PP, _I32, _I32, _P, _I32]),
    "tal_comm_destroy": (_I32, [_P]),
    "tal_halo_pack": (_I32, [_P, _I64, _I64, _P, _I32, _I64, _P, _P]),
    "tal_halo_exchange": (_I32, [_P, _I32, _PP, _PI64, _PP, _PI64, _P]),
    "tal_comm_init_local": (_I32, [_PP, _I32, _PI32]),
    "tal_halo_exchange_local": (_I32, [_PP, _I32, _PP, _PI64, _PP, _PI64, _PP]),
    "tal_fill_counter": (_I32, [_P, _I64, _I32, _P, _PI64, _P]),
    "tal_host_agg_f32": (_I32, [_PP, _PD, _I32, _P, _I64, _I32]),
    "tal_host_agg_i64": (_I32, [_PP, _PD, _I32, _P, _I64]),
    "tal_host_agg_bf16": (_I32, [_PP, _PD, _I32, _P, _I64, _I32]),
    "tal_host_cosine": (_I32, [_PP, _PP, _I32, _PI64, _P]),
}

_lock = threading.Lock()
_lib = None


def load(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load (once) and return the library; raises TalLibraryError if it is not there."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = Path(path) if path is not None else LIB_PATH
        if not p.exists():
            raise TalLibraryError(
                f"{p} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback."
            )
        try:
            lib = ctypes.CDLL(str(p))
        except OSError as exc:  # pragma: no cover - depends on the box
            raise TalLibraryError(f"cannot load {p}: {exc}") from exc
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        ver = lib.tal_abi_version()
        if ver != ABI_VERSION:
            raise TalLibraryError(f"{p} has ABI {ver}, expected {ABI_VERSION}: rebuild it")
        if path is None:
            _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != TAL_OK:
        msg = load().tal_last_error().decode(errors="replace")
        raise TalError(rc, msg)


def ptr_array(ptrs) -> ctypes.Array:
    return (ctypes.c_void_p * len(ptrs))(*map(int, ptrs))


def double_array(vals) -> ctypes.Array:
    return (ctypes.c_double * len(vals))(*map(float, vals))
