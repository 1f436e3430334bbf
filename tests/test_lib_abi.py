"""The C-ABI library loads and exports every symbol include/tal_agg.h declares; argument
errors are reported through status codes + tal_last_error (no GPU needed); the product path
refuses CPU tensors instead of computing on the CPU."""
import ctypes
import re

import numpy as np
import pytest
import torch

from topology_aware_learning_amd import _lib, ops

from conftest import ROOT


def header_functions():
    text = (ROOT / "include" / "tal_agg.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int32_t|int64_t)\s+(tal_\w+)\(", text, re.M)))


def test_exports_every_declared_symbol():
    L = _lib.load()
    declared = header_functions()
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTED) == declared
    assert L.tal_abi_version() == _lib.ABI_VERSION


def test_library_is_gfx950_code():
    data = (ROOT / "topology_aware_learning_amd" / "libtal_agg.so").read_bytes()
    assert b"gfx950" in data


def test_error_status_and_message():
    L = _lib.load()
    P = (ctypes.c_void_p * 1)()
    W = (ctypes.c_double * 1)(1.0)
    rc = L.tal_agg_f32(P, W, 0, None, 10, 1, None)
    assert rc == _lib.TAL_ERR_INVALID and b"m must be" in L.tal_last_error()
    rc = L.tal_agg_i64(P, W, 1, None, 10, None)
    assert rc == _lib.TAL_ERR_INVALID and b"null" in L.tal_last_error()
    rc = L.tal_agg_f32(P, W, 1, None, 0, 1, None)  # n == 0: nothing to do
    assert rc == _lib.TAL_OK
    info = _lib.RoundPlanInfo()
    rc = L.tal_agg_round_f32(None, 4, None, 4, 4, None, ctypes.byref(info), 1, None)
    assert rc == _lib.TAL_ERR_INVALID
    assert L.tal_round_plan_words(-1, 0) == -1
    assert L.tal_cosine_scratch_bytes(None, 1) == -1


def test_cosine_plan_threads_word():
    """The cosine plan carries torch's intra-op thread count (header word 2): 1 after build,
    set by tal_cosine_plan_set_threads within 1..1024; an unbuilt plan or a count out of range
    is refused."""
    import numpy as np

    from topology_aware_learning_amd import ops

    plan = ops.build_cosine_plan([(0, 768, 3, 256), (196608 * 3, 768, 1, 1)])
    assert plan.host[2] == 1 and plan.threads == 1
    plan8 = ops.build_cosine_plan([(0, 768, 3, 256)], threads=8)
    assert plan8.host[2] == 8
    L = _lib.load()
    P64 = ctypes.POINTER(ctypes.c_int64)
    for bad in (0, -3, 1025):
        assert L.tal_cosine_plan_set_threads(plan.host.ctypes.data_as(P64), bad) == _lib.TAL_ERR_INVALID
        assert b"threads" in L.tal_last_error()
    blank = np.zeros(8, dtype=np.int64)
    assert L.tal_cosine_plan_set_threads(blank.ctypes.data_as(P64), 4) == _lib.TAL_ERR_INVALID
    assert L.tal_cosine_plan_set_threads(None, 4) == _lib.TAL_ERR_INVALID
    assert L.tal_cosine_plan_set_threads(plan.host.ctypes.data_as(P64), 1024) == _lib.TAL_OK
    assert plan.host[2] == 1024


def test_halo_exchange_argument_errors():
    """The halo section's entry points validate before touching a GPU or RCCL."""
    L = _lib.load()
    comm = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(_lib.TAL_COMM_ID_BYTES)
    assert L.tal_comm_init(None, 1, 0, uid, 0) == _lib.TAL_ERR_INVALID
    assert L.tal_comm_init(ctypes.byref(comm), 0, 0, uid, 0) == _lib.TAL_ERR_INVALID
    assert L.tal_comm_init(ctypes.byref(comm), 2, 2, uid, 0) == _lib.TAL_ERR_INVALID
    assert L.tal_comm_unique_id(None) == _lib.TAL_ERR_INVALID
    assert L.tal_comm_destroy(None) == _lib.TAL_ERR_INVALID
    n = (ctypes.c_int64 * 1)(0)
    assert L.tal_halo_exchange(None, 1, None, n, None, n, None) == _lib.TAL_ERR_INVALID
    assert b"bad arguments" in L.tal_last_error()
    fake = ctypes.c_void_p(0x1000)
    assert L.tal_halo_pack(fake, 64, 4, fake, 0, 64, fake, None) == _lib.TAL_OK  # no rows: nothing
    assert L.tal_halo_pack(fake, 64, 4, fake, 2, 6, fake, None) == _lib.TAL_ERR_INVALID  # 6-byte rows
    assert b"aligned" in L.tal_last_error()
    assert L.tal_halo_pack(fake, 32, 4, fake, 2, 64, fake, None) == _lib.TAL_ERR_INVALID  # pitch < row


def test_in_place_multi_group_rejected():
    import networkx as nx

    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    row_ptr = np.cumsum([0] + [len(o) for o in orders]).astype(np.int32)
    col = np.concatenate(orders).astype(np.int32)
    w = np.full(len(col), 1 / 9)
    plan = ops.build_plan(row_ptr, col, w, np.arange(64, dtype=np.int32), c4=64, lds_bytes=16 * 1024)
    assert plan.info.n_groups > 1
    L = _lib.load()
    buf = ctypes.c_void_p(0x1000)
    rc = L.tal_agg_round_f32(buf, 64, buf, 64, 64, buf, ctypes.byref(plan.info), 1, None)
    assert rc == _lib.TAL_ERR_INVALID and b"in-place" in L.tal_last_error()


def test_ops_refuse_cpu_tensors():
    x = torch.zeros(8)
    with pytest.raises(ValueError, match="GPU"):
        ops.agg_f32([x], [1.0], torch.zeros(8))
    with pytest.raises(ValueError, match="GPU"):
        ops.agg_i64([x.long()], [1.0], torch.zeros(8, dtype=torch.int64))


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.TalLibraryError, match="no CPU fallback"):
        _lib.load(tmp_path / "libtal_agg.so")


def test_aggregate_without_gpu_runs_the_library_or_fails_loudly(monkeypatch):
    """No GPU visible: the aggregation is the library's host reduction (native code, the
    kernels' arithmetic; tests/test_host_backend.py pins it bitwise), and without the library
    it raises TalLibraryError - there is no Python arithmetic path."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from topology_aware_learning_amd import _lib
    from topology_aware_learning_amd.aggregate import aggregate_models

    a, b = torch.nn.Linear(2, 2), torch.nn.Linear(2, 2)
    want = {k: (0.5 * a.state_dict()[k] + 0.5 * b.state_dict()[k]) for k in a.state_dict()}
    aggregate_models([a, b], [0.5, 0.5], b)
    for k, v in b.state_dict().items():
        assert torch.equal(v, want[k])
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", _lib.LIB_PATH.with_name("missing_libtal_agg.so"))
    with pytest.raises(_lib.TalLibraryError):
        aggregate_models([a, b], [0.5, 0.5], b)
