"""tal_fill_counter: the library's generator of seeded pool rows (synth.py's counter generator).

The benchmark and the full-size parity tests fill their pools with it; the reference-generated
sha256 fixtures (tests/golden/full_round_c{3,4,5}_*.json) pin the rounds computed on exactly
these inputs, so the generator must equal synth.synth_state_dict bit for bit.

CPU: synth.fill_table's runs and running_var ranges, evaluated with numpy, give every segment row
of synth_state_dict.  GPU: the kernel equals synth_state_dict for ResNet-50 and ViT-B/16 rows
(fp32, bf16, int64 segments), including rows with a pitch wider than the segment and a table the
C-ABI must refuse.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from topology_aware_learning_amd import synth
from topology_aware_learning_amd.arena import ModelPool, StateLayout


def _segment_row(layout, seed: int, dtype: str) -> np.ndarray:
    """The `dtype` entries of synth_state_dict(layout, seed) back to back (a pool segment row),
    as bit patterns."""
    sd = synth.synth_state_dict(layout, seed)
    parts = [v.reshape(-1) for (name, _, dt), v in zip(layout, sd.values()) if dt == dtype]
    if not parts:
        return np.zeros(0, dtype=np.int64)
    row = torch.cat(parts)
    return row.view({"float32": torch.int32, "bfloat16": torch.int16, "int64": torch.int64}[dtype]).numpy()


def _emulate(tab: np.ndarray, dtype: str) -> np.ndarray:
    """tal_fill_counter's contract (include/tal_agg.h) evaluated on the host."""
    n_rows, n, n_runs, n_rv, hi = (int(v) for v in tab[:5])
    seeds = tab[8:8 + n_rows]
    runs = tab[8 + n_rows:8 + n_rows + 3 * n_runs].reshape(-1, 3)
    rv = tab[8 + n_rows + 3 * n_runs:].reshape(-1, 2)
    out = []
    for s in seeds:
        pos = np.concatenate([np.arange(p, p + k, dtype=np.uint64) for p, c, k in runs])
        with np.errstate(over="ignore"):
            u = synth._splitmix(pos ^ (np.uint64(int(s)) << np.uint64(40)))
        if dtype == "int64":
            out.append((u % np.uint64(hi)).astype(np.int64))
            continue
        mant = (u & np.uint64(0x7FFFFF)).astype(np.uint32)
        expo = (np.uint64(121) + ((u >> np.uint64(23)) & np.uint64(7))).astype(np.uint32)
        sign = ((u >> np.uint64(31)) & np.uint64(1)).astype(np.uint32)
        f = ((sign << np.uint32(31)) | (expo << np.uint32(23)) | mant).view(np.float32)
        for c, k in rv:
            f[c:c + k] = np.abs(f[c:c + k]) + np.float32(0.5)
        if dtype == "float32":
            out.append(f.view(np.int32))
        else:
            out.append(torch.from_numpy(f.copy()).to(torch.bfloat16).view(torch.int16).numpy())
    assert all(len(o) == n for o in out)
    return np.stack(out) if out else np.zeros((0, n))


@pytest.mark.parametrize("model", ["resnet50", "cifar10"])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16", "int64"])
def test_fill_table_matches_synth(model, dtype):
    lay = synth.get_layout(model)
    if dtype == "bfloat16":
        lay = synth.as_bf16(lay)
    seeds = [3000, 3001 + (1 << 33)]  # only the low 32 bits of a seed count
    tab = synth.fill_table(lay, seeds, dtype)
    want = [_segment_row(lay, s, dtype) for s in seeds]
    if not len(want[0]):
        assert int(tab[1]) == 0
        return
    got = _emulate(tab, dtype)
    for r in range(len(seeds)):
        assert np.array_equal(got[r], want[r]), (model, dtype, r)


def test_fill_table_merges_adjacent_runs():
    """ViT-B/16 has no int64 entry: its fp32 segment is one generator run."""
    tab = synth.fill_table(synth.vit_b16_layout(), [1], "float32")
    assert int(tab[2]) == 1 and int(tab[3]) == 0 and int(tab[1]) == 86_567_656


def test_cpu_fill_rows_torch_unchanged():
    """CPU tensors (the gloo tests) keep the torch generator; it equals synth_state_dict."""
    lay = synth.resnet_layout("resnet18")
    layout = StateLayout.from_layout(lay)
    pool = ModelPool(layout, 2, torch.device("cpu"))
    synth.fill_rows_torch(pool.f32[:2], lay, [5, 6])
    synth.fill_rows_torch(pool.i64[:2], lay, [5, 6], dtype="int64")
    for r, s in enumerate([5, 6]):
        assert np.array_equal(pool.f32[r, :layout.n_f32].view(torch.int32).numpy(), _segment_row(lay, s, "float32"))
        assert np.array_equal(pool.i64[r, :layout.n_i64].numpy(), _segment_row(lay, s, "int64"))


# ------------------------------------------------------------------------------------------
# GPU: the kernel
# ------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("model", ["resnet50", "vit_b16"])
def test_gpu_fill_counter_equals_synth(cuda, model):
    lay = synth.get_layout(model)
    seeds = [3000 + 7, 11 + (1 << 35)] if model == "resnet50" else [5000 + 255]
    for dtype in ("float32", "bfloat16", "int64"):
        dl = synth.as_bf16(lay) if dtype == "bfloat16" else lay
        layout = StateLayout.from_layout(dl)
        pool = ModelPool(layout, len(seeds) + 1, cuda)
        seg = {"float32": pool.f32, "bfloat16": pool.b16, "int64": pool.i64}[dtype]
        n = {"float32": layout.n_f32, "bfloat16": layout.n_b16, "int64": layout.n_i64}[dtype]
        if not n:
            continue
        seg.zero_()
        synth.fill_rows_torch(seg[: len(seeds)], dl, seeds, dtype=dtype)
        view = {"float32": torch.int32, "bfloat16": torch.int16, "int64": torch.int64}[dtype]
        for r, s in enumerate(seeds):
            got = seg[r, :n].view(view).cpu().numpy()
            assert np.array_equal(got, _segment_row(dl, s, dtype)), (model, dtype, r)
            if seg.shape[1] > n:  # the row's padding is not written
                assert not seg[r, n:].view(view).any().item()
        assert not seg[len(seeds)].view(view).any().item()  # rows past the seeds untouched


@pytest.mark.gpu
def test_gpu_fill_counter_one_launch(cuda):
    """The generator is one library launch per segment, whatever the rows and entries."""
    from topology_aware_learning_amd import _lib

    lay = synth.get_layout("resnet50")
    layout = StateLayout.from_layout(lay)
    pool = ModelPool(layout, 64, cuda)
    calls = []
    L = _lib.load()
    real = L.tal_fill_counter

    class Spy:
        def __call__(self, *a):
            calls.append(a)
            return real(*a)

    L.tal_fill_counter = Spy()
    try:
        synth.fill_rows_torch(pool.f32, lay, list(range(64)))
    finally:
        L.tal_fill_counter = real
    assert len(calls) == 1
    torch.cuda.synchronize(cuda)
    want = _segment_row(lay, 63, "float32")
    assert np.array_equal(pool.f32[63, :layout.n_f32].view(torch.int32).cpu().numpy(), want)


@pytest.mark.gpu
def test_gpu_fill_counter_refuses_bad_tables(cuda):
    from topology_aware_learning_amd import ops
    from topology_aware_learning_amd._lib import TalError

    seg = torch.zeros(2, 64, dtype=torch.float32, device=cuda)
    good = np.array([1, 64, 1, 0, 10, 0, 0, 0, 7, 0, 0, 64], dtype=np.int64)
    ops.fill_counter(seg, good, 0)
    gap = np.array([1, 64, 2, 0, 10, 0, 0, 0, 7, 0, 0, 30, 40, 31, 33], dtype=np.int64)  # columns 30 missing
    with pytest.raises(TalError):
        ops.fill_counter(seg, gap, 0)
    short = np.array([1, 64, 1, 0, 10, 0, 0, 0, 7, 0, 0, 60], dtype=np.int64)  # runs end before n
    with pytest.raises(TalError):
        ops.fill_counter(seg, short, 0)
    with pytest.raises(ValueError):
        ops.fill_counter(seg, np.array([3, 64, 1, 0, 10, 0, 0, 0, 1, 2, 3, 0, 0, 64], dtype=np.int64), 0)  # 3 rows > 2
