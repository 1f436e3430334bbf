"""GPU: K1 on the rows of one device pool (ops.agg_pool_rows, the per-call app path on
pool-bound models) is bitwise K1 on the rows' tensor views (agg_model_f32 / agg_f32 / agg_bf16 /
agg_i64), including the in-place case where the output row is the last operand (the app's own
model, decentralized_client.py:399-413), and rejects rows outside the pool."""
import numpy as np
import pytest
import torch

from topology_aware_learning_amd import ops
from topology_aware_learning_amd.arena import ModelPool, StateLayout

pytestmark = pytest.mark.gpu

LAYOUTS = {
    "f32_i64": [("w", (1000, 37), "float32"), ("b", (13,), "float32"), ("n", (3,), "int64")],
    "b16_i64": [("w", (1000, 37), "bfloat16"), ("b", (13,), "bfloat16"), ("n", (3,), "int64")],
    "f32": [("w", (4099,), "float32")],
}


def _pool(lay, rows, dev, seed):
    pool = ModelPool(StateLayout.from_layout(lay), rows, dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    pool.f32.normal_(generator=g)
    pool.b16.copy_(torch.randn(pool.b16.shape, generator=g, device=dev))
    pool.i64.random_(-10 ** 6, 10 ** 6, generator=g)
    return pool


def _views(pool, r):
    return {"f32": pool.row_f32(r), "b16": pool.row_b16(r), "i64": pool.row_i64(r)}


@pytest.mark.parametrize("mode", [ops.MODE_EXACT, ops.MODE_FMA], ids=["exact", "fma"])
@pytest.mark.parametrize("name", list(LAYOUTS))
def test_pool_rows_bitwise_views(cuda, name, mode):
    rows = [3, 0, 7, 5, 1, 6]  # self (6) last, as the apps order their operands
    w = [1 / 6.0] * 5 + [0.3]
    a = _pool(LAYOUTS[name], 8, cuda, 1)
    b = _pool(LAYOUTS[name], 8, cuda, 1)  # same contents: one runs through views, one through rows
    lay = a.layout
    ops.agg_pool_rows(a, rows, w, 6, mode)  # in place on row 6
    segs = [(g, n) for g, n in (("f32", lay.n_f32), ("b16", lay.n_b16), ("i64", lay.n_i64)) if n]
    if lay.n_f32 and lay.n_i64 and not lay.n_b16:
        ops.agg_model_f32([b.row_f32(r) for r in rows], [b.row_i64(r) for r in rows], w, b.row_f32(6),
                          b.row_i64(6), mode)
    else:
        for g, _ in segs:
            xs = [_views(b, r)[g] for r in rows]
            out = _views(b, 6)[g]
            if g == "i64":
                ops.agg_i64(xs, w, out)
            elif g == "f32":
                ops.agg_f32(xs, w, out, mode=mode)
            else:
                ops.agg_bf16(xs, w, out, mode=mode)
    torch.cuda.synchronize()
    for g, t, _ in a.segments():
        iv = {torch.float32: torch.int32, torch.bfloat16: torch.int16, torch.int64: torch.int64}[t.dtype]
        assert torch.equal(t.view(iv), dict((k, tt) for k, tt, _ in b.segments())[g].view(iv)), g
    # the untouched rows really are untouched
    c = _pool(LAYOUTS[name], 8, cuda, 1)
    for g, t, _ in a.segments():
        ref = dict((k, tt) for k, tt, _ in c.segments())[g]
        keep = [r for r in range(8) if r != 6]
        assert torch.equal(t[keep], ref[keep]), g
        assert not torch.equal(t[6], ref[6]), g


def test_pool_rows_rejects_bad_rows(cuda):
    a = _pool(LAYOUTS["f32_i64"], 4, cuda, 2)
    with pytest.raises(IndexError):
        ops.agg_pool_rows(a, [0, 4], [0.5, 0.5], 1)
    with pytest.raises(IndexError):
        ops.agg_pool_rows(a, [0, 1], [0.5, 0.5], -1)
    with pytest.raises(ValueError):
        ops.agg_pool_rows(a, [0, 1], [1.0], 1)
    with pytest.raises(ValueError):
        ops.agg_pool_rows(a, [], [], 1)
    host = ModelPool(a.layout, 2, "cpu")
    with pytest.raises(ValueError):
        ops.agg_pool_rows(host, [0], [1.0], 1)
    np.testing.assert_equal(a.rows, 4)


def test_app_seed_matches_torch_manual_seed(cuda):
    """The apps' per-call seeding (src.decentralized_client.manual_seed) leaves the CPU and every
    GPU generator exactly as the reference's torch.manual_seed(seed) does."""
    from src.decentralized_client import manual_seed

    for seed in (0, 7, 2 ** 40 + 3):
        torch.manual_seed(seed)
        ref_cpu = torch.default_generator.get_state()
        ref_gpu = [g.get_state() for g in torch.cuda.default_generators]
        torch.manual_seed(seed + 1)
        torch.rand(3, device=cuda)
        manual_seed(seed)
        assert torch.equal(torch.default_generator.get_state(), ref_cpu)
        for g, ref in zip(torch.cuda.default_generators, ref_gpu):
            assert torch.equal(g.get_state(), ref)
        a = torch.rand(5, device=cuda)
        torch.manual_seed(seed)
        assert torch.equal(a, torch.rand(5, device=cuda))
