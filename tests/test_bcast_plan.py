"""Host side of the narrow kernel's broadcast form (tal_round_plan_build_bcast): the wavefront
programs laid out in the plan blob must decode back to every row's operands, weights and output
row, in reference order, with identity pads only where a pass's rows are shorter than its
longest.  No GPU: this reads the blob the kernel reads (include/tal_agg.h, narrow_bcast)."""
import networkx as nx
import numpy as np
import pytest

from oracle import reference_alg as ra
from topology_aware_learning_amd import ops

import bench

HDR = 8


def _decode(plan, c4):
    """{out_row: [(slot, weight bits)]} from the blob, plus the pad count."""
    info, h = plan.info, plan.host
    waves = info.narrow_bcast
    R = info.bc_rec_max
    assert R == 128 // waves and R * waves >= 120
    one = np.float32(1.0).view(np.int32)
    rows = {}
    pads = 0
    for g in range(info.n_groups):
        ns = h[info.off_grp_src_ptr + g + 1] - h[info.off_grp_src_ptr + g]
        src = h[info.off_src_row + h[info.off_grp_src_ptr + g]: info.off_src_row + h[info.off_grp_src_ptr + g + 1]]
        for wv in range(waves):
            o = int(h[info.off_bc_prog + g * waves + wv])
            assert o % 2 == 0
            n_rec, n_pass, data = int(h[o]), int(h[o + 1]), int(h[o + 2])
            assert n_rec <= R and data % 2 == 0 and data >= HDR + R + 4 * n_pass
            acc = {}
            for r in range(n_rec):
                d = int(h[o + HDR + r])
                cnt, last, ps = d & 0xFF, (d >> 8) & 1, d >> 16
                assert 1 <= cnt <= 16 and ps < n_pass
                rec = h[o + data + 128 * r: o + data + 128 * (r + 1)].reshape(64, 2)
                for lane in range(64):  # 4 rows of 16 lanes at both widths (c4 = 32: two chunks a lane)
                    sub, u = lane // 16, lane % 16
                    if u >= cnt:
                        continue
                    off, wb = int(rec[lane, 0]), int(rec[lane, 1])
                    assert off % (c4 * 16) == 0
                    acc.setdefault((ps, sub), []).append((off // (c4 * 16), wb))
                if last:
                    outs = h[o + HDR + R + 4 * ps: o + HDR + R + 4 * ps + 4]
                    for sub in range(4):
                        ops_ = acc.pop((ps, sub), [])
                        if outs[sub] < 0:
                            assert all(s == ns and wb == one for s, wb in ops_)
                            continue
                        real, padded = [], False
                        for s, wb in ops_:
                            if s == ns:  # identity pad: -0.0 tile, weight 1.0, only at the end
                                assert wb == one
                                pads += 1
                                padded = True
                                continue
                            assert not padded
                            real.append((int(src[s]), wb))
                        assert int(outs[sub]) not in rows
                        rows[int(outs[sub])] = real
            assert not acc
    return rows, pads


@pytest.mark.parametrize("waves,wg", [(8, 2), (12, 2), (16, 2), (16, 1)])
@pytest.mark.parametrize("c4", [16, 32])
@pytest.mark.parametrize("graph", ["sbm256", "regular", "gnp", "ring"])
def test_bcast_programs_decode_to_csr(graph, c4, waves, wg):
    if graph == "sbm256":
        orders, ws = bench.round_spec(256, 8, kind="sbm", weights="degcent")
    else:
        g = {"regular": nx.random_regular_graph(8, 64, seed=0), "gnp": nx.gnp_random_graph(150, 0.08, seed=2),
             "ring": nx.cycle_graph(16)}[graph]
        cent = nx.degree_centrality(g)
        orders = [sorted(g.neighbors(i)) + [i] for i in sorted(g.nodes)]
        ws = [ra.centrality_weights(o, cent, True, 10.0) for o in orders]
    row_ptr, col, w = ra.round_csr(orders, ws)
    rows = len(orders)
    out_rows = np.random.default_rng(rows).permutation(rows).astype(np.int32)
    plan = ops.build_plan(row_ptr, col, w, out_rows, c4=c4, lds_bytes=160 * 1024, bcast=waves, bcast_wg=wg)
    info = plan.info
    assert info.narrow_bcast == waves and info.c4 == c4 and info.narrow_roww == 0 and info.bc_wg_per_cu == wg
    assert info.lds_bytes <= (80 if wg == 2 else 160) * 1024
    # staging: at most what the form's launch stages - the library's one table, which the
    # launcher reads too (tests/test_gpu_bcast.py launches plans at and past the limit)
    max_loads = ops._lib.load().tal_round_bcast_max_loads(c4, waves, wg)
    assert max_loads >= 2 * 64 * waves
    assert max(plan.host[info.off_grp_src_ptr + g + 1] - plan.host[info.off_grp_src_ptr + g]
               for g in range(info.n_groups)) * c4 <= max_loads
    assert info.lds_bytes == max(
        (plan.host[info.off_grp_src_ptr + g + 1] - plan.host[info.off_grp_src_ptr + g] + 1) * c4 * 16
        for g in range(info.n_groups))
    dec, pads = _decode(plan, c4)
    assert sorted(dec) == sorted(out_rows.tolist())
    for r in range(rows):
        want = [(int(col[k]), int(np.float32(w[k]).view(np.int32))) for k in range(row_ptr[r], row_ptr[r + 1])]
        assert dec[int(out_rows[r])] == want
    if graph == "sbm256" and (c4 == 16 or wg == 1):
        assert info.n_groups == 1 and info.total_src == 256  # every source read once per round
    assert info.bc_records * 16 * 4 >= len(col)  # a record carries 16 operands of each row of a pass


def test_bcast_rejects_bad_arguments():
    L = ops._lib.load()
    assert L.tal_round_bcast_max_loads(64, 16, 2) == -1 and L.tal_round_bcast_max_loads(16, 10, 2) == -1
    orders, ws = bench.round_spec(64, 8)
    row_ptr, col, w = ra.round_csr(orders, ws)
    out = np.arange(64, dtype=np.int32)
    for c4, waves, wg in ((64, 16, 2), (16, 4, 2), (16, 10, 2), (16, 16, 3)):
        with pytest.raises(ops._lib.TalError):
            ops.build_plan(row_ptr, col, w, out, c4=c4, lds_bytes=80 * 1024, bcast=waves, bcast_wg=wg)


def test_bcast_record_capacity():
    """A group whose records exceed the wavefronts' registers splits; a single row with more
    operands than 16 x (128 / waves) cannot be placed at all (TAL_ERR_CAPACITY)."""
    m = 16 * 16 + 1  # one row of 257 operands: 17 records > 16 (8 waves) and > 8 (16 waves)
    row_ptr = np.array([0, m], dtype=np.int32)
    col = np.arange(m, dtype=np.int32) % 200
    w = np.full(m, 1.0 / m)
    with pytest.raises(ops._lib.TalError):
        ops.build_plan(row_ptr, col, w, np.zeros(1, dtype=np.int32), c4=16, lds_bytes=160 * 1024, bcast=8)
