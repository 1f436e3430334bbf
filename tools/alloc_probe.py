"""Probe (not part of the product): the config-3 round kernel timed on pools from different
allocations in one process (torch's caching allocator, plain hipMalloc, hipExtMallocWithFlags
with hipDeviceMallocContiguous) - isolates placement effects when bench.py and
tools/tune/bw_probe disagree on the same board."""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from topology_aware_learning_amd import _lib, ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import StateLayout  # noqa: E402
from topology_aware_learning_amd.round import csr_from_lists  # noqa: E402


def main():
    import networkx as nx

    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    n, ld = lay.n_f32, lay.ld_f32
    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    rp, col, w = csr_from_lists(orders, [[1 / 9] * 9] * 64)
    dev = torch.device("cuda", 0)
    L = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    nbytes = 64 * ld * 4
    src = torch.randn(64, ld, device=dev)
    plans = {c4: ops.plan_from_spec(rp, col, w, np.arange(64, dtype=np.int32), {"c4": c4, "lds": 81920, "dense": 0}).to(dev)
             for c4 in (64, 32)}
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def alloc(kind):
        if kind == "torch":
            t = torch.empty(nbytes // 4, device=dev)
            return t.data_ptr(), t
        p = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(p), nbytes) if kind == "hipMalloc" else \
            hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, 4)  # hipDeviceMallocContiguous
        assert rc == 0, (kind, rc)
        return p.value, None

    hip.hipFree.argtypes = [ctypes.c_void_p]
    keep = []
    sweep = [a for a in sys.argv[1:] if a.startswith("pad")]
    kinds = [a for a in sys.argv[1:] if not a.startswith("pad")] or ["torch", "hipMalloc", "contiguous",
                                                                     "hipMalloc", "contiguous", "torch"]
    pads = [int(a[3:]) for a in sweep] or [0]
    base_ld = ld
    for kind in kinds:
      for pad in pads:
        ld = base_ld + pad
        nbytes = 64 * ld * 4
        pin, t1 = alloc(kind)
        pout, t2 = alloc(kind)
        keep += [t1, t2]
        assert hip.hipMemcpy(ctypes.c_void_p(pin), ctypes.c_void_p(src.data_ptr()), 64 * base_ld * 4, 3) == 0
        res = {}
        for c4, plan in plans.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for r in range(13):
                s.record()
                rc = L.tal_agg_round_f32(ctypes.c_void_p(pin), ld, ctypes.c_void_p(pout), ld, n,
                                         ctypes.c_void_p(plan.device.data_ptr()), ctypes.byref(plan.info), 1, stream)
                e.record()
                e.synchronize()
                assert rc == 0
                if r >= 3:
                    ts.append(s.elapsed_time(e))
            res[c4] = round(float(np.mean(ts)), 3)
        print(kind, "ld+%d" % pad, res, hex(pin), hex(pout), flush=True)
        if kind != "torch":
            hip.hipFree(ctypes.c_void_p(pin))
            hip.hipFree(ctypes.c_void_p(pout))
        keep.clear()
        torch.cuda.empty_cache()


def combos():
    """Two input and three output pools (plain hipMalloc), every pairing timed: does the slow
    mode follow one pool or the pair?"""
    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    n, ld = lay.n_f32, lay.ld_f32
    import networkx as nx

    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    rp, col, w = csr_from_lists(orders, [[1 / 9] * 9] * 64)
    dev = torch.device("cuda", 0)
    L = _lib.load()
    plan = ops.plan_from_spec(rp, col, w, np.arange(64, dtype=np.int32), {"c4": 32, "lds": 81920, "dense": 0}).to(dev)
    ins = [torch.randn(64, ld, device=dev) for _ in range(3)]
    outs = [torch.empty(64, ld, device=dev) for _ in range(3)]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i, a in enumerate(ins):
        row = []
        for j, b in enumerate(outs):
            ts = []
            for r in range(8):
                s.record()
                ops.round_f32(a, b, plan, n=n)
                e.record()
                e.synchronize()
                if r >= 2:
                    ts.append(s.elapsed_time(e))
            row.append(round(float(np.mean(ts)), 3))
        print("in", i, "outs:", row, flush=True)
    # read-only and write-only streams over each pool (torch reduction / fill)
    for i, a in enumerate(ins):
        s.record(); a.sum(); e.record(); e.synchronize()
        s.record(); x = a.sum(); e.record(); e.synchronize()
        rd = s.elapsed_time(e)
        s.record(); outs[i].fill_(1.0); e.record(); e.synchronize()
        s.record(); outs[i].fill_(1.0); e.record(); e.synchronize()
        print("pool", i, "read GB/s %.0f" % (a.numel() * 4 / rd / 1e6), "write(out %d) GB/s %.0f" % (i, a.numel() * 4 / s.elapsed_time(e) / 1e6))


def stride_sweep():
    """One input pool; three output buffers; on each the output row stride ld + d is swept over
    the SAME memory: does the slow mode follow the stride or the allocation?"""
    lay = StateLayout.from_layout(synth.get_layout("resnet50"))
    n, ld = lay.n_f32, lay.ld_f32
    import networkx as nx

    g = nx.random_regular_graph(8, 64, seed=0)
    orders = [sorted(g.neighbors(i)) + [i] for i in range(64)]
    rp, col, w = csr_from_lists(orders, [[1 / 9] * 9] * 64)
    dev = torch.device("cuda", 0)
    plan = ops.plan_from_spec(rp, col, w, np.arange(64, dtype=np.int32), {"c4": 32, "lds": 81920, "dense": 0}).to(dev)
    a = torch.randn(64, ld, device=dev)
    ds = [0, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 65536]
    bufs = [torch.empty(64 * (ld + max(ds)), device=dev) for _ in range(3)]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for bi, buf in enumerate(bufs):
        row = []
        for d in ds:
            b = buf[: 64 * (ld + d)].view(64, ld + d)
            ts = []
            for r in range(8):
                s.record()
                ops.round_f32(a, b, plan, n=n)
                e.record()
                e.synchronize()
                if r >= 2:
                    ts.append(s.elapsed_time(e))
            row.append(round(float(np.mean(ts)), 2))
        print("out buf", bi, dict(zip(ds, row)), flush=True)


if __name__ == "__main__":
    combos() if "--combos" in sys.argv else stride_sweep() if "--stride" in sys.argv else main()
