"""K2 staged-kernel phase timing (not part of the product): one tensor shape, 8 pairs, with a
diagnostic build of the library that stamps s_memtime at each phase boundary of k_cosine_staged
(tools/tune/libtal_agg_stamps.so, TAL_LIB_PATH).  Prints per-phase median cycles over
workgroups: plan reads, staging (loads + LDS writes + barrier), norms, level-0 runs, combine.
usage: TAL_LIB_PATH=tools/tune/libtal_agg_stamps.so python tools/cosine_stamps.py 512,512,3,3
Historical: it patches the slab-staged K2 kernel, which the streamed column kernels replaced
(run it on a checkout of commit 17a9a02 or earlier; profiles/r06/stamps holds its output)."""
import ctypes
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from topology_aware_learning_amd import _lib, ops  # noqa: E402


def main():
    shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "512,512,3,3").split(","))
    n = int(np.prod(shape))
    seg = (0, shape[0], shape[1] if len(shape) > 1 else 1, int(np.prod(shape[2:])) if len(shape) > 2 else 1)
    g = torch.Generator(device="cuda").manual_seed(0)
    rows = torch.randn(9, n, device="cuda", generator=g)
    plan = ops.build_cosine_plan([seg])
    a, b = [rows[0]] * 8, [rows[1 + j] for j in range(8)]
    for _ in range(3):
        ops.cosine(a, b, plan)
    torch.cuda.synchronize()
    L = _lib.load()
    L.tal_debug_stamps.restype = ctypes.c_int32
    L.tal_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    buf = np.zeros(16384 * 8, dtype=np.uint64)
    assert L.tal_debug_stamps(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(-1, 8).astype(np.int64)
    live = st[:, 5] > 0
    st = st[live]
    if not len(st):
        print(json.dumps(dict(shape=shape, staged=False, note="no staged chunk: the direct form")), flush=True)
        return
    names = ["plan", "stage", "norms", "runs", "combine"]
    d = {nm: float(np.median(st[:, k + 1] - st[:, k])) for k, nm in enumerate(names)}
    d["total"] = float(np.median(st[:, 5] - st[:, 0]))
    d["span_start_to_last_end"] = float(st[:, 5].max() - st[:, 0].min())
    d["workgroups"] = int(live.sum())
    print(json.dumps(dict(shape=shape, median_cycles=d)), flush=True)


if __name__ == "__main__":
    main()
