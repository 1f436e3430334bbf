"""Debug (not part of the product): K2's per-output values and per-tensor means against the C
oracle's on one tiny golden case; prints the first differing tensors."""
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from topology_aware_learning_amd import _lib, ops, synth  # noqa: E402
from topology_aware_learning_amd.arena import StateLayout  # noqa: E402

G = ROOT / "tests" / "golden"
TINY = json.loads((G / "tiny_cases.json").read_text())
Z = np.load(G / "tiny_cases.npz")
lay = [(n, tuple(s), d) for n, s, d in TINY["layout"]]
layout = StateLayout.from_layout(lay)
segs = layout.param_segments(synth.param_names(lay))
plan = ops.build_cosine_plan(segs)
dev = torch.device("cuda", 0)
L = _lib.load()
bad = 0
for case in [c for c in TINY["cases"] if c["fn"] == "sim_centrality_module_avg"]:
    ci, M = case["case"], case["M"]
    flat = [np.concatenate([Z[f"c{ci}_in{i}_{n}"].reshape(-1) for n, _, d in lay if d == "float32"]) for i in range(M)]
    for j in range(M - 1):
        s_ref, m_ref = oracle.cosine_outputs(flat[-1], flat[j], segs)
        a = torch.from_numpy(flat[-1]).to(dev)
        b = torch.from_numpy(flat[j]).to(dev)
        plan.device = torch.from_numpy(plan.host).to(dev)
        hp = plan.host.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
        nb = int(L.tal_cosine_scratch_bytes(hp, 1))
        scratch = torch.zeros(nb // 4, dtype=torch.float32, device=dev)
        out = torch.empty(1, dtype=torch.float32, device=dev)
        _lib.check(L.tal_cosine_params(_lib.ptr_array([a.data_ptr()]), _lib.ptr_array([b.data_ptr()]), 1,
                                       ctypes.c_void_p(plan.device.data_ptr()), hp, plan.n_chunks,
                                       ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(out.data_ptr()), None))
        sc = scratch.cpu().numpy()
        s_got, m_got = sc[: len(s_ref)], sc[len(s_ref): len(s_ref) + len(segs)]
        ds = np.flatnonzero(s_got.view(np.uint32) != s_ref.view(np.uint32))
        dm = np.flatnonzero(m_got.view(np.uint32) != m_ref.view(np.uint32))
        if len(ds) or len(dm):
            bad += 1
            starts = np.cumsum([0] + [int(r[1]) * int(r[3]) for r in segs])
            print("case", ci, "pair", j, "out diffs at", ds[:8].tolist(), "tensors",
                  sorted({int(np.searchsorted(starts, d, side="right") - 1) for d in ds}),
                  "mean diffs", dm.tolist(), [segs[t] for t in dm.tolist()][:4])
            for d in ds[:3]:
                print("   s", d, s_got[d], s_ref[d])
print("pairs with differences:", bad)
