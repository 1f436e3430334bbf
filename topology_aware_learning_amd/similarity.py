"""Model-to-model cosine similarity (K2), for the `*_sim` aggregation strategies: the GPU kernels,
or - in a process that sees no GPU - the library's host form of the same arithmetic
(tal_host_cosine).

Reference: cosine_similarity, src/decentralized_client.py:661-681 — over `named_parameters`
(buffers excluded), nn.CosineSimilarity(dim=1, eps=1e-6) per tensor (1-D tensors get a
trailing unit dim), mean per tensor, average over tensors.  K2 performs the reference's fp32
operations in the order of the torch CPU kernels it runs on (include/tal_agg.h), so the
values are the reference's bit for bit and sim_centrality_module_avg's arg-min (:511) —
near-ties and exact fp32 ties included — picks the reference's neighbor
(tests/golden/near_ties.*).  A tensor mean over >= 32768 outputs (ViT-B/16's patch embedding,
196,608) is a two-pass parallel sum in torch whose order depends on the intra-op thread count;
K2 follows torch.get_num_threads() of the calling process (tests/golden/cosine_threads.json).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn as nn

from . import ops
from .aggregate import _device_for, _stage, layout_of_module
from .arena import bound_row

_plans: Dict[Tuple, ops.CosinePlan] = {}


def _param_names(model: nn.Module) -> List[str]:
    return [n for n, _ in model.named_parameters()]


def _flat(models: Sequence[nn.Module], layout, device) -> List[torch.Tensor]:
    out: List = [None] * len(models)
    rest = []
    for j, m in enumerate(models):
        b = bound_row(m)
        if b is not None and b[0].device == device and b[0].layout == layout:
            out[j] = b[0].row_f32(b[1])
        else:
            rest.append(j)
    if rest:
        staged = _stage([models[j] for j in rest], layout, device)
        for k, j in enumerate(rest):
            out[j] = staged[k]["f32"]
    return out


def cosine_pairs(model: nn.Module, others: Sequence[nn.Module]) -> List[float]:
    """[cosine_similarity(model, o) for o in others] in one kernel launch."""
    if not others:
        return []
    layout = layout_of_module(model)
    names = _param_names(model)
    # a tensor mean over >= 32768 outputs follows torch's parallel order for this process's
    # intra-op thread count, as the reference's own call would (tal_agg.h K2).  The plan holds
    # at most 1024 (tal_cosine_plan_set_threads); a process with more intra-op threads gets
    # 1024's order, which differs from torch's only for a tensor mean over > 1024 x 32768
    # outputs (none in the reference's models: ViT-B/16's largest is 196,608)
    threads = max(1, min(torch.get_num_threads(), 1024))
    key = (layout.key, tuple(names), threads)
    plan = _plans.get(key)
    if plan is None:
        plan = ops.build_cosine_plan(layout.param_segments(names), threads=threads)
        _plans[key] = plan
    if not torch.cuda.is_available():  # no GPU (config 1's setting): the library's host K2
        flats = _host_flat([model, *others], layout)
        return [float(x) for x in ops.host_cosine([flats[0]] * len(others), flats[1:], plan).tolist()]
    device = _device_for([model, *others])
    b0 = bound_row(model)
    mp = getattr(b0[0], "multi", None) if b0 is not None else None
    bounds = [bound_row(m) for m in others]
    if mp is not None and all(b is not None and mp[0].member(b[0]) is not None for b in bounds):
        # clients over several GPUs (multipool.MultiPool): the neighbors other GPUs own are read
        # from this GPU's ghost rows, refreshed first
        pool = b0[0]
        with torch.cuda.device(pool.device):
            rows = mp[0].rows_for(mp[1], bounds)
            res = ops.cosine([pool.row_f32(b0[1])] * len(others), [pool.row_f32(r) for r in rows], plan)
            return [float(x) for x in res.cpu().tolist()]
    flats = _flat([model, *others], layout, device)
    res = ops.cosine([flats[0]] * len(others), flats[1:], plan)
    return [float(x) for x in res.cpu().tolist()]


def _host_flat(models: Sequence[nn.Module], layout) -> List[torch.Tensor]:
    """Each model's fp32 segment as a contiguous CPU tensor: a pinned-row view when the model
    is bound to a host row, else its fp32 entries concatenated in state_dict order."""
    out = []
    for j, m in enumerate(models):
        b = bound_row(m)
        if b is not None and b[0].device.type == "cpu" and b[0].layout == layout:
            out.append(b[0].row_f32(b[1]))
            continue
        sd = m.state_dict()
        layout.check_compatible(sd, f"model {j}")
        if any(t.device.type != "cpu" for t in sd.values()):
            raise RuntimeError("no GPU is visible, but a model has tensors off the CPU")
        out.append(torch.cat([t.detach().reshape(-1) for t in layout.flatten_cat(sd, "f32")]))
    return out
