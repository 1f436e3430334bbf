"""Fused FedProx proximal term over device-pool models.

Reference (tasks.py:277-286), once per training batch:

    proximal_term = 0.0
    for neighbor in neighbors:
        for w, w_t in zip(client.model.parameters(), neighbor.model.parameters()):
            proximal_term += (w - w_t).norm(2)
    loss += (prox_coeff / 2) * proximal_term

With the client and its neighbors bound to rows of one ModelPool, `prox_term` computes every
norm in one pass over the rows (tal_prox_norms: the client row read once per 8 neighbors from
cache, each neighbor row once) and its gradient in one more (tal_prox_grad), instead of
2·K·P small torch ops per batch.  Gradients flow to the client's parameters and, as in the
reference (whose neighbor parameters are leaves with requires_grad), to neighbor parameters
that require grad.  Numerics: fp32 squares summed per chunk, chunks combined in double
(deterministic); the reference's torch norm uses its own fp32 reduction order, so parity is a
tolerance (tests/test_gpu_interface.py).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check
from .arena import StateLayout, bound_row


class ProxPlan:
    """Chunk plan of the parameter segments of one layout on one device."""

    def __init__(self, layout: StateLayout, param_names: Sequence[str], device):
        entries = [layout.by_name[n] for n in param_names]
        for n, e in zip(param_names, entries):
            if e.seg != "f32":
                raise NotImplementedError(f"parameter {n} is not fp32")
        self.names = list(param_names)
        self.offsets = [int(e.offset) for e in entries]
        self.shapes = [tuple(e.shape) for e in entries]
        self.numels = [int(e.numel) for e in entries]
        seg = np.array([x for o, m in zip(self.offsets, self.numels) for x in (o, m)], dtype=np.int64)
        L = _lib.load()
        P64 = ctypes.POINTER(ctypes.c_int64)
        words = L.tal_prox_plan_words(seg.ctypes.data_as(P64), len(entries))
        if words < 0:
            raise ValueError("empty or invalid parameter segments")
        blob = np.zeros(words, dtype=np.int64)
        nc = ctypes.c_int32()
        check(L.tal_prox_plan_build(seg.ctypes.data_as(P64), len(entries), blob.ctypes.data_as(P64), words,
                                    ctypes.byref(nc)))
        self.n_seg = len(entries)
        self.n_chunks = int(nc.value)
        self.device = torch.device(device)
        self.plan = torch.from_numpy(blob).to(self.device)


_plans: Dict[tuple, ProxPlan] = {}


def _plan_for(layout: StateLayout, names: Sequence[str], device) -> ProxPlan:
    key = (id(layout), tuple(names), str(device))
    p = _plans.get(key)
    if p is None:
        p = _plans[key] = ProxPlan(layout, names, device)
    return p


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def prox_norms(pool, row: int, neighbor_rows: Sequence[int], plan: ProxPlan) -> torch.Tensor:
    """norms[t, p] = ||w_p - wt_p||_2 for the pool rows (float32 [K, P])."""
    L = _lib.load()
    k = len(neighbor_rows)
    scratch = torch.empty(int(L.tal_prox_scratch_bytes(plan.n_chunks, k)), dtype=torch.uint8, device=pool.device)
    norms = torch.empty((k, plan.n_seg), dtype=torch.float32, device=pool.device)
    wt = _lib.ptr_array([pool.row_f32(r).data_ptr() for r in neighbor_rows])
    check(L.tal_prox_norms(ctypes.c_void_p(pool.row_f32(row).data_ptr()), wt, k,
                           ctypes.c_void_p(plan.plan.data_ptr()), plan.n_chunks, plan.n_seg,
                           ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(norms.data_ptr()),
                           _stream(pool.device)))
    return norms


class _ProxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, plan, pool, row, neighbor_rows, n_client, *params):
        norms = prox_norms(pool, row, neighbor_rows, plan)
        ctx.plan, ctx.pool, ctx.row, ctx.neighbor_rows, ctx.n_client = plan, pool, row, list(neighbor_rows), n_client
        ctx.needs = [p.requires_grad for p in params]
        ctx.save_for_backward(norms)
        return norms.double().sum().float()

    @staticmethod
    def backward(ctx, g):
        (norms,) = ctx.saved_tensors
        plan, pool, k, P = ctx.plan, ctx.pool, len(ctx.neighbor_rows), ctx.n_client
        L = _lib.load()
        scale = g.detach().to(torch.float32).reshape(1).contiguous()
        n = pool.layout.ld_f32
        gw = torch.zeros(n, dtype=torch.float32, device=pool.device)
        want_t = [any(ctx.needs[P + t * P: P + (t + 1) * P]) for t in range(k)]
        gwt = [torch.zeros(n, dtype=torch.float32, device=pool.device) if wnt else None for wnt in want_t]
        wt = _lib.ptr_array([pool.row_f32(r).data_ptr() for r in ctx.neighbor_rows])
        gwt_p = _lib.ptr_array([x.data_ptr() if x is not None else 0 for x in gwt])
        check(L.tal_prox_grad(ctypes.c_void_p(pool.row_f32(ctx.row).data_ptr()), wt, k,
                              ctypes.c_void_p(plan.plan.data_ptr()), plan.n_chunks, plan.n_seg,
                              ctypes.c_void_p(norms.data_ptr()), ctypes.c_void_p(scale.data_ptr()),
                              ctypes.c_void_p(gw.data_ptr()), gwt_p, _stream(pool.device)))

        def views(buf, need):
            return [buf[o: o + m].view(s) if nd else None
                    for o, m, s, nd in zip(plan.offsets, plan.numels, plan.shapes, need)]

        grads = views(gw, ctx.needs[:P])
        for t in range(k):
            need = ctx.needs[P + t * P: P + (t + 1) * P]
            grads += views(gwt[t], need) if gwt[t] is not None else [None] * P
        return (None, None, None, None, None, *grads)


def prox_term(model: torch.nn.Module, neighbor_models: Sequence[torch.nn.Module]) -> Optional[torch.Tensor]:
    """sum_t sum_p ||w_p - wt_p||_2 with autograd, when the model and every neighbor are rows of
    one device ModelPool; None otherwise (the caller keeps the reference's torch loop)."""
    if not neighbor_models:
        return None
    b = bound_row(model)
    if b is None or b[0].device.type != "cuda":
        return None
    pool, row = b
    rows: List[int] = []
    for m in neighbor_models:
        nb = bound_row(m)
        if nb is None or nb[0] is not pool:
            return None
        rows.append(nb[1])
    names = [n for n, _ in model.named_parameters()]
    plan = _plan_for(pool.layout, names, pool.device)
    params = [p for _, p in model.named_parameters()]
    for m in neighbor_models:
        params += [p for _, p in m.named_parameters()]
    return _ProxFn.apply(plan, pool, row, rows, len(names), *params)
