"""Whole-round parity of a device-resident round that does not trust the exchange.

Every simulated device's model is a pure function of (layout, seed) — synth's counter
generator, bitwise the same on any machine — and the bench seeds device i with
``seed_base + i``.  So after the first round each rank can check EVERY output row it owns
without looking at what it received from other GPUs:

* against the reference's own sha256 of that output model, when the workload is one the
  reference-generated fixtures cover (tests/golden/full_round_c{3,4,5}_*.json: the reference's
  aggregation apps, /root/reference/src/decentralized_client.py:418-448 / :553-612, driven per
  client as decentralized_app.py:605-641 does, on exactly these seeded inputs);
* otherwise against K1 (the per-call kernel, pinned to the reference separately) run on the
  row's operands REGENERATED locally from their seeds, never on the received ones.

A halo message that delivers the wrong rows, stale rows or truncated bytes, or an all-to-all
chunk that lands in the wrong place, changes the owned outputs but not the regenerated
operands, so the check fails where a check on the received operands (``spot_check``) passes.
"""
from __future__ import annotations

import hashlib
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Sequence

import torch

from . import ops, synth

_DT = {"f32": ("float32", torch.float32, torch.int32), "b16": ("bfloat16", torch.bfloat16, torch.int16),
       "i64": ("int64", torch.int64, torch.int64)}


def fill_owned(pool, lay, own_ids: Sequence[int], seed_base: int) -> None:
    """Rows 0..len(own_ids)-1 of `pool` = the models of devices own_ids (seed seed_base + id)."""
    seeds = [seed_base + int(g) for g in own_ids]
    for g, t, n in pool.segments():
        synth.fill_rows_torch(t[: len(seeds)], lay, seeds, dtype=_DT[g][0])


def row_digests(seg: torch.Tensor, rows: Sequence[int], ranges, view) -> List[List[str]]:
    """sha256 of seg[r, a:b] (bit patterns as `view`) for r in rows and (a, b) in ranges; rows
    copied to the host one at a time and hashed on a thread pool."""
    lo = min(a for a, _ in ranges)
    hi = max(b for _, b in ranges)
    out: List[List[Optional[str]]] = [[None] * len(ranges) for _ in rows]

    def h(buf, a, b):
        return hashlib.sha256(memoryview(buf[a:b])).hexdigest()

    with ThreadPoolExecutor(8) as ex:
        pending = []
        for k, r in enumerate(rows):
            host = seg[r, lo:hi].view(view).cpu().numpy()
            for q, (a, b) in enumerate(ranges):
                pending.append((k, q, ex.submit(h, host, a - lo, b - lo)))
            if len(pending) > 64:
                for kk, qq, f in pending:
                    out[kk][qq] = f.result()
                pending = []
        for kk, qq, f in pending:
            out[kk][qq] = f.result()
    return out  # type: ignore[return-value]


def check_against_digests(out_pool, own_ids: Sequence[int], expected: Dict[str, Dict[int, List[str]]],
                          ranges: Dict[str, list]) -> List[int]:
    """Own output rows whose digests differ from `expected[seg][global id]` (one digest per
    range of ranges[seg]).  Returns the differing global ids."""
    bad = set()
    for g, t, n in out_pool.segments():
        if g not in expected:
            continue
        got = row_digests(t, range(len(own_ids)), ranges[g], _DT[g][2])
        for k, gid in enumerate(own_ids):
            if got[k] != expected[g][int(gid)]:
                bad.add(int(gid))
    return sorted(bad)


def _k1(seg: str):
    return {"f32": ops.agg_f32, "b16": ops.agg_bf16}.get(seg)


def check_against_k1(out_pool, own_ids: Sequence[int], lay, orders, weights, seed_base: int, mode: int,
                     agg: Optional[Callable] = None, budget_bytes: int = 8 << 30) -> List[int]:
    """Own output rows that differ (bitwise, every segment) from K1 on their operands
    regenerated from the seeds.  Operands are generated once per batch of output rows (as many
    rows as keep the batch's distinct operands within `budget_bytes`) into a scratch pool.
    agg(seg, operand rows, weights, out, mode): the reducer (default K1: ops.agg_f32 /
    agg_bf16 / agg_i64); tests on a host without a GPU pass the oracle.  Returns differing ids."""
    from .arena import ModelPool

    layout = out_pool.layout
    row_bytes = 4 * layout.ld_f32 * bool(layout.n_f32) + 2 * layout.ld_b16 * bool(layout.n_b16) + 8 * layout.ld_i64
    cap = max(max(len(orders[int(g)]) for g in own_ids), int(budget_bytes // max(row_bytes, 1)))

    def default_agg(seg, xs, w, out, m):
        if seg == "i64":
            ops.agg_i64(xs, w, out)
        else:
            _k1(seg)(xs, w, out, mode=m)

    agg = agg or default_agg
    bad = []
    batch: List[int] = []
    need: Dict[int, int] = {}

    def flush():
        if not batch:
            return
        ids = sorted(need)
        slot = {j: s for s, j in enumerate(ids)}
        scratch = ModelPool(layout, len(ids), out_pool.device)
        fill_owned(scratch, lay, ids, seed_base)
        for k in batch:
            gid = int(own_ids[k])
            same = True
            for g, t, n in out_pool.segments():
                src = dict((s, tt) for s, tt, _ in scratch.segments())[g]
                chk = torch.empty(n, dtype=t.dtype, device=t.device)
                agg(g, [src[slot[j], :n] for j in orders[gid]], list(weights[gid]), chk, mode)
                iv = _DT[g][2]
                same = same and torch.equal(chk.view(iv), t[k, :n].view(iv))
            if not same:
                bad.append(gid)
        batch.clear()
        need.clear()
        del scratch

    for k, gid in enumerate(own_ids):
        new = [j for j in orders[int(gid)] if j not in need]
        if batch and len(need) + len(new) > cap:
            flush()
            new = list(orders[int(gid)])
        batch.append(k)
        for j in new:
            need[int(j)] = 1
    flush()
    return sorted(bad)


def check_round(out_pool, own_ids: Sequence[int], lay, orders, weights, seed_base: int, mode: int,
                reference: Optional[dict] = None, agg: Optional[Callable] = None) -> dict:
    """Check every owned output row of one round (the module docstring).  reference: {"name":
    fixture name, "expected": {seg: {global id: [digest per range]}}, "ranges": {seg: [(a, b)]}}
    or None (K1 on regenerated operands).  Returns rows_checked, rows_differing, first_bad and
    the reference used."""
    if reference is not None:
        bad = check_against_digests(out_pool, own_ids, reference["expected"], reference["ranges"])
        ref = f"reference sha256 ({reference['name']})"
    else:
        bad = check_against_k1(out_pool, own_ids, lay, orders, weights, seed_base, mode, agg=agg)
        ref = "K1 on operands regenerated from their seeds"
    return dict(rows_checked=len(own_ids), rows_differing=len(bad), first_bad=bad[:8], reference=ref)
