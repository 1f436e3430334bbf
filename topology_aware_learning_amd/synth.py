"""Deterministic synthetic state_dicts and model layouts.

The values come from a counter-based integer generator (splitmix64 of (seed, index)) turned
into fp32 by bit assembly, so the same (layout, seed) gives the same bytes on any machine —
the golden sha256 fixtures in tests/golden were produced from exactly these inputs by the
reference's own aggregation functions.

Layouts are lists of (name, shape, dtype) in state_dict order.  The CIFAR CNN / ResNet-18 /
ResNet-50 layouts match the reference's models (src/modules.py:18-54, src/models/resnet.py:122,130;
pinned by tests/golden/layouts.json); ViT-B/16 is not in the reference and follows the
torchvision vit_b_16 state_dict (BASELINE config 5).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Iterable, List, Sequence, Tuple

import numpy as np
import torch

Layout = List[Tuple[str, Tuple[int, ...], str]]  # dtype in {"float32", "bfloat16", "int64"}

_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)
_M3 = np.uint64(0x94D049BB133111EB)


def _splitmix(x: np.ndarray) -> np.ndarray:
    x = x + _M1
    x = (x ^ (x >> np.uint64(30))) * _M2
    x = (x ^ (x >> np.uint64(27))) * _M3
    return x ^ (x >> np.uint64(31))


def counter_bits(seed: int, start: int, n: int) -> np.ndarray:
    idx = np.arange(start, start + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _splitmix(idx ^ (np.uint64(seed & 0xFFFFFFFF) << np.uint64(40)))


def counter_f32(seed: int, start: int, n: int) -> np.ndarray:
    """fp32 values with random sign, exponent in [2^-6, 2^2) and full random mantissa."""
    u = counter_bits(seed, start, n)
    mant = (u & np.uint64(0x7FFFFF)).astype(np.uint32)
    expo = (np.uint64(121) + ((u >> np.uint64(23)) % np.uint64(8))).astype(np.uint32)
    sign = ((u >> np.uint64(31)) & np.uint64(1)).astype(np.uint32)
    bits = (sign << np.uint32(31)) | (expo << np.uint32(23)) | mant
    return bits.view(np.float32)


def counter_i64(seed: int, start: int, n: int, hi: int = 1_000_000) -> np.ndarray:
    return (counter_bits(seed, start, n) % np.uint64(hi)).astype(np.int64)


def layout_of(sd) -> Layout:
    out: Layout = []
    for k, v in sd.items():
        dt = str(v.dtype).replace("torch.", "")
        out.append((k, tuple(int(s) for s in v.shape), dt))
    return out


def numel(shape: Sequence[int]) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n


def as_bf16(layout: Layout) -> Layout:
    """The layout of `model.to(torch.bfloat16)`: fp32 entries become bf16, int64 buffers stay."""
    return [(n, s, "bfloat16" if d == "float32" else d) for n, s, d in layout]


def layout_counts(layout: Layout) -> Tuple[int, int]:
    nf = sum(numel(s) for _, s, d in layout if d == "float32")
    ni = sum(numel(s) for _, s, d in layout if d == "int64")
    return nf, ni


def synth_state_dict(layout: Layout, seed: int, entries=None) -> "OrderedDict[str, torch.Tensor]":
    """CPU tensors for `layout`; entry values depend only on (seed, position in the layout).
    `entries`: indices of the entries to make (default all) - a sub-state-dict with the values
    those entries have in the whole one."""
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    pos = 0
    keep = None if entries is None else set(int(e) for e in entries)
    for k, (name, shape, dt) in enumerate(layout):
        n = numel(shape)
        if keep is not None and k not in keep:
            pos += n
            continue
        if dt == "float32":
            a = counter_f32(seed, pos, n)
            if name.endswith("running_var"):
                a = np.abs(a) + np.float32(0.5)
        elif dt == "int64":
            a = counter_i64(seed, pos, n)
        elif dt == "bfloat16":
            sd[name] = torch.from_numpy(counter_f32(seed, pos, n).reshape(shape).copy()).to(torch.bfloat16)
            pos += n
            continue
        else:
            raise ValueError(f"unsupported dtype {dt} for {name}")
        sd[name] = torch.from_numpy(a.reshape(shape).copy())
        pos += n
    return sd


def _i64(u: int) -> int:
    """uint64 constant as the int64 with the same bits (torch has no wrapping uint64 ops)."""
    return u - (1 << 64) if u >= 1 << 63 else u


def _srl(x: "torch.Tensor", k: int) -> "torch.Tensor":
    """Logical right shift of int64 bit patterns."""
    return (x >> k) & ((1 << (64 - k)) - 1)


def counter_f32_torch(seed: int, start: int, n: int, device, out: "torch.Tensor" = None) -> "torch.Tensor":
    """counter_f32 computed on `device` (int64 arithmetic wraps like uint64): bitwise the host
    generator, for full-size test pools that would take minutes to generate with numpy."""
    x = torch.arange(start, start + n, dtype=torch.int64, device=device)
    x ^= _i64((seed & 0xFFFFFFFF) << 40 & 0xFFFFFFFFFFFFFFFF)
    x += _i64(int(_M1))
    x = (x ^ _srl(x, 30)) * _i64(int(_M2))
    x = (x ^ _srl(x, 27)) * _i64(int(_M3))
    x = x ^ _srl(x, 31)
    mant = x & 0x7FFFFF
    expo = 121 + (_srl(x, 23) & 7)
    sign = _srl(x, 31) & 1
    bits = (sign << 31) | (expo << 23) | mant
    bits = torch.where(bits >= 1 << 31, bits - (1 << 32), bits).to(torch.int32)
    if out is None:
        return bits.view(torch.float32)
    out.view(torch.int32).copy_(bits)
    return out


_ROWGEN: dict = {}


def _row_plan(layout: Layout, dtype: str, device):
    """How a `dtype` segment row maps onto the generator's positions (cached per layout, dtype
    and device): the total position count, the segment's contiguous position runs as
    (first position, first segment column, length), a device index of every segment column's
    position when there is more than one run, and the segment columns of float32 running_var
    entries (|v| + 0.5, as synth_state_dict makes them)."""
    key = (tuple(layout), dtype, str(device))
    hit = _ROWGEN.get(key)
    if hit is not None:
        return hit
    runs, rv, pos, off = [], [], 0, 0
    for name, shape, dt in layout:
        n = numel(shape)
        if dt == dtype and n:
            if runs and runs[-1][0] + runs[-1][2] == pos:
                runs[-1][2] += n
            else:
                runs.append([pos, off, n])
            if dtype == "float32" and name.endswith("running_var"):
                rv.append((off, n))
            off += n
        pos += n
    fidx = None
    if len(runs) > 1:
        lo = runs[0][0]  # positions relative to the first run's
        fidx = torch.cat([torch.arange(p0 - lo, p0 - lo + n, dtype=torch.int64) for p0, _, n in runs]).to(device)
    rvidx = torch.cat([torch.arange(a, a + n, dtype=torch.int64) for a, n in rv]).to(device) if rv else None
    hit = (pos, [tuple(r) for r in runs], fidx, rvidx, off)
    _ROWGEN[key] = hit
    return hit


_FILL_DT = {"float32": 0, "bfloat16": 1, "int64": 2}
_FILL_HI = 1_000_000  # counter_i64's default range


def fill_table(layout: Layout, seeds: Sequence[int], dtype: str = "float32") -> np.ndarray:
    """The int64 table of tal_fill_counter (include/tal_agg.h) for the `dtype` segment rows of
    synth_state_dict(layout, seed) for each seed: header, seeds, the segment's generator-position
    runs and (float32) its running_var column ranges."""
    runs, rv, pos, off = [], [], 0, 0
    for name, shape, dt in layout:
        k = numel(shape)
        if dt == dtype and k:
            if runs and runs[-1][0] + runs[-1][2] == pos:
                runs[-1][2] += k
            else:
                runs.append([pos, off, k])
            if dtype == "float32" and name.endswith("running_var"):
                if rv and rv[-1][0] + rv[-1][1] == off:
                    rv[-1][1] += k
                else:
                    rv.append([off, k])
            off += k
        pos += k
    head = [len(seeds), off, len(runs), len(rv), _FILL_HI, 0, 0, 0]
    seeds = [int(s) & 0xFFFFFFFF for s in seeds]
    return np.array(head + seeds + [v for r in runs for v in r] + [v for r in rv for v in r], dtype=np.int64)


def fill_rows_torch(seg: "torch.Tensor", layout: Layout, seeds: Sequence[int], dtype: str = "float32",
                    chunk: int = 1 << 25) -> None:
    """seg[r, :n] = the `dtype` entries of synth_state_dict(layout, seeds[r]) concatenated in
    state_dict order (a pool segment row), generated on seg's device.  float32, bfloat16 (the
    bf16 of the fp32 counter value, as synth_state_dict makes it) and int64 segments.

    On a GPU: one tal_fill_counter launch for all the rows (the library's generator kernel).
    Round 5's torch form (kept below for CPU tensors: the gloo tests) took ~20 element-wise
    launches per `chunk` per row - about 15,000 dispatches for 256 ViT-B/16 rows - and crashed
    the process under rocprofv3 --pmc, which serializes and samples every dispatch."""
    if seg.device.type == "cuda":
        if not len(seeds):
            return
        from . import ops  # the library; no CPU fallback on a GPU tensor

        ops.fill_counter(seg, fill_table(layout, seeds, dtype), _FILL_DT[dtype])
        return
    total, runs, fidx, rvidx, n = _row_plan(layout, dtype, seg.device)
    if dtype == "int64":  # a few counters per model: host values
        for r, seed in enumerate(seeds):
            for p0, c0, k in runs:
                seg[r, c0:c0 + k].copy_(torch.from_numpy(counter_i64(seed, p0, k)))
        return
    if not n:
        return
    lo = runs[0][0]
    hi = runs[-1][0] + runs[-1][2]
    full = torch.empty(hi - lo, dtype=torch.float32, device=seg.device)
    for r, seed in enumerate(seeds):
        for c0 in range(lo, hi, chunk):
            c1 = min(hi, c0 + chunk)
            counter_f32_torch(seed, c0, c1 - c0, seg.device, out=full[c0 - lo:c1 - lo])
        v = full if fidx is None else full.index_select(0, fidx)
        if rvidx is not None:  # (v may be `full` itself: regenerated for the next row anyway)
            v[rvidx] = v[rvidx].abs() + 0.5
        seg[r, :n].copy_(v)  # bfloat16: round to nearest even, as .to()


# ------------------------------------------------------------------------------------------
# layouts
# ------------------------------------------------------------------------------------------
def _bn(prefix: str, c: int) -> Layout:
    return [
        (f"{prefix}.weight", (c,), "float32"),
        (f"{prefix}.bias", (c,), "float32"),
        (f"{prefix}.running_mean", (c,), "float32"),
        (f"{prefix}.running_var", (c,), "float32"),
        (f"{prefix}.num_batches_tracked", (), "int64"),
    ]


def cifar_cnn_layout(num_classes: int = 10) -> Layout:
    """CifarModule (reference src/modules.py:18-54): conv stack in `network` Sequential."""
    convs = [(0, 3, 32), (2, 32, 64), (5, 64, 128), (7, 128, 128), (10, 128, 256), (12, 256, 256)]
    out: Layout = []
    for idx, cin, cout in convs:
        out.append((f"network.{idx}.weight", (cout, cin, 3, 3), "float32"))
        out.append((f"network.{idx}.bias", (cout,), "float32"))
    for idx, fin, fout in [(16, 4096, 1024), (18, 1024, 512), (20, 512, num_classes)]:
        out.append((f"network.{idx}.weight", (fout, fin), "float32"))
        out.append((f"network.{idx}.bias", (fout,), "float32"))
    return out


def resnet_layout(kind: str, num_classes: int = 10) -> Layout:
    """CIFAR ResNet-18 / ResNet-50 (reference src/models/resnet.py:122,130)."""
    if kind == "resnet18":
        blocks, expansion, bottleneck = [2, 2, 2, 2], 1, False
    elif kind == "resnet50":
        blocks, expansion, bottleneck = [3, 4, 6, 3], 4, True
    else:
        raise ValueError(kind)
    out: Layout = [("conv1.weight", (64, 3, 3, 3), "float32")] + _bn("bn1", 64)
    in_planes = 64
    for li, (planes, nb) in enumerate(zip([64, 128, 256, 512], blocks), start=1):
        for bi in range(nb):
            stride = 1 if (li == 1 or bi > 0) else 2
            p = f"layer{li}.{bi}"
            if bottleneck:
                out.append((f"{p}.conv1.weight", (planes, in_planes, 1, 1), "float32"))
                out += _bn(f"{p}.bn1", planes)
                out.append((f"{p}.conv2.weight", (planes, planes, 3, 3), "float32"))
                out += _bn(f"{p}.bn2", planes)
                out.append((f"{p}.conv3.weight", (planes * expansion, planes, 1, 1), "float32"))
                out += _bn(f"{p}.bn3", planes * expansion)
            else:
                out.append((f"{p}.conv1.weight", (planes, in_planes, 3, 3), "float32"))
                out += _bn(f"{p}.bn1", planes)
                out.append((f"{p}.conv2.weight", (planes, planes, 3, 3), "float32"))
                out += _bn(f"{p}.bn2", planes)
            if stride != 1 or in_planes != planes * expansion:
                out.append((f"{p}.shortcut.0.weight", (planes * expansion, in_planes, 1, 1), "float32"))
                out += _bn(f"{p}.shortcut.1", planes * expansion)
            in_planes = planes * expansion
    out.append(("linear.weight", (num_classes, 512 * expansion), "float32"))
    out.append(("linear.bias", (num_classes,), "float32"))
    return out


def vit_b16_layout(num_classes: int = 1000, image_size: int = 224) -> Layout:
    """torchvision vit_b_16 state_dict layout (BASELINE config 5; not in the reference)."""
    d, mlp, layers, patch = 768, 3072, 12, 16
    seq = (image_size // patch) ** 2 + 1
    out: Layout = [
        ("class_token", (1, 1, d), "float32"),
        ("conv_proj.weight", (d, 3, patch, patch), "float32"),
        ("conv_proj.bias", (d,), "float32"),
        ("encoder.pos_embedding", (1, seq, d), "float32"),
    ]
    for i in range(layers):
        p = f"encoder.layers.encoder_layer_{i}"
        out += [
            (f"{p}.ln_1.weight", (d,), "float32"),
            (f"{p}.ln_1.bias", (d,), "float32"),
            (f"{p}.self_attention.in_proj_weight", (3 * d, d), "float32"),
            (f"{p}.self_attention.in_proj_bias", (3 * d,), "float32"),
            (f"{p}.self_attention.out_proj.weight", (d, d), "float32"),
            (f"{p}.self_attention.out_proj.bias", (d,), "float32"),
            (f"{p}.ln_2.weight", (d,), "float32"),
            (f"{p}.ln_2.bias", (d,), "float32"),
            (f"{p}.mlp.0.weight", (mlp, d), "float32"),
            (f"{p}.mlp.0.bias", (mlp,), "float32"),
            (f"{p}.mlp.3.weight", (d, mlp), "float32"),
            (f"{p}.mlp.3.bias", (d,), "float32"),
        ]
    out += [
        ("encoder.ln.weight", (d,), "float32"),
        ("encoder.ln.bias", (d,), "float32"),
        ("heads.head.weight", (num_classes, d), "float32"),
        ("heads.head.bias", (num_classes,), "float32"),
    ]
    return out


LAYOUTS = {
    "cifar10": cifar_cnn_layout,
    "resnet18": lambda: resnet_layout("resnet18"),
    "resnet50": lambda: resnet_layout("resnet50"),
    "vit_b16": vit_b16_layout,
}


def get_layout(name: str) -> Layout:
    return LAYOUTS[name]()


def param_names(layout: Layout, buffers: Iterable[str] = ("running_mean", "running_var", "num_batches_tracked")) -> List[str]:
    """Entries that are nn.Parameters (named_parameters order = state_dict order minus buffers)."""
    bufs = tuple(buffers)
    return [n for n, _, _ in layout if not n.endswith(bufs)]


def truncate_layout(layout: Layout, max_float: int) -> Layout:
    """The layout's leading float entries up to `max_float` elements in all (the entry that
    crosses the budget is cut to a flat remainder), every int64 entry kept: a reduced model of
    the same segment structure for multi-rank rehearsals (bench.py --max-params)."""
    out: Layout = []
    left = int(max_float)
    for name, shape, dt in layout:
        if dt == "int64":
            out.append((name, shape, dt))
            continue
        if left <= 0:
            continue
        n = numel(shape)
        out.append((name, shape, dt) if n <= left else (name, (left,), dt))
        left -= min(n, left)
    return out
