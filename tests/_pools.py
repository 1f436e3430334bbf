"""Device pools for the round-kernel parity tests.

The round entry points take the float4 body through the vector kernels only when every row is
16-B aligned with a stride that is a multiple of 4 elements (tal_agg_round_f32 / _bf16); a
contiguous [rows, n] copy of an odd-n host pool therefore runs entirely through the scalar
kernel.  `dev_rows(..., pad=True)` lays the rows out as ModelPool does (stride rounded up to 64
elements), so the vector kernel computes the body and the scalar kernel the n % 4 tail."""
import numpy as np
import torch


def dev_rows(pool: np.ndarray, dev, pad: bool = True) -> torch.Tensor:
    """[rows, ld] device copy of host rows (fp32, or bf16 given as uint16 / int16 bits)."""
    rows, n = pool.shape
    bits = pool.dtype in (np.uint16, np.int16)
    src = torch.from_numpy(np.ascontiguousarray(pool).view(np.int16)).view(torch.bfloat16) if bits else \
        torch.from_numpy(np.ascontiguousarray(pool))
    if not pad:
        return src.to(dev)
    ld = (n + 63) // 64 * 64
    t = torch.zeros((rows, ld), dtype=src.dtype, device=dev)
    t[:, :n] = src.to(dev)
    return t


def host(t: torch.Tensor, n: int) -> np.ndarray:
    """The first n columns back on the host (bf16 as uint16 bits)."""
    x = t[:, :n].cpu()
    return x.view(torch.int16).numpy().view(np.uint16) if x.dtype == torch.bfloat16 else x.numpy()
