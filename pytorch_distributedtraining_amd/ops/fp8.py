"""OCP fp8 (e4m3fn -- the gfx950 encoding, not MI300's fnuz) quantise / dequantise with per-tensor
scaling and a fused amax reduction (delayed-scaling recipe).  BASELINE.json north star: "bf16/fp8
loss-scaled cast"."""
from __future__ import annotations

import torch

from . import _lib

E4M3_MAX = 448.0


def quantize_fp8(x: torch.Tensor, scale: torch.Tensor, amax: torch.Tensor | None = None):
    """Return uint8 storage of fp8-e4m3fn(x * scale) (saturating); optionally max-accumulate |x| into
    ``amax`` (fp32 [1], reinterpreted as uint32 bits by the kernel, so it must start >= 0)."""
    x = x.contiguous()
    if not x.is_cuda:
        q = (x.float() * scale.float()).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
        if amax is not None:
            amax.copy_(torch.maximum(amax, x.abs().max().float().reshape(1)))
        return q.view(torch.uint8)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _lib.call("pdt_fp8_quant", x.data_ptr(), q.data_ptr(), x.numel(), _lib.dtype_code(x.dtype), scale.data_ptr(),
              _lib.ptr(amax), _lib.stream_handle(x.device))
    return q


def dequantize_fp8(q: torch.Tensor, scale_inv: torch.Tensor, dtype=torch.bfloat16):
    if not q.is_cuda:
        return (q.view(torch.float8_e4m3fn).float() * scale_inv.float()).to(dtype)
    y = torch.empty(q.shape, dtype=dtype, device=q.device)
    _lib.call("pdt_fp8_dequant", q.data_ptr(), y.data_ptr(), q.numel(), _lib.dtype_code(dtype), scale_inv.data_ptr(),
              _lib.stream_handle(q.device))
    return y


def scale_from_amax(amax: torch.Tensor, margin: int = 0) -> torch.Tensor:
    """Delayed-scaling scale = E4M3_MAX / amax / 2^margin (1 where amax == 0)."""
    a = amax.float()
    s = torch.where(a > 0, E4M3_MAX / a / (2.0 ** margin), torch.ones_like(a))
    return s
