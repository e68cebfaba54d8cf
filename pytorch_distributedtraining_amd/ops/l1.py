"""Fused L1 loss (``csrc/kernels/l1_loss.hip``): mean |a - b| and the gradient sign(a - b) / n from one read of a and
b, in the tensors' own dtype -- the feature-map terms of the reference's perceptual loss (models/losses.py,
Stoke-DDP.py:224), which autocast would otherwise run as fp32 copies, subtraction, abs, mean and a sign pass."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib

FUSED = os.environ.get("PDT_FUSED_L1", "1") != "0"     # 0: torch's l1_loss (A/B measurements)


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


class _L1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        lib = _lib.require()
        n = a.numel()
        g = torch.empty_like(a) if a.requires_grad else None
        out = torch.empty((), dtype=torch.float32, device=a.device)
        ws = torch.empty(lib.pdt_l1_partials(n), dtype=torch.float32, device=a.device)
        _lib.call("pdt_l1_fwd_grad", a.data_ptr(), b.data_ptr(), _lib.ptr(g), out.data_ptr(), ws.data_ptr(), n,
                  _lib.dtype_code(a.dtype), _lib.stream_handle(a.device))
        ctx.save_for_backward(g)
        return out

    @staticmethod
    def backward(ctx, go):
        (g,) = ctx.saved_tensors
        return g.mul_(go.to(g.dtype)), None       # g is this Function's own buffer, used once


def l1_loss(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """F.l1_loss(a, b) (mean) -- fused on the GPU for bf16 / fp32 operands of one dense layout; b takes no gradient."""
    if (FUSED and a.is_cuda and a.dtype in (torch.bfloat16, torch.float32) and b.dtype == a.dtype and a.shape == b.shape
            and a.stride() == b.stride() and _dense(a) and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and not b.requires_grad and a.numel() > 0):
        return _L1Fn.apply(a, b)
    return F.l1_loss(a, b)
