"""Fused narrow MLP (fc1 -> exact GELU -> fc2) for SwinIR-S's C = 60 / hidden 120 blocks on the gfx950 MFMA kernel
``csrc/kernels/swin_mlp.hip`` (skinny GEMMs where fusion pays).  Forward keeps the hidden activation
in registers; backward recomputes it and produces dx, dW1, db1, dW2, db2 in one pass over the tokens (plus a
partial-sum reduction).  Only the MLP input is saved for backward (the [tokens, 120] hidden never touches HBM).

Reference counterpart: timm/SwinIR ``Mlp`` (fc1, nn.GELU, fc2) built by Stoke-DDP.py:206-208 (SwinIR-S x2).
"""
from __future__ import annotations

import os

import torch

from . import _lib

ENABLED = os.environ.get("PDT_SWIN_FUSED_MLP", "1") == "1"


def fused_mlp_ok(x: torch.Tensor, w1: torch.Tensor, b1, w2: torch.Tensor, b2) -> bool:
    if not (ENABLED and x.is_cuda and b1 is not None and b2 is not None):
        return False
    if any(t.dtype != torch.bfloat16 for t in (x, w1, b1, w2, b2)):
        return False
    H, C = w1.shape
    if x.shape[-1] != C or tuple(w2.shape) != (C, H) or not (w1.is_contiguous() and w2.is_contiguous()):
        return False
    return bool(_lib.require().pdt_swin_mlp_ok(C, H))


class _FusedMlpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, res):
        H, C = w1.shape
        x2 = x.reshape(-1, C)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        T = x2.shape[0]
        y = torch.empty(T, C, dtype=x.dtype, device=x.device)
        r2 = None
        if res is not None:
            r2 = res.reshape(-1, C)
            if not r2.is_contiguous():
                r2 = r2.contiguous()
        _lib.call("pdt_swin_mlp_fwd", x2.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                  _lib.ptr(r2), y.data_ptr(), T, C, H, _lib.stream_handle(x.device))
        ctx.save_for_backward(x2, w1, b1, w2)
        ctx.xshape = x.shape
        ctx.has_res = res is not None
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w1, b1, w2 = ctx.saved_tensors
        H, C = w1.shape
        T = x2.shape[0]
        dy2 = dy.reshape(-1, C)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        lib = _lib.require()
        nb = int(lib.pdt_swin_mlp_bwd_blocks(T))
        ws = torch.empty(int(lib.pdt_swin_mlp_ws_floats(nb)), dtype=torch.float32, device=dy.device)
        dx = torch.empty(T, C, dtype=dy.dtype, device=dy.device)
        dw1, db1 = torch.empty_like(w1), torch.empty_like(b1)
        dw2, db2 = torch.empty_like(w2), torch.empty(C, dtype=w2.dtype, device=w2.device)
        _lib.call("pdt_swin_mlp_bwd", x2.data_ptr(), dy2.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                  dx.data_ptr(), dw1.data_ptr(), db1.data_ptr(), dw2.data_ptr(), db2.data_ptr(),
                  _lib.dtype_code(w1.dtype), ws.data_ptr(), nb, T, C, H, _lib.stream_handle(dy.device))
        return dx.view(ctx.xshape), dw1, db1, dw2, db2, (dy if ctx.has_res else None)


def fused_mlp(x, w1, b1, w2, b2, residual=None):
    """[residual +] GELU(x W1^T + b1) W2^T + b2 (exact erf GELU) on the fused HIP kernel; callers check
    fused_mlp_ok (and that ``residual`` is a bf16 tensor of x's shape)."""
    return _FusedMlpFn.apply(x, w1, b1, w2, b2, residual)
