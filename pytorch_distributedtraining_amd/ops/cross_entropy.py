"""Fused softmax cross-entropy over large vocabularies (gfx950 kernel, single streaming pass).

With ``inplace_backward=True`` (what the LM heads in ``models/`` pass, since their logits are dead
after the loss) the backward writes (softmax - onehot) * g IN PLACE over the saved logits, which
removes one [tokens, vocab] buffer (0.8 GB at GPT-2 1.3B / 8192 tokens per GPU).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, reduction, inplace_backward):
        V = logits.shape[-1]
        x2 = logits.reshape(-1, V)
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        t = target.reshape(-1).to(torch.int64).contiguous()
        rows = x2.shape[0]
        loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
        lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
        _lib.call("pdt_ce_fwd", x2.data_ptr(), t.data_ptr(), loss.data_ptr(), lse.data_ptr(), rows, V, x2.stride(0),
                  _lib.dtype_code(x2.dtype), int(ignore_index), _lib.stream_handle(logits.device))
        ctx.save_for_backward(x2, t, lse)
        ctx.reduction, ctx.ignore_index, ctx.inplace = reduction, ignore_index, inplace_backward
        ctx.shape = logits.shape
        if reduction == "none":
            return loss.view(target.shape)
        valid = (t != ignore_index).sum().clamp_min(1).float()
        ctx.valid = valid
        s = loss.sum()
        return s / valid if reduction == "mean" else s

    @staticmethod
    def backward(ctx, g):
        x2, t, lse = ctx.saved_tensors
        rows, V = x2.shape
        grad = x2 if ctx.inplace else torch.empty_like(x2)
        if ctx.reduction == "none":
            grow = g.reshape(-1).float().contiguous()
            gscale = None
        else:
            grow = None
            gscale = (g.float() / ctx.valid).reshape(1) if ctx.reduction == "mean" else g.float().reshape(1)
        _lib.call("pdt_ce_bwd", x2.data_ptr(), t.data_ptr(), lse.data_ptr(), _lib.ptr(grow), _lib.ptr(gscale),
                  grad.data_ptr(), rows, V, x2.stride(0), grad.stride(0), _lib.dtype_code(x2.dtype),
                  int(ctx.ignore_index), _lib.stream_handle(x2.device))
        return grad.view(ctx.shape), None, None, None, None


def cross_entropy(logits, target, ignore_index: int = -100, reduction: str = "mean", inplace_backward: bool = False):
    if not logits.is_cuda or logits.dtype not in (torch.float32, torch.bfloat16):
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), target.reshape(-1),
                               ignore_index=ignore_index, reduction=reduction).reshape(
            target.shape if reduction == "none" else ())
    return _CEFn.apply(logits, target, ignore_index, reduction, inplace_backward)
