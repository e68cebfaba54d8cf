"""Fused softmax cross-entropy over large vocabularies (gfx950 kernel, single streaming pass).

With ``inplace_backward=True`` (what the LM heads in ``models/`` pass, since their logits are dead
after the loss) the backward writes (softmax - onehot) * g IN PLACE over the saved logits, which
removes one [tokens, vocab] buffer (0.8 GB at GPT-2 1.3B / 8192 tokens per GPU).  The logits stay intact until
that backward runs.

``grad_in_forward=True`` (a separate opt-in, implies ``inplace_backward``; the LM heads pass it in training mode
only) goes one step further: where the row fits the registers of one workgroup (bf16, vocab <= 65,536: GPT-2)
and the logits require grad, the FORWARD already writes (softmax - onehot) / count over the logits in its single
read (``pdt_ce_fwd_grad``) and the backward only applies a non-unit upstream gradient: one read + one write of
the logits instead of two reads + one write.  **The logits tensor is clobbered by the forward** -- the returned
loss is correct, but any later read of the logits (or a loss taken without a backward) sees gradient values.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _lib


class _CEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, reduction, inplace_backward, grad_in_forward):
        V = logits.shape[-1]
        x2 = logits.reshape(-1, V)
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        t = target.reshape(-1).to(torch.int64).contiguous()
        rows = x2.shape[0]
        loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
        lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
        ctx.reduction, ctx.ignore_index, ctx.inplace = reduction, ignore_index, inplace_backward
        ctx.shape = logits.shape
        ctx.eager = False
        valid = (t != ignore_index).sum().clamp_min(1).float() if reduction != "none" else None
        if (grad_in_forward and reduction != "none" and FWD_GRAD and logits.requires_grad
                and x2.dtype == torch.bfloat16 and x2.data_ptr() == logits.data_ptr()):
            # gradient written over the logits now (the row is in registers); backward applies g only
            inv = (1.0 / valid).reshape(1) if reduction == "mean" else None
            rc = _lib.require().pdt_ce_fwd_grad(x2.data_ptr(), t.data_ptr(), loss.data_ptr(), lse.data_ptr(),
                                                _lib.ptr(inv), rows, V, x2.stride(0), _lib.dtype_code(x2.dtype),
                                                int(ignore_index), _lib.stream_handle(logits.device))
            if rc == 0:
                ctx.eager = True
            elif rc != -1:
                _lib.check(rc, "pdt_ce_fwd_grad")
        if not ctx.eager:
            _lib.call("pdt_ce_fwd", x2.data_ptr(), t.data_ptr(), loss.data_ptr(), lse.data_ptr(), rows, V,
                      x2.stride(0), _lib.dtype_code(x2.dtype), int(ignore_index), _lib.stream_handle(logits.device))
        ctx.save_for_backward(x2, t, lse)
        if reduction == "none":
            return loss.view(target.shape)
        ctx.valid = valid
        s = loss.sum()
        return s / valid if reduction == "mean" else s

    @staticmethod
    def backward(ctx, g):
        x2, t, lse = ctx.saved_tensors
        rows, V = x2.shape
        if ctx.eager:   # x2 already holds (softmax - onehot) [/ count]: scale by g on the device unless g == 1
            gs = g.float().reshape(1).contiguous()
            _lib.call("pdt_ce_scale", x2.data_ptr(), gs.data_ptr(), rows, V, x2.stride(0), _lib.dtype_code(x2.dtype),
                      _lib.stream_handle(x2.device))
            return x2.view(ctx.shape), None, None, None, None, None
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
        return grad.view(ctx.shape), None, None, None, None, None


# PDT_CE_FWD_GRAD=0: the two-pass forward / backward even where the fused one applies
FWD_GRAD = os.environ.get("PDT_CE_FWD_GRAD", "1") == "1"


def cross_entropy(logits, target, ignore_index: int = -100, reduction: str = "mean", inplace_backward: bool = False,
                  grad_in_forward: bool = False):
    if not logits.is_cuda or logits.dtype not in (torch.float32, torch.bfloat16):
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), target.reshape(-1),
                               ignore_index=ignore_index, reduction=reduction).reshape(
            target.shape if reduction == "none" else ())
    return _CEFn.apply(logits, target, ignore_index, reduction, inplace_backward or grad_in_forward, grad_in_forward)
