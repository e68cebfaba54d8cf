"""Linear layer whose backward reduces the bias gradient with the framework's column-sum kernel
(2x the bandwidth of the generic reduction torch uses for ``grad_output.sum(0)``; GEMMs stay on
hipBLASLt).  ``Linear`` subclasses nn.Linear, so parameters / state_dict keys are unchanged."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .activations import _colsum


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy2, w).view(*dy.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = torch.mm(dy2.t(), x.reshape(-1, x.shape[-1]))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _colsum(dy2, w.dtype) if dy2.shape[1] % 8 == 0 else dy2.sum(0).to(w.dtype)
        return dx, dw, db


def linear(x, weight, bias=None):
    if (x.is_cuda and bias is not None and x.dtype == weight.dtype and x.dtype in (torch.bfloat16, torch.float32)
            and not torch.is_autocast_enabled("cuda")):
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class Linear(nn.Linear):
    def forward(self, x):
        return linear(x, self.weight, self.bias)
