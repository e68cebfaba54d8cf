"""Max pooling over channels-last bf16 activations (the ResNet stem's 3x3 / stride-2 / pad-1 pool, BASELINE.json
config 2) on ``csrc/kernels/pool.hip``: the forward keeps one byte per output element naming the winning window
slot instead of torch's int64 argmax (8x smaller), the backward gathers dy per input pixel (deterministic, no
atomics).  ``MaxPool2d`` subclasses nn.MaxPool2d (no parameters, same module tree); anything the kernel does not
cover (CPU, other dtypes / layouts, dilation, ceil_mode, return_indices, C % 8) runs torch's own op.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, C, H, W = x.shape
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        slot = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        _lib.call("pdt_maxpool_fwd", x.data_ptr(), y.data_ptr(), slot.data_ptr(), N, C, H, W, OH, OW, k, s, p,
                  _lib.stream_handle(x.device))
        ctx.save_for_backward(slot)
        ctx.geom = (N, C, H, W, OH, OW, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (slot,) = ctx.saved_tensors
        N, C, H, W, OH, OW, k, s, p = ctx.geom
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _lib.call("pdt_maxpool_bwd", dy.data_ptr(), slot.data_ptr(), dx.data_ptr(), N, C, H, W, OH, OW, k, s, p,
                  _lib.stream_handle(dy.device))
        return dx, None, None, None


def maxpool_ok(x, k, s, p, dilation=1, ceil_mode=False, return_indices=False) -> bool:
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    if dilation != 1 or ceil_mode or return_indices:
        return False
    return bool(_lib.require().pdt_maxpool_ok(x.shape[1], k, s, p))


def max_pool2d(x, kernel_size, stride=None, padding=0):
    """F.max_pool2d for square windows; the HIP kernels on channels-last bf16 CUDA tensors."""
    k, s, p = kernel_size, stride if stride is not None else kernel_size, padding
    if maxpool_ok(x, k, s, p):
        return _MaxPoolFn.apply(x, k, s, p)
    return F.max_pool2d(x, k, s, p)


class MaxPool2d(nn.MaxPool2d):
    """nn.MaxPool2d on the channels-last HIP kernels where they apply (square kernel / stride / padding)."""

    def forward(self, x):
        k, s, p, d = _pair(self.kernel_size), _pair(self.stride), _pair(self.padding), _pair(self.dilation)
        if k[0] == k[1] and s[0] == s[1] and p[0] == p[1] and d == (1, 1) and \
                maxpool_ok(x, k[0], s[0], p[0], 1, self.ceil_mode, self.return_indices):
            return _MaxPoolFn.apply(x, k[0], s[0], p[0])
        return super().forward(x)
