"""SyncBatchNorm over the framework's Comm (RCCL on MI355X, gloo on CPU) with gfx950 kernels.

Reference: DDPConfig(convert_to_sync_batch_norm=True) in Stoke-DDP.py:190-193 (SURVEY.md B3, K12,
collective C9).  Semantics follow torch/nn/modules/_functions.py:36-200:
  forward  -- batch statistics over ALL ranks' samples, running stats updated with the unbiased
              global variance, same parameter/buffer names as nn.BatchNorm2d;
  backward -- sum(dy), sum(dy*(x-mean)) all-reduced; weight/bias grads stay local (the DP engine
              reduces them like any other gradient).
MI355X design: every cross-rank exchange is ONE all-reduce of 2C+1 doubles (sums + count; fp64 so
the E[x^2]-E[x]^2 variance does not cancel), launched on RCCL's stream; the count stays on device so
ranks with different batch sizes need no host sync.  NCHW and channels_last (NHWC) layouts.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import _lib
from .comm import Comm, default_comm


def _layout(x):
    """-> (outer, C, inner) such that x is contiguous as [outer, C, inner]."""
    C = x.shape[1]
    if x.dim() == 2:
        return x.shape[0], C, 1, x.contiguous()
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        n, c, h, w = x.shape
        return n * h * w, C, 1, x
    x = x.contiguous()
    inner = 1
    for s in x.shape[2:]:
        inner *= s
    return x.shape[0], C, inner, x


def _ws(C, dev):
    return torch.empty(2 * C * 1024 + 64, dtype=torch.float32, device=dev)


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, comm):
        outer, C, inner, xc = _layout(x)
        dev = x.device
        stream = _lib.stream_handle(dev)
        stats = torch.empty(2 * C + 1, dtype=torch.float64, device=dev)
        _lib.call("pdt_syncbn_stats", xc.data_ptr(), outer, C, inner, _lib.dtype_code(x.dtype),
                  _ws(C, dev).data_ptr(), stats.data_ptr(), stream)
        stats[2 * C].fill_(float(outer * inner))
        comm.all_reduce(stats, "sum")
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        invstd = torch.empty(C, dtype=torch.float32, device=dev)
        rm = running_mean if running_mean is not None and running_mean.dtype == torch.float32 else None
        rv = running_var if rm is not None else None
        _lib.call("pdt_syncbn_finalize", stats.data_ptr(), C, float(eps), float(momentum), mean.data_ptr(),
                  invstd.data_ptr(), _lib.ptr(rm), _lib.ptr(rv), stream)
        if running_mean is not None and rm is None:  # non-fp32 running stats: update via torch
            cnt = stats[2 * C]
            var = (stats[C:2 * C] / cnt - (stats[:C] / cnt) ** 2).clamp_min(0)
            running_mean.mul_(1 - momentum).add_((stats[:C] / cnt).to(running_mean.dtype), alpha=momentum)
            running_var.mul_(1 - momentum).add_((var * cnt / (cnt - 1).clamp_min(1)).to(running_var.dtype),
                                                alpha=momentum)
        y = torch.empty_like(xc)
        wdt = _lib.dtype_code(weight.dtype) if weight is not None else _lib.F32
        _lib.call("pdt_syncbn_elemt", xc.data_ptr(), y.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                  _lib.ptr(weight), _lib.ptr(bias), outer, C, inner, _lib.dtype_code(x.dtype), wdt, stream)
        ctx.save_for_backward(xc, weight, mean, invstd, stats[2 * C:].clone())
        ctx.comm, ctx.layout = comm, (outer, C, inner)
        ctx.has_w, ctx.has_b = weight is not None, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, weight, mean, invstd, count = ctx.saved_tensors
        outer, C, inner = ctx.layout
        dev = xc.device
        stream = _lib.stream_handle(dev)
        dyc = dy.contiguous(memory_format=torch.channels_last) if (inner == 1 and xc.dim() == 4) else dy.contiguous()
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        _lib.call("pdt_syncbn_bwd_reduce", dyc.data_ptr(), xc.data_ptr(), mean.data_ptr(), outer, C, inner,
                  _lib.dtype_code(xc.dtype), _ws(C, dev).data_ptr(), sums.data_ptr(), stream)
        gw = (sums[C:] * invstd.double()).to(weight.dtype) if ctx.has_w else None
        gb = sums[:C].to(weight.dtype if ctx.has_w else torch.float32) if ctx.has_b else None
        ctx.comm.all_reduce(sums, "sum")
        dx = torch.empty_like(xc)
        wdt = _lib.dtype_code(weight.dtype) if weight is not None else _lib.F32
        _lib.call("pdt_syncbn_bwd_elemt", dyc.data_ptr(), xc.data_ptr(), dx.data_ptr(), mean.data_ptr(),
                  invstd.data_ptr(), _lib.ptr(weight), sums.data_ptr(), count.data_ptr(), outer, C, inner,
                  _lib.dtype_code(xc.dtype), wdt, stream)
        return dx, gw, gb, None, None, None, None, None


def _sync_bn_reference(x, weight, bias, running_mean, running_var, eps, momentum, comm, training):
    """CPU / non-kernel path with identical math (used by the gloo tests)."""
    C = x.shape[1]
    dims = [0] + list(range(2, x.dim()))
    if not training:
        return torch.nn.functional.batch_norm(x, running_mean, running_var, weight, bias, False, 0.0, eps)
    xf = x.float()
    local = torch.cat([xf.sum(dims).double(), (xf * xf).sum(dims).double(),
                       torch.tensor([x.numel() / C], dtype=torch.float64, device=x.device)])
    stats = local.clone()
    if comm.world_size > 1:
        stats = _AllReduceSum.apply(local, comm)
    cnt = stats[2 * C]
    mean = stats[:C] / cnt
    var = (stats[C:2 * C] / cnt - mean * mean).clamp_min(0)
    if running_mean is not None:
        with torch.no_grad():
            running_mean.mul_(1 - momentum).add_(mean.detach().to(running_mean.dtype), alpha=momentum)
            running_var.mul_(1 - momentum).add_((var.detach() * cnt / (cnt - 1).clamp_min(1)).to(running_var.dtype),
                                                alpha=momentum)
    shape = [1, C] + [1] * (x.dim() - 2)
    y = (xf - mean.float().view(shape)) * torch.rsqrt(var.float().view(shape) + eps)
    if weight is not None:
        y = y * weight.float().view(shape)
    if bias is not None:
        y = y + bias.float().view(shape)
    return y.to(x.dtype)


class _AllReduceSum(torch.autograd.Function):
    """all-reduce whose gradient is also all-reduced (so the stats path is differentiable)."""

    @staticmethod
    def forward(ctx, t, comm):
        ctx.comm = comm
        out = t.clone()
        comm.all_reduce(out, "sum")
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        ctx.comm.all_reduce(g, "sum")
        return g, None


class SyncBatchNorm(nn.modules.batchnorm._BatchNorm):
    """Drop-in for nn.BatchNorm{1,2,3}d / nn.SyncBatchNorm (same parameters and buffers)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, comm=None,
                 device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device=device, dtype=dtype)
        self.comm = comm

    def _check_input_dim(self, x):
        if x.dim() < 2:
            raise ValueError(f"expected at least 2D input (got {x.dim()}D)")

    def forward(self, x):
        self._check_input_dim(x)
        comm = self.comm or default_comm()
        momentum = self.momentum if self.momentum is not None else 0.0
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:
                momentum = 1.0 / float(self.num_batches_tracked)
        use_batch = self.training or not self.track_running_stats
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        if not use_batch:
            return torch.nn.functional.batch_norm(x, rm, rv, self.weight, self.bias, False, 0.0, self.eps)
        if (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and self.num_features % 8 == 0
                and self.num_features <= 2048 and x.is_contiguous(memory_format=torch.channels_last)
                and (not self.affine or self.weight.dtype == torch.float32)
                and (rm is None or rm.dtype == torch.float32)):
            # channels-last bf16: the fused BN kernels (ops/batchnorm.py) with cross-rank statistics
            from ..ops.batchnorm import _BNActFn
            return _BNActFn.apply(x, None, self.weight, self.bias, rm if self.training else None,
                                  rv if self.training else None, self.eps, momentum, False, comm)
        if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16):
            return _SyncBNFn.apply(x, self.weight, self.bias, rm if self.training else None,
                                   rv if self.training else None, self.eps, momentum, comm)
        return _sync_bn_reference(x, self.weight, self.bias, rm, rv, self.eps, momentum, comm, True)


def convert_sync_batchnorm(module: nn.Module, comm: Comm | None = None) -> nn.Module:
    """Recursively replace BatchNorm layers by SyncBatchNorm, keeping parameters and buffers
    (semantics of torch.nn.SyncBatchNorm.convert_sync_batchnorm, batchnorm.py:842)."""
    from ..ops.batchnorm import BatchNormAct2d
    out = module
    if isinstance(module, BatchNormAct2d):
        module.comm = comm if comm is not None else default_comm()   # fused kernels all-reduce their stats
        return module
    if isinstance(module, nn.modules.batchnorm._BatchNorm) and not isinstance(module, SyncBatchNorm):
        out = SyncBatchNorm(module.num_features, module.eps, module.momentum, module.affine,
                            module.track_running_stats, comm=comm)
        if module.affine:
            with torch.no_grad():
                out.weight = module.weight
                out.bias = module.bias
        out.running_mean = module.running_mean
        out.running_var = module.running_var
        out.num_batches_tracked = module.num_batches_tracked
        out.training = module.training
        out.to(next(module.parameters()).device if module.affine else module.running_mean.device)
    for name, child in module.named_children():
        out.add_module(name, convert_sync_batchnorm(child, comm))
    return out
