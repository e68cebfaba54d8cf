"""BatchNorm2d fused with the residual add and ReLU for channels-last bf16 activations (ResNet, BASELINE.json
config 2).  ``BatchNormAct2d`` subclasses nn.BatchNorm2d -- same parameters, buffers and
state_dict keys (torchvision checkpoints load) -- and adds ``act`` ('relu' or None) and an optional
``residual`` input, so a ResNet block's ``relu(bn3(conv3(h)) + identity)`` is ONE forward pass over HBM
instead of three (csrc/kernels/batchnorm.hip), and its backward two instead of four (after a residual add the
ReLU mask travels as 1 bit per element instead of re-reading the bf16 output).

Cross-rank statistics (SyncBatchNorm semantics, torch/nn/modules/_functions.py:36-200) when ``comm`` is set:
one all-reduce of 2C+1 doubles in forward and 2C doubles in backward (``parallel.syncbn.convert_sync_batchnorm``
sets it instead of swapping the module).  Anything the kernels do not cover (CPU, fp32 activations, NCHW,
C % 8 != 0, eval mode) runs the equivalent torch / SyncBN ops.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib


_WS: dict = {}


def _workspace(c, dev):
    """Per-(device, C) fp32 partial-sum workspace, reused by every layer of that width (stream-ordered)."""
    key = (dev, c)
    ws = _WS.get(key)
    if ws is None:
        ws = _WS[key] = torch.empty(_lib.require().pdt_bn_ws_floats(c), dtype=torch.float32, device=dev)
    return ws


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, eps, momentum, relu, comm):
        n, c, h, w = x.shape
        rows = n * h * w
        dev, stream = x.device, _lib.stream_handle(x.device)
        ws = _workspace(c, dev)
        stats = torch.empty(2 * c + 1, dtype=torch.float64, device=dev)
        coef = torch.empty(4, c, dtype=torch.float32, device=dev)        # mean, invstd, scale, shift
        if comm is not None and comm.world_size > 1:
            _lib.call("pdt_bn_stats", x.data_ptr(), rows, c, ws.data_ptr(), stats.data_ptr(), stream)
            comm.all_reduce(stats, "sum")
            _lib.call("pdt_bn_finalize", stats.data_ptr(), c, float(eps), float(momentum), _lib.ptr(weight),
                      _lib.ptr(bias), coef[0].data_ptr(), coef[1].data_ptr(), coef[2].data_ptr(), coef[3].data_ptr(),
                      _lib.ptr(running_mean), _lib.ptr(running_var), stream)
        else:       # local statistics: the combine and the finalize are one kernel
            _lib.call("pdt_bn_stats_finalize", x.data_ptr(), rows, c, ws.data_ptr(), stats.data_ptr(), float(eps),
                      float(momentum), _lib.ptr(weight), _lib.ptr(bias), coef[0].data_ptr(), coef[1].data_ptr(),
                      coef[2].data_ptr(), coef[3].data_ptr(), _lib.ptr(running_mean), _lib.ptr(running_var), stream)
        y = torch.empty_like(x, memory_format=torch.channels_last)
        # ReLU after a residual add: the backward's mask can not be recomputed from x, so the apply writes it as
        # bits (1/16 of the bytes of reading y back in both backward passes)
        mbits = torch.empty((rows, c // 8), dtype=torch.uint8, device=dev) if relu and res is not None else None
        _lib.call("pdt_bn_apply", x.data_ptr(), _lib.ptr(res), coef[2].data_ptr(), coef[3].data_ptr(), y.data_ptr(),
                  rows, c, 1 if relu else 0, _lib.ptr(mbits), stream)
        ctx.save_for_backward(x, mbits if mbits is not None else y, weight, coef, stats[2 * c:])
        ctx.relu, ctx.comm, ctx.has_res = relu, comm, res is not None
        ctx.has_w, ctx.has_b = weight is not None, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, coef, count = ctx.saved_tensors
        n, c, h, w = x.shape
        rows = n * h * w
        dev, stream = x.device, _lib.stream_handle(x.device)
        if not dy.is_contiguous(memory_format=torch.channels_last) or dy.dtype != x.dtype:
            dy = dy.contiguous(memory_format=torch.channels_last).to(x.dtype)
        ws = _workspace(c, dev)
        sums = torch.empty(2 * c, dtype=torch.float64, device=dev)
        # parameter gradients are LOCAL sums (the data-parallel engine reduces them like any gradient),
        # written in fp32 by the combine kernel
        pg = torch.empty(2, c, dtype=torch.float32, device=dev)
        gw = pg[0] if ctx.has_w and ctx.needs_input_grad[2] else None
        gb = pg[1] if ctx.has_b and ctx.needs_input_grad[3] else None
        # ReLU mask: recomputed from x with the forward's scale / shift when there is no residual (y is not
        # read: one bf16 stream less in both passes); from the forward's mask bits after a residual add (``y`` is
        # then that uint8 [rows, C / 8] tensor)
        mask = 0 if not ctx.relu else (3 if ctx.has_res else 2)
        _lib.call("pdt_bn_bwd_reduce", dy.data_ptr(), y.data_ptr(), x.data_ptr(), coef[0].data_ptr(),
                  coef[1].data_ptr(), coef[2].data_ptr(), rows, c, mask, ws.data_ptr(), sums.data_ptr(),
                  _lib.ptr(gw), _lib.ptr(gb), stream)
        if ctx.comm is not None and ctx.comm.world_size > 1:
            ctx.comm.all_reduce(sums, "sum")
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res else None
        _lib.call("pdt_bn_bwd_apply", dy.data_ptr(), y.data_ptr(), x.data_ptr(), coef[0].data_ptr(),
                  coef[1].data_ptr(), _lib.ptr(weight), coef[2].data_ptr(), sums.data_ptr(), count.data_ptr(),
                  dx.data_ptr(), _lib.ptr(dres), rows, c, mask, stream)
        return dx, dres, gw, gb, None, None, None, None, None, None


class BatchNormAct2d(nn.BatchNorm2d):
    """nn.BatchNorm2d (+ residual) (+ ReLU) with the fused channels-last kernels.

    forward(x, residual=None) = act(batch_norm(x) + residual)."""

    def __init__(self, num_features, act: str | None = None, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device=device, dtype=dtype)
        if act not in (None, "relu"):
            raise ValueError(f"unsupported activation {act}")
        self.act = act
        self.comm = None          # set by convert_sync_batchnorm -> cross-rank statistics

    def extra_repr(self):
        return super().extra_repr() + f", act={self.act}"

    def _fused_ok(self, x, residual) -> bool:
        if not (x.is_cuda and self.training and x.dim() == 4 and x.dtype == torch.bfloat16):
            return False
        if not x.is_contiguous(memory_format=torch.channels_last) or self.num_features % 8 or self.num_features > 2048:
            return False
        if self.affine and (self.weight.dtype != torch.float32 or self.bias.dtype != torch.float32):
            return False
        if self.track_running_stats and self.running_mean is not None and self.running_mean.dtype != torch.float32:
            return False
        if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype or
                                     not residual.is_contiguous(memory_format=torch.channels_last)):
            return False
        return True

    def forward(self, x, residual=None):
        momentum = self.momentum if self.momentum is not None else 0.0
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:
                momentum = 1.0 / float(self.num_batches_tracked)
        if self._fused_ok(x, residual):
            rm = self.running_mean if self.track_running_stats else None
            rv = self.running_var if self.track_running_stats else None
            return _BNActFn.apply(x, residual, self.weight, self.bias, rm, rv, self.eps, momentum,
                                  self.act == "relu", self.comm)
        y = self._bn_fallback(x, momentum)
        if residual is not None:
            y = y + residual
        return F.relu(y) if self.act == "relu" else y

    def _bn_fallback(self, x, momentum):
        use_batch = self.training or not self.track_running_stats
        if use_batch and self.comm is not None and self.comm.world_size > 1:
            from ..parallel.syncbn import _sync_bn_reference, _SyncBNFn
            rm = self.running_mean if self.track_running_stats else None
            rv = self.running_var if self.track_running_stats else None
            if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16):
                return _SyncBNFn.apply(x, self.weight, self.bias, rm, rv, self.eps, momentum, self.comm)
            return _sync_bn_reference(x, self.weight, self.bias, rm, rv, self.eps, momentum, self.comm, True)
        return F.batch_norm(x, self.running_mean if not self.training or self.track_running_stats else None,
                            self.running_var if not self.training or self.track_running_stats else None,
                            self.weight, self.bias, use_batch, momentum, self.eps)
