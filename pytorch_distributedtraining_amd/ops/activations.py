"""Fused bias + GELU (tanh or erf) and SwiGLU with gfx950 kernels (Llama MLP).

``bias_gelu(h, b)`` computes ``gelu(h + b)`` in one pass and saves only ``h`` for backward (the
pre-activation is recomputed in the backward kernel), so the MLP keeps one [tokens, 4d] activation
instead of two.  The backward kernel also accumulates the bias gradient (per-thread column partials +
a deterministic two-level column reduce), so ``dh`` is written once and never re-read.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


def colsum_ok(n: int) -> bool:
    """Widths the HIP column-sum kernel takes: N % 8 == 0, or N % 4 == 0 below 1024 columns."""
    return n % 8 == 0 or (n % 4 == 0 and n < 1024)


def _colsum(x2, out_dtype):
    rows, n = x2.shape
    lib = _lib.require()
    out = torch.empty(n, dtype=out_dtype, device=x2.device)
    ws = torch.empty(lib.pdt_colsum_ws_floats(rows, n), dtype=torch.float32, device=x2.device)
    _lib.call("pdt_colsum", x2.data_ptr(), rows, n, _lib.dtype_code(x2.dtype), out.data_ptr(),
              _lib.dtype_code(out_dtype), ws.data_ptr(), 0, _lib.stream_handle(x2.device))
    return out


class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, bias, tanh):
        shape = h.shape
        h2 = h.reshape(-1, shape[-1]).contiguous()
        y = torch.empty_like(h2)
        bdt = _lib.dtype_code(bias.dtype) if bias is not None else _lib.BF16
        _lib.call("pdt_bias_gelu_fwd", h2.data_ptr(), _lib.ptr(bias), y.data_ptr(), h2.shape[0], h2.shape[1],
                  _lib.dtype_code(h2.dtype), bdt, 1 if tanh else 0, _lib.stream_handle(h.device))
        ctx.save_for_backward(h2, bias)
        ctx.tanh = tanh
        ctx.has_bias = bias is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        h2, bias = ctx.saved_tensors
        dy2 = dy.reshape(h2.shape).contiguous()
        dh = torch.empty_like(h2)
        rows, n = h2.shape
        if ctx.has_bias:
            # GELU backward + bias gradient in one sweep (no second pass over dh)
            lib = _lib.require()
            db = torch.empty_like(bias)
            ws = torch.empty(lib.pdt_colsum_ws_floats(rows, n), dtype=torch.float32, device=h2.device)
            _lib.call("pdt_bias_gelu_bwd_db", dy2.data_ptr(), h2.data_ptr(), bias.data_ptr(), dh.data_ptr(),
                      db.data_ptr(), ws.data_ptr(), rows, n, _lib.dtype_code(h2.dtype), _lib.dtype_code(bias.dtype),
                      1 if ctx.tanh else 0, 0, _lib.stream_handle(h2.device))
            return dh.view(dy.shape), db, None
        _lib.call("pdt_bias_gelu_bwd", dy2.data_ptr(), h2.data_ptr(), None, dh.data_ptr(), rows, n,
                  _lib.dtype_code(h2.dtype), _lib.BF16, 1 if ctx.tanh else 0, _lib.stream_handle(h2.device))
        return dh.view(dy.shape), None, None


def bias_gelu(h, bias=None, approximate: str = "tanh"):
    """gelu(h + bias); approximate in {'tanh', 'none'} like torch.nn.functional.gelu."""
    tanh = approximate == "tanh"
    if not h.is_cuda or h.shape[-1] % 8 != 0 or h.dtype not in (torch.float32, torch.bfloat16):
        u = h if bias is None else h + bias.to(h.dtype)
        return F.gelu(u, approximate=approximate)
    return _BiasGeluFn.apply(h, bias, tanh)


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        shape = x.shape
        f = shape[-1] // 2
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y = torch.empty((x2.shape[0], f), dtype=x.dtype, device=x.device)
        _lib.call("pdt_swiglu_fwd", x2.data_ptr(), y.data_ptr(), x2.shape[0], f, _lib.dtype_code(x.dtype),
                  _lib.stream_handle(x.device))
        ctx.save_for_backward(x2)
        ctx.shape = shape
        return y.view(*shape[:-1], f)

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        f = x2.shape[1] // 2
        dy2 = dy.reshape(-1, f).contiguous()
        dx = torch.empty_like(x2)
        _lib.call("pdt_swiglu_bwd", dy2.data_ptr(), x2.data_ptr(), dx.data_ptr(), x2.shape[0], f,
                  _lib.dtype_code(x2.dtype), _lib.stream_handle(x2.device))
        return dx.view(ctx.shape)


def swiglu(x):
    """silu(x[..., :F]) * x[..., F:] for a fused gate/up projection of width 2F."""
    f = x.shape[-1] // 2
    if not x.is_cuda or f % 8 != 0 or x.dtype not in (torch.float32, torch.bfloat16):
        a, b = x[..., :f], x[..., f:]
        return F.silu(a) * b
    return _SwiGLUFn.apply(x)
