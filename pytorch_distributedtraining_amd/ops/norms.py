"""LayerNorm / RMSNorm with hand-written gfx950 forward and backward kernels.

Drop-in modules (`LayerNorm`, `RMSNorm`) keep torch's parameter names (``weight``, ``bias``) so
state_dicts stay interchangeable with ``torch.nn.LayerNorm`` checkpoints (north star: same
state_dict / checkpoint layout).  SURVEY.md K3 (LayerNorm sites in SwinIR / GPT-2) and K16
(RMSNorm for Llama-3).
"""
from __future__ import annotations

import numbers

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .attention import stash_bias_grad


def _norm_fwd(x2, w, b, eps, rms, res2=None, rb=None):
    rows, n = x2.shape
    y = torch.empty_like(x2)
    s = torch.empty_like(x2) if res2 is not None else None
    rstd = torch.empty(rows, dtype=torch.float32, device=x2.device)
    mean = None if rms else torch.empty(rows, dtype=torch.float32, device=x2.device)
    _lib.call("pdt_norm_fwd", x2.data_ptr(), _lib.ptr(res2), _lib.ptr(rb), _lib.ptr(s), w.data_ptr(), _lib.ptr(b),
              y.data_ptr(), _lib.ptr(mean), rstd.data_ptr(), rows, n, float(eps), _lib.dtype_code(x2.dtype),
              _lib.dtype_code(w.dtype), 1 if rms else 0, _lib.stream_handle(x2.device))
    return y, mean, rstd, s


def _norm_bwd(dy2, x2, w, mean, rstd, need_b, rms, dres2=None, need_ds=False):
    """(dx, dgamma, dbeta | None, colsum(dx) | None) -- the last is the gradient of a residual bias (rb)."""
    rows, n = x2.shape
    lib = _lib.require()
    dx = torch.empty_like(x2)
    dw = torch.empty_like(w)
    db = torch.empty_like(w) if need_b else None
    ds = torch.empty_like(w) if need_ds else None
    ws = torch.empty(lib.pdt_norm_bwd_workspace_floats(rows, n), dtype=torch.float32, device=x2.device)
    _lib.call("pdt_norm_bwd", dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), _lib.ptr(mean), rstd.data_ptr(),
              _lib.ptr(dres2), dx.data_ptr(), dw.data_ptr(), _lib.ptr(db), _lib.ptr(ds), ws.data_ptr(), rows, n,
              _lib.dtype_code(x2.dtype), _lib.dtype_code(w.dtype), 1 if rms else 0, 0, _lib.stream_handle(x2.device))
    return dx, dw, db, ds


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd, _ = _norm_fwd(x2, weight, bias, eps, rms=False)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.has_bias = bias is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1]).contiguous()
        dx, dw, db, _ = _norm_bwd(dy2, x2, w, mean, rstd, ctx.has_bias, rms=False)
        return dx.view(dy.shape), dw, db, None


class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, _, rstd, _ = _norm_fwd(x2, weight, None, eps, rms=True)
        ctx.save_for_backward(x2, weight, rstd)
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dy2 = dy.reshape(-1, x2.shape[-1]).contiguous()
        dx, dw, _, _ = _norm_bwd(dy2, x2, w, None, rstd, False, rms=True)
        return dx.view(dy.shape), dw, None


class _AddNormFn(torch.autograd.Function):
    """(y, s) = (norm(x + r + rb), x + r + rb) in one pass; backward folds the residual gradient ds into dx and,
    with a residual bias rb (the bias of the Linear that produced r), returns its gradient colsum(dx) from the
    same pass -- the Linear then runs bias-free and skips its own column sum over dY."""

    @staticmethod
    def forward(ctx, x, r, rb, weight, bias, eps, rms, r_colsum):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        r2 = r.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd, s = _norm_fwd(x2, weight, bias, eps, rms, res2=r2, rb=rb)
        ctx.save_for_backward(s, weight, mean, rstd)
        ctx.has_bias, ctx.rms, ctx.has_rb, ctx.r_colsum = bias is not None, rms, rb is not None, r_colsum
        return y.view(shape), s.view(shape)

    @staticmethod
    def backward(ctx, dy, ds):
        s, w, mean, rstd = ctx.saved_tensors
        n = s.shape[-1]
        if dy is None:
            dy = torch.zeros_like(s)
        dy2 = dy.reshape(-1, n).contiguous()
        ds2 = ds.reshape(-1, n).contiguous() if ds is not None else None
        need_rb = ctx.has_rb and ctx.needs_input_grad[2]
        stash = ctx.r_colsum and not need_rb and ctx.needs_input_grad[1]
        dx, dw, db, drb = _norm_bwd(dy2, s, w, mean, rstd, ctx.has_bias, ctx.rms, dres2=ds2,
                                    need_ds=need_rb or stash)
        if stash:   # r came from a biased Linear in another FSDP unit: its backward takes colsum(dx) from here
            stash_bias_grad(dx, drb)
            drb = None
        dx = dx.view(dy.shape)
        return dx, dx, drb, dw, db, None, None, None


class _NormPassFn(torch.autograd.Function):
    """(y, x) = (norm(x), x): the residual stream passes through so that its LATER use's gradient ds comes back
    here and is folded into dx by the same backward pass (no separate add over the stream); ``r_colsum``: x came
    from a biased Linear that added the residual itself (``ops.linear.linear_residual``) -- the backward sums dx
    per column in the same pass and stashes it as that Linear's bias gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, rms, r_colsum):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        x2 = x2 if x2.is_contiguous() else x2.contiguous()
        y, mean, rstd, _ = _norm_fwd(x2, weight, bias, eps, rms)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.has_bias, ctx.rms, ctx.r_colsum = bias is not None, rms, r_colsum
        return y.view(shape), x

    @staticmethod
    def backward(ctx, dy, ds):
        x2, w, mean, rstd = ctx.saved_tensors
        n = x2.shape[-1]
        shape = dy.shape if dy is not None else ds.shape
        dy2 = dy.reshape(-1, n).contiguous() if dy is not None else torch.zeros_like(x2)
        ds2 = ds.reshape(-1, n).contiguous() if ds is not None else None
        dx, dw, db, dcs = _norm_bwd(dy2, x2, w, mean, rstd, ctx.has_bias, ctx.rms, dres2=ds2, need_ds=ctx.r_colsum)
        if ctx.r_colsum:
            stash_bias_grad(dx, dcs)
        return dx.view(shape), dw, db, None, None, None


# ------------------------------------------------------------------------------------------------
# Swin blocks: the shifted-window permutation folded into the narrow-row LayerNorms (csrc/kernels/norms.hip WinMap).
# norm1 writes its output rows straight into window order (the qkv projection's input) and its backward reads dy
# from window order; norm2 reads the attention output from window order as its residual input and its backward
# writes that input's gradient back in window order.  The block then has no separate roll / partition / reverse
# pass in either direction.
# ------------------------------------------------------------------------------------------------
def window_norm_ok(x, H: int, W: int, ws: int, shift: int) -> bool:
    C = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 3 and x.shape[1] == H * W
            and C <= 64 and C % 4 == 0 and H % ws == 0 and W % ws == 0 and 0 <= shift < ws and _lib.available())


def _win_norm_fwd(x2, res2, w, b, eps, geom, mode):
    rows, n = x2.shape
    H, W, ws, shift = geom
    y = torch.empty_like(x2)
    s = torch.empty_like(x2) if res2 is not None else None
    rstd = torch.empty(rows, dtype=torch.float32, device=x2.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x2.device)
    _lib.call("pdt_norm_fwd_win", x2.data_ptr(), _lib.ptr(res2), _lib.ptr(s), w.data_ptr(), _lib.ptr(b), y.data_ptr(),
              mean.data_ptr(), rstd.data_ptr(), rows, n, float(eps), _lib.dtype_code(x2.dtype), _lib.dtype_code(w.dtype),
              0, H, W, ws, shift, mode, _lib.stream_handle(x2.device))
    return y, s, mean, rstd


def _win_norm_bwd(dy2, x2, w, mean, rstd, need_b, dres2, geom, mode):
    rows, n = x2.shape
    H, W, ws, shift = geom
    lib = _lib.require()
    dx = torch.empty_like(x2)
    dr = torch.empty_like(x2) if mode & 2 else None
    dw = torch.empty_like(w)
    db = torch.empty_like(w) if need_b else None
    wsp = torch.empty(lib.pdt_norm_bwd_workspace_floats(rows, n), dtype=torch.float32, device=x2.device)
    _lib.call("pdt_norm_bwd_win", dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
              _lib.ptr(dres2), dx.data_ptr(), dw.data_ptr(), _lib.ptr(db), wsp.data_ptr(), rows, n,
              _lib.dtype_code(x2.dtype), _lib.dtype_code(w.dtype), 0, H, W, ws, shift, mode, _lib.ptr(dr),
              _lib.stream_handle(x2.device))
    return dx, dr, dw, db


class _NormToWindowsFn(torch.autograd.Function):
    """(y_win, x): y_win = window_partition(roll(LayerNorm(x), -shift)) -- [B, H*W, C] in, [B*nW, ws*ws, C] out, one
    pass -- and x passed through (as _NormPassFn): the block's residual use of x hands its gradient back here and
    the backward kernel adds it to dx (no separate add over the stream per block)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, geom):
        B, L, C = x.shape
        x2 = x.reshape(-1, C).contiguous()
        y, _, mean, rstd = _win_norm_fwd(x2, None, weight, bias, eps, geom, 1)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.geom, ctx.has_bias, ctx.shape = geom, bias is not None, x.shape
        ws = geom[2]
        return y.view(-1, ws * ws, C), x

    @staticmethod
    def backward(ctx, dy, ds):
        x2, w, mean, rstd = ctx.saved_tensors
        n = x2.shape[1]
        dy2 = dy.reshape(-1, n).contiguous() if dy is not None else torch.zeros_like(x2)
        ds2 = ds.reshape(-1, n).contiguous() if ds is not None else None
        dx, _, dw, db = _win_norm_bwd(dy2, x2, w, mean, rstd, ctx.has_bias, ds2, ctx.geom, 1)
        return dx.view(ctx.shape), dw, db, None, None


class _AddNormFromWindowsFn(torch.autograd.Function):
    """(LayerNorm(s), s) with s = x + roll(window_reverse(a_win), +shift): the attention output joins the residual
    stream inside the norm's read; backward returns d(s) for x and the same values in window order for a_win."""

    @staticmethod
    def forward(ctx, x, a_win, weight, bias, eps, geom):
        B, L, C = x.shape
        x2 = x.reshape(-1, C).contiguous()
        a2 = a_win.reshape(-1, C).contiguous()
        y, s, mean, rstd = _win_norm_fwd(x2, a2, weight, bias, eps, geom, 2)
        ctx.save_for_backward(s, weight, mean, rstd)
        ctx.geom, ctx.has_bias, ctx.shape, ctx.wshape = geom, bias is not None, x.shape, a_win.shape
        return y.view(x.shape), s.view(x.shape)

    @staticmethod
    def backward(ctx, dy, ds):
        s, w, mean, rstd = ctx.saved_tensors
        n = s.shape[-1]
        dy2 = dy.reshape(-1, n).contiguous() if dy is not None else torch.zeros_like(s)
        ds2 = ds.reshape(-1, n).contiguous() if ds is not None else None
        dx, dr, dw, db = _win_norm_bwd(dy2, s, w, mean, rstd, ctx.has_bias, ds2, ctx.geom, 2)
        return dx.view(ctx.shape), dr.view(ctx.wshape), dw, db, None, None


def layer_norm_to_windows(x, weight, bias, eps, H, W, ws, shift):
    """(LayerNorm of [B, H*W, C] written in shifted-window order [B*nW, ws*ws, C], x) -- use the returned x for the
    residual so its gradient is folded into this norm's backward (see window_norm_ok)."""
    return _NormToWindowsFn.apply(x, weight, bias, eps, (H, W, ws, shift))


def add_layer_norm_from_windows(x, a_win, weight, bias, eps, H, W, ws, shift):
    """(LayerNorm(s), s), s = x + the window-ordered ``a_win`` put back in image order (see window_norm_ok)."""
    return _AddNormFromWindowsFn.apply(x, a_win, weight, bias, eps, (H, W, ws, shift))


def norm_pass(x, weight, bias=None, eps=1e-5, rms=False, r_colsum=False):
    """(norm(x), x) with the stream's later gradient folded into this norm's backward pass (``_NormPassFn``)."""
    if not x.is_cuda or x.dtype not in (torch.float32, torch.bfloat16):
        return (rms_norm(x, weight, eps) if rms else layer_norm(x, weight, bias, eps)), x
    return _NormPassFn.apply(x, weight, bias, eps, rms, bool(r_colsum))


def add_norm(x, r, weight, bias=None, eps=1e-5, rms=False, r_bias=None, r_colsum=False):
    """Fused residual add + LayerNorm/RMSNorm: returns (norm(x + r + r_bias), x + r + r_bias); ``r_bias``
    (optional, [N], the norm's parameter dtype) is the bias of the Linear that produced r.  ``r_colsum``: r came
    from a biased Linear whose bias cannot be passed here (another FSDP unit's parameter): the backward still
    sums its dx per column in the same pass and stashes it for that Linear (``ops.attention.take_bias_grad``)."""
    if (not x.is_cuda or x.dtype not in (torch.float32, torch.bfloat16) or r.dtype != x.dtype
            or (r_bias is not None and r_bias.dtype != weight.dtype)):
        s = x + r if r_bias is None else x + (r + r_bias.to(r.dtype))
        return (rms_norm(s, weight, eps) if rms else layer_norm(s, weight, bias, eps)), s
    return _AddNormFn.apply(x, r, r_bias, weight, bias, eps, rms, bool(r_colsum))


def _use_native(x):
    return x.is_cuda


def layer_norm(x, weight, bias=None, eps=1e-5):
    """LayerNorm over the last dim.  bf16/fp32 activations, bf16/fp32 affine params."""
    if not _use_native(x):
        y = F.layer_norm(x.float(), (x.shape[-1],), weight.float(), None if bias is None else bias.float(), eps)
        return y.to(x.dtype)
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return _LayerNormFn.apply(x, weight, bias, eps)


def rms_norm(x, weight, eps=1e-6):
    if not _use_native(x):
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * weight.float()
        return y.to(x.dtype)
    if x.dtype not in (torch.float32, torch.bfloat16):
        x = x.float()
    return _RMSNormFn.apply(x, weight, eps)


class LayerNorm(nn.Module):
    """Same parameters/state_dict as torch.nn.LayerNorm (last-dim only)."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, bias=True, device=None, dtype=None):
        super().__init__()
        if isinstance(normalized_shape, numbers.Integral):
            normalized_shape = (int(normalized_shape),)
        assert len(normalized_shape) == 1, "only last-dim LayerNorm is supported"
        self.normalized_shape = tuple(normalized_shape)
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(normalized_shape, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(normalized_shape, device=device, dtype=dtype)) if bias else None

    def forward(self, x):
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            # autocast would run layer_norm in fp32; we keep bf16 activations and fp32 statistics
            x = x.to(torch.get_autocast_dtype("cuda"))
            with torch.autocast("cuda", enabled=False):
                return layer_norm(x, self.weight, self.bias, self.eps)
        return layer_norm(x, self.weight, self.bias, self.eps)

    def forward_add(self, x, r, r_bias=None, r_colsum=False):
        """(LN(x + r + r_bias), x + r + r_bias) with one kernel pass (``add_norm``)."""
        return _ln_forward_add(self, x, r, rms=False, r_bias=r_bias, r_colsum=r_colsum)

    def forward_pass(self, x, r_colsum=False):
        """(LN(x), x) for a stream the producing GEMM already summed (``norm_pass``)."""
        return norm_pass(x, self.weight, getattr(self, "bias", None), self.eps, False, r_colsum)

    def extra_repr(self):
        return f"{self.normalized_shape}, eps={self.eps}"


def _ln_forward_add(mod, x, r, rms, r_bias=None, r_colsum=False):
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return add_norm(x.to(dt), r.to(dt), mod.weight, getattr(mod, "bias", None), mod.eps, rms, r_bias,
                            r_colsum)
    return add_norm(x, r, mod.weight, getattr(mod, "bias", None), mod.eps, rms, r_bias, r_colsum)


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-6, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, device=device, dtype=dtype))

    def forward(self, x):
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            x = x.to(torch.get_autocast_dtype("cuda"))
            with torch.autocast("cuda", enabled=False):
                return rms_norm(x, self.weight, self.eps)
        return rms_norm(x, self.weight, self.eps)

    def forward_add(self, x, r, r_bias=None, r_colsum=False):
        return _ln_forward_add(self, x, r, rms=True, r_bias=r_bias, r_colsum=r_colsum)

    def forward_pass(self, x, r_colsum=False):
        """(RMSNorm(x), x) for a stream the producing GEMM already summed (``norm_pass``)."""
        return norm_pass(x, self.weight, None, self.eps, True, r_colsum)
