"""3x3 / stride 1 / pad 1 convolution: an implicit-GEMM HIP kernel for narrow NHWC bf16 channels, else im2col (HIP
kernel) + one hipBLASLt GEMM per pass.

Narrow channels (<= 64, bf16, NHWC-contiguous; SwinIR-S's 60 -> 60 body convolutions): ``csrc/kernels/conv_igemm.hip``
forward and data gradient (the same kernel on dY with the flipped weight), picked per shape against the im2col path;
the weight gradient keeps the im2col + row-split GEMM below.  Otherwise:

For the small-channel convolutions of SwinIR-S (3->60, 60->60, 60->12 at 18 x 128 x 128)
MIOpen has no implicit-GEMM solver in bf16 and runs its naive direct kernels (the weight gradients alone
cost hundreds of ms per call, profiles/r1_v5_swinir_stoke_kernel_stats.csv).  Here every pass is one GEMM
on the matrix cores over an im2col matrix written by ``csrc/kernels/conv.hip`` (which reads any input
strides, so NCHW images and the NHWC-strided token views SwinIR produces need no layout copy):

    forward   y[P, Cout]  = cols(x)[P, Kp] @ Wm[Kp, Cout] + b
    backward  dW          = dY[P, Cout]^T @ cols(x)        (cols recomputed: 9x smaller saved state)
              dX          = cols(dY)[P, Kq] @ Wflip[Kq, Cin]  (3x3 conv of dY with the flipped weight)

The output is returned channels_last ([N, Cout, H, W] view of an NHWC buffer): SwinIR's
``flatten(2).transpose(1, 2)`` of it is then a free view.  ``Conv2d3x3`` subclasses nn.Conv2d, so
parameters / state_dict keys are unchanged.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .activations import _colsum, colsum_ok
from .linear import wgrad

_MAX_ELEMS = (1 << 31) - 1


def _round8(k: int) -> int:
    return (k + 7) // 8 * 8


def _im2col(x: torch.Tensor, kp: int) -> torch.Tensor:
    N, C, H, W = x.shape
    out = torch.empty((N * H * W, kp), dtype=x.dtype, device=x.device)
    sn, sc, sh, sw = x.stride()
    _lib.call("pdt_im2col3x3", x.data_ptr(), sn, sc, sh, sw, N, C, H, W, kp, out.data_ptr(),
              _lib.dtype_code(x.dtype), _lib.stream_handle(x.device))
    return out


def _w_rows(w: torch.Tensor, kp: int) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> [Kp, Cout], rows ordered (kh, kw, cin), zero rows past 9*Cin."""
    co, ci = w.shape[0], w.shape[1]
    m = w.permute(2, 3, 1, 0).reshape(9 * ci, co)
    return F.pad(m, (0, 0, 0, kp - 9 * ci)) if kp != 9 * ci else m.contiguous()


def _w_flip_rows(w: torch.Tensor, kq: int) -> torch.Tensor:
    """Data-gradient weight: rows (kh, kw, cout) of w[cout, cin, 2-kh, 2-kw] -> [Kq, Cin]."""
    co, ci = w.shape[0], w.shape[1]
    m = w.flip(2, 3).permute(2, 3, 0, 1).reshape(9 * co, ci)
    return F.pad(m, (0, 0, 0, kq - 9 * co)) if kq != 9 * co else m.contiguous()


def _nhwc_rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] -> [N*H*W, C] (a view when t is channels_last-contiguous)."""
    N, C, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(N * H * W, C)


# ---- implicit GEMM (csrc/kernels/conv_igemm.hip): narrow channels (<= 64), NHWC, bf16 -- no im2col matrix at all
IGEMM = os.environ.get("PDT_CONV_IGEMM", "auto")     # "auto": per shape, timed against im2col + GEMM; "0" / "1"
_IG_CHOICE: dict = {}


def _nhwc_contig(t: torch.Tensor) -> bool:
    return t.dim() == 4 and t.permute(0, 2, 3, 1).is_contiguous()


def _igemm_ok(t: torch.Tensor, ci: int, co: int) -> bool:
    N, _, H, W = t.shape
    return (IGEMM != "0" and t.is_cuda and t.dtype == torch.bfloat16 and _nhwc_contig(t) and t.data_ptr() % 8 == 0
            and bool(_lib.require().pdt_conv3x3_igemm_ok(N, H, W, ci, co)))


def _w_taps(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] -> [Cout, 9 taps x 64] bf16 (channels zero-padded to 64), the igemm kernel's weight."""
    co, ci = w.shape[0], w.shape[1]
    m = w.permute(0, 2, 3, 1)                                       # [co, kh, kw, ci]
    return F.pad(m, (0, 64 - ci)).reshape(co, 9 * 64).to(torch.bfloat16).contiguous()


def _w_taps_flip(w: torch.Tensor) -> torch.Tensor:
    """Data-gradient weight: w'[ci][kh][kw][co] = w[co][ci][2-kh][2-kw], channels (co) padded to 64."""
    co, ci = w.shape[0], w.shape[1]
    m = w.flip(2, 3).permute(1, 2, 3, 0)                            # [ci, kh, kw, co]
    return F.pad(m, (0, 64 - co)).reshape(ci, 9 * 64).to(torch.bfloat16).contiguous()


def _igemm(t: torch.Tensor, wk: torch.Tensor, bias, co: int, relu: bool = False) -> torch.Tensor:
    """3x3 conv of the NHWC-contiguous [N, C, H, W] ``t`` with the prepared tap weight -> channels_last output
    (``relu``: max(0, .) in the same store)."""
    N, C, H, W = t.shape
    y = torch.empty((N, H, W, co), dtype=torch.bfloat16, device=t.device)
    _lib.call("pdt_conv3x3_igemm_act", t.data_ptr(), wk.data_ptr(), _lib.ptr(bias), y.data_ptr(), N, H, W, C, co,
              int(relu), _lib.stream_handle(t.device))
    return y.permute(0, 3, 1, 2)


def _prefer_igemm(key, fa, fb) -> bool:
    if IGEMM == "1":
        return True
    c = _IG_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return True
        from .picks import timed_choice
        c = _IG_CHOICE[key] = timed_choice(fa, fb, table=_IG_CHOICE, key=key, name="conv_igemm")
    return c


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        N, C, H, W = x.shape
        co = weight.shape[0]
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        if _igemm_ok(x, C, co) and (bias is None or bias.dtype == torch.bfloat16):
            wk = _w_taps(weight)
            kp = _round8(9 * C)
            if _prefer_igemm(("fwd", tuple(x.shape), co, x.device), lambda: _igemm(x, wk, bias, co),
                             lambda: torch.addmm(bias, _im2col(x, kp), _w_rows(weight, kp)) if bias is not None
                             else _im2col(x, kp) @ _w_rows(weight, kp)):
                return _igemm(x, wk, bias, co)
        kp = _round8(9 * C)
        cols = _im2col(x, kp)
        wm = _w_rows(weight, kp)
        y = torch.addmm(bias, cols, wm) if bias is not None else cols @ wm
        return y.view(N, H, W, co).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        return _conv3x3_bwd(x, weight, ctx.has_bias, ctx.needs_input_grad, dy)


def _conv3x3_bwd(x, weight, has_bias, needs, dy):
    """(dx, dw, db) of a 3x3 / stride-1 / pad-1 conv (``needs``: which of x, weight, bias want a gradient)."""
    N, C, H, W = x.shape
    co = weight.shape[0]
    dym = _nhwc_rows(dy)
    if not dym.is_contiguous():
        dym = dym.contiguous()
    dx = dw = db = None
    if needs[1]:
        kp = _round8(9 * C)
        cols = _im2col(x, kp)
        # [Cout, (kh, kw, c)]: K = N*H*W rows (295k for SwinIR) -> the row-split batched weight-gradient
        # GEMM of ops.linear (one mm here ran at 27 TFLOP/s: 710 us per 60->60 conv, r1_v9 profile)
        g = wgrad(dym, cols, torch.float32)[:, :9 * C]
        dw = g.reshape(co, 3, 3, C).permute(0, 3, 1, 2).to(weight.dtype)
        del cols
    if has_bias and needs[2]:
        db = _colsum(dym, weight.dtype) if colsum_ok(co) and dym.is_contiguous() else \
            dym.float().sum(0).to(weight.dtype)
    if needs[0]:
        kq = _round8(9 * co)
        dyc = dym.view(N, H, W, co).permute(0, 3, 1, 2)         # NHWC-contiguous view of dY
        if _igemm_ok(dyc, co, C):
            wf = _w_taps_flip(weight)
            if _prefer_igemm(("dgrad", tuple(dy.shape), C, dy.device), lambda: _igemm(dyc, wf, None, C),
                             lambda: _im2col(dy, kq) @ _w_flip_rows(weight.to(dy.dtype), kq)):
                return _igemm(dyc, wf, None, C), dw, db
        dcols = _im2col(dy, kq)
        dxm = dcols @ _w_flip_rows(weight.to(dy.dtype), kq)    # [P, Cin]
        dx = dxm.view(N, H, W, C).permute(0, 3, 1, 2)
    return dx, dw, db


class _Conv3x3ReluFn(torch.autograd.Function):
    """relu(conv3x3(x)) with the ReLU in the implicit-GEMM conv's store; backward masks dY by y > 0 (one pass) and
    runs the conv's backward."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        y = _igemm(x, _w_taps(weight), bias, weight.shape[0], relu=True)
        ctx.save_for_backward(x, weight, y)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        return _conv3x3_bwd(x, weight, ctx.has_bias, ctx.needs_input_grad,
                            torch.ops.aten.threshold_backward(dy, y, 0))


def conv3x3_relu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """relu(conv3x3(x, weight, bias)): one implicit-GEMM pass where the kernel applies (bf16, NHWC, <= 64 channels)."""
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return conv3x3_relu(x.to(dt), weight.to(dt), None if bias is None else bias.to(dt))
    if (x.is_cuda and x.dim() == 4 and weight.dtype == x.dtype and _igemm_ok(x, x.shape[1], weight.shape[0])
            and (bias is None or bias.dtype == torch.bfloat16)):
        return _Conv3x3ReluFn.apply(x, weight, bias)
    return F.relu(conv3x3(x, weight, bias))


def conv3x3(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """3x3, stride 1, padding 1 convolution (bf16 / fp32).  Autocast-aware like F.conv2d."""
    if not x.is_cuda:
        return F.conv2d(x, weight, bias, 1, 1)
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return conv3x3(x.to(dt), weight.to(dt), None if bias is None else bias.to(dt))
    if x.dtype not in (torch.float32, torch.bfloat16) or weight.dtype != x.dtype:
        return F.conv2d(x, weight, bias, 1, 1)
    N, C, H, W = x.shape
    kp = max(_round8(9 * C), _round8(9 * weight.shape[0]))
    if N * H * W * kp > _MAX_ELEMS:           # keep the im2col matrix addressable: split the batch
        per = max(1, _MAX_ELEMS // (H * W * kp))
        return torch.cat([conv3x3(xs, weight, bias) for xs in x.split(per)], 0)
    _lib.require()
    return _Conv3x3Fn.apply(x, weight, bias)


class Conv2d3x3(nn.Conv2d):
    """nn.Conv2d(cin, cout, 3, 1, 1) running on im2col + hipBLASLt (same parameters / state_dict)."""

    def __init__(self, in_channels, out_channels, bias=True, device=None, dtype=None):
        super().__init__(in_channels, out_channels, 3, 1, 1, bias=bias, device=device, dtype=dtype)

    def forward(self, x):
        return conv3x3(x, self.weight, self.bias)


class _PixelShuffleAffineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, r, a, b):
        N, Crr, H, W = y.shape
        C = Crr // (r * r)
        out = torch.empty((N, H * r, W * r, C), dtype=y.dtype, device=y.device)   # channels_last
        bb = None if b is None else b.detach().reshape(-1).float().contiguous()
        _lib.call("pdt_pixel_shuffle_affine_fwd", y.data_ptr(), *y.stride(), N, C, H, W, r, float(a), _lib.ptr(bb),
                  out.data_ptr(), _lib.dtype_code(y.dtype), _lib.stream_handle(y.device))
        ctx.r, ctx.a, ctx.shape = r, float(a), (N, C, H, W)
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        N, C, H, W = ctx.shape
        r = ctx.r
        dy = torch.empty((N, H, W, C * r * r), dtype=dout.dtype, device=dout.device)
        _lib.call("pdt_pixel_shuffle_affine_bwd", dout.data_ptr(), *dout.stride(), N, C, H, W, r, ctx.a,
                  dy.data_ptr(), _lib.dtype_code(dout.dtype), _lib.stream_handle(dout.device))
        return dy.permute(0, 3, 1, 2), None, None, None


def pixel_shuffle_affine(y: torch.Tensor, r: int, a: float = 1.0, b: torch.Tensor | None = None) -> torch.Tensor:
    """``F.pixel_shuffle(y, r) * a + b[c]`` in one HIP pass (SwinIR's 'pixelshuffledirect'
    upsampler followed by the ``x / img_range + mean`` de-normalisation, Stoke-DDP.py:206-208).  ``y`` may be
    any-strided (the channels_last output of ``conv3x3``); the result is channels_last like torch's
    pixel_shuffle of a channels_last input, and the gradient is returned channels_last, the layout the
    convolution's backward GEMMs consume without a copy.  ``b`` is a constant (no gradient)."""
    if not y.is_cuda or y.dtype not in (torch.float32, torch.bfloat16):
        out = F.pixel_shuffle(y, r) * a
        return out if b is None else out + b.reshape(1, -1, 1, 1).to(out.dtype)
    _lib.require()
    return _PixelShuffleAffineFn.apply(y, r, a, b)


# ------------------------------------------------------------------------------------------------------------------
# 1x1 / stride-1 convolutions (ResNet bottlenecks) on channels_last storage ARE GEMMs: y[NHW, Co] = x[NHW, Ci] W^T,
# dX = dY W, dW = dY^T X.  MIOpen's 1x1 kernels win some forward shapes (56x56, C <= 256), hipBLASLt + the
# framework weight-gradient path win most backward ones (ResNet-50 at batch 256: up to 0.41 -> 0.32 ms per
# backward, profiles/r2_resnet50_conv1x1_miopen_vs_gemm.jsonl) -- so each direction of each shape is timed once
# (first uncaptured call) and the faster implementation kept.  PDT_CONV1X1=miopen / gemm forces one side.
# ------------------------------------------------------------------------------------------------------------------
import os as _os

_C1_MODE = _os.environ.get("PDT_CONV1X1", "auto")
_C1_CHOICE: dict = {}


def _c1_rows(t):
    N, C, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(N * H * W, C)


def _c1_from_rows(y2, N, H, W):
    return y2.view(N, H, W, y2.shape[1]).permute(0, 3, 1, 2)


def _c1_fwd_gemm(x, w):
    N, _, H, W = x.shape
    return _c1_from_rows(_c1_rows(x) @ w.view(w.shape[0], -1).t(), N, H, W)


def _c1_bwd_gemm(dy, x, w):
    N, _, H, W = x.shape
    dy2, x2 = _c1_rows(dy), _c1_rows(x)
    dx = _c1_from_rows(dy2 @ w.view(w.shape[0], -1), N, H, W)
    dw = wgrad(dy2, x2, w.dtype).view_as(w)
    return dx, dw


def _c1_bwd_miopen(dy, x, w):
    dx, dw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
                                                     (True, True, False))
    return dx, dw


def _c1_pick(key, gemm_fn, miopen_fn):
    if _C1_MODE != "auto":
        return _C1_MODE == "gemm"
    c = _C1_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return True
        from .picks import timed_choice
        c = _C1_CHOICE[key] = timed_choice(gemm_fn, miopen_fn, table=_C1_CHOICE, key=key, name="conv1x1")
    return c


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        key = ("f", tuple(x.shape), w.shape[0], x.device)
        if _c1_pick(key, lambda: _c1_fwd_gemm(x, w), lambda: F.conv2d(x, w)):
            y = _c1_fwd_gemm(x, w)
        else:
            y = F.conv2d(x, w)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        key = ("b", tuple(x.shape), w.shape[0], x.device)
        if _c1_pick(key, lambda: _c1_bwd_gemm(dy, x, w), lambda: _c1_bwd_miopen(dy, x, w)):
            dx, dw = _c1_bwd_gemm(dy, x, w)
        else:
            dx, dw = _c1_bwd_miopen(dy, x, w)
        return dx, dw


class _Conv1x1ForkFn(torch.autograd.Function):
    """(conv1x1(x), x) for a ResNet bottleneck without downsample: x feeds both conv1 and the identity branch,
    so autograd would sum two full-size input gradients in a separate add kernel (16 such adds were 1.3 ms of
    a 32 ms ResNet-50 step, profiles/r3_resnet50_kernel_breakdown.jsonl).  Returning the identity from the same
    Function hands both gradients to ONE backward, where the identity's is folded into the data-gradient GEMM
    as its C operand: dX = dIdt + dY W in one in-place hipBLASLt call (beta = 1) on dIdt's buffer."""

    @staticmethod
    def forward(ctx, x, w):
        key = ("f", tuple(x.shape), w.shape[0], x.device)
        if _c1_pick(key, lambda: _c1_fwd_gemm(x, w), lambda: F.conv2d(x, w)):
            y = _c1_fwd_gemm(x, w)
        else:
            y = F.conv2d(x, w)
        ctx.save_for_backward(x, w)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, didt):
        x, w = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        N, _, H, W = x.shape
        dy2, x2 = _c1_rows(dy), _c1_rows(x)
        w2 = w.view(w.shape[0], -1)
        if didt is None:
            dx2 = dy2 @ w2
        else:
            if not didt.is_contiguous(memory_format=torch.channels_last) or didt.dtype != dy.dtype:
                didt = didt.contiguous(memory_format=torch.channels_last).to(dy.dtype)
            # in place into the identity's gradient buffer (this backward is its only consumer): an
            # out-of-place addmm first copies C into a fresh output (a full DtoD pass per block)
            dx2 = _c1_rows(didt).addmm_(dy2, w2)
        dw = wgrad(dy2, x2, w.dtype).view_as(w)
        return _c1_from_rows(dx2, N, H, W), dw


def conv1x1_ok(x, w) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[0] * x.shape[2] * x.shape[3] >= 4096)


class Conv2d1x1(nn.Conv2d):
    """1x1 / stride-1 / bias-free nn.Conv2d (same parameters and state_dict) whose passes run on MIOpen or as
    GEMMs on the channels_last storage, whichever is measured faster per shape and direction."""

    def __init__(self, in_channels, out_channels, device=None, dtype=None):
        super().__init__(in_channels, out_channels, 1, stride=1, padding=0, bias=False, device=device, dtype=dtype)

    def forward(self, x):
        w = self.weight
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            x, w = x.to(dt), w.to(dt)
            if conv1x1_ok(x, w):
                with torch.autocast("cuda", enabled=False):
                    return _Conv1x1Fn.apply(x, w)
            return F.conv2d(x, w)
        if conv1x1_ok(x, w):
            return _Conv1x1Fn.apply(x, w)
        return F.conv2d(x, w)

    def forward_fork(self, x):
        """(self(x), identity x) with the identity's gradient accumulated inside this conv's data-gradient GEMM
        (``_Conv1x1ForkFn``); falls back to (self(x), x) where the GEMM form does not apply."""
        w = self.weight
        if x.is_cuda and x.dtype == torch.bfloat16 and torch.is_autocast_enabled("cuda") \
                and torch.get_autocast_dtype("cuda") == torch.bfloat16:
            w = w.to(torch.bfloat16)
            if conv1x1_ok(x, w):
                with torch.autocast("cuda", enabled=False):
                    return _Conv1x1ForkFn.apply(x, w)
        elif conv1x1_ok(x, w):
            return _Conv1x1ForkFn.apply(x, w)
        return self(x), x
