"""OCP fp8 (e4m3fn -- the gfx950 encoding, not MI300's fnuz) quantise / dequantise with per-tensor
scaling and a fused amax reduction (delayed-scaling recipe).  BASELINE.json north star: "bf16/fp8
loss-scaled cast"."""
from __future__ import annotations

import torch

from . import _lib

E4M3_MAX = 448.0


def quantize_fp8(x: torch.Tensor, scale: torch.Tensor, amax: torch.Tensor | None = None):
    """Return uint8 storage of fp8-e4m3fn(x * scale) (saturating); optionally max-accumulate |x| into
    ``amax`` (fp32 [1], reinterpreted as uint32 bits by the kernel, so it must start >= 0)."""
    x = x.contiguous()
    if not x.is_cuda:
        q = (x.float() * scale.float()).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
        if amax is not None:
            amax.copy_(torch.maximum(amax, x.abs().max().float().reshape(1)))
        return q.view(torch.uint8)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    _lib.call("pdt_fp8_quant", x.data_ptr(), q.data_ptr(), x.numel(), _lib.dtype_code(x.dtype), scale.data_ptr(),
              _lib.ptr(amax), _lib.stream_handle(x.device))
    return q


def dequantize_fp8(q: torch.Tensor, scale_inv: torch.Tensor, dtype=torch.bfloat16):
    if not q.is_cuda:
        return (q.view(torch.float8_e4m3fn).float() * scale_inv.float()).to(dtype)
    y = torch.empty(q.shape, dtype=dtype, device=q.device)
    _lib.call("pdt_fp8_dequant", q.data_ptr(), y.data_ptr(), q.numel(), _lib.dtype_code(dtype), scale_inv.data_ptr(),
              _lib.stream_handle(q.device))
    return y


def scale_from_amax(amax: torch.Tensor, margin: int = 0) -> torch.Tensor:
    """Delayed-scaling scale = E4M3_MAX / amax / 2^margin (1 where amax == 0)."""
    a = amax.float()
    s = torch.where(a > 0, E4M3_MAX / a / (2.0 ** margin), torch.ones_like(a))
    return s


# ---------------------------------------------------------------------------------------------------------------
# fp8 training linears (delayed scaling, HYBRID recipe: e4m3 activations / weights, e5m2 gradients)
# ---------------------------------------------------------------------------------------------------------------
#
# Every GEMM of an fp8 linear runs on gfx950's fp8 MFMA through hipBLASLt (torch._scaled_mm, per-tensor
# dequantisation scales, bf16 output):
#   forward          Y  = Xq  Wq^T                    A = Xq  [M, K] row-major,   B = Wq^T (view of [N, K])
#   data gradient    dX = dYq Wq                      A = dYq [M, N],             B = (WqT)^T (view of [K, N])
#   weight gradient  dW = dYq^T Xq                    A = dYqT [N, M],            B = (XqT)^T (view of [K, M])
# so each operand is needed in both layouts; csrc/kernels/fp8.hip writes both from ONE read of the bf16
# tensor (cast + transpose + amax in one pass).  The delayed-scaling bookkeeping (amax history roll, new
# scale) is one tiny kernel per module per pass, so the recipe never syncs the host.
# Scope: the scales are per rank (amax is not all-reduced across data-parallel ranks -- FSDP ranks see the
# same weights, hence the same weight scales; activation scales may differ per rank, as in TE's default).

E5M2_MAX = 57344.0
SLOT_X, SLOT_W, SLOT_DY = 0, 1, 2
_FMT_DTYPE = {0: torch.float8_e4m3fn, 1: torch.float8_e5m2}
_FMT_MAX = {0: E4M3_MAX, 1: E5M2_MAX}


class _Fp8State:
    enabled = False
    margin = 0
    history = 16


class fp8_autocast:
    """``with fp8_autocast():`` -- framework ``Linear`` layers inside run their three GEMMs in fp8 (see
    above).  Norms, attention, the LM head and the optimizer stay bf16 / fp32 (the usual fp8 recipe)."""

    def __init__(self, enabled: bool = True, margin: int = 0, amax_history_len: int = 16):
        self.enabled, self.margin, self.history = enabled, margin, amax_history_len

    def __enter__(self):
        self._prev = (_Fp8State.enabled, _Fp8State.margin, _Fp8State.history)
        _Fp8State.enabled, _Fp8State.margin, _Fp8State.history = self.enabled, self.margin, self.history
        return self

    def __exit__(self, *exc):
        _Fp8State.enabled, _Fp8State.margin, _Fp8State.history = self._prev
        return False


def fp8_enabled() -> bool:
    return _Fp8State.enabled


def fp8_recompute_safe(fn):
    """Wrap an activation-checkpointed function so its backward-time recomputation runs under the fp8 setting
    of the original forward (the recompute happens outside ``fp8_autocast``; without this it would take the
    bf16 path and save different tensors)."""
    state = (_Fp8State.enabled, _Fp8State.margin, _Fp8State.history)

    def run(*args, **kwargs):
        with fp8_autocast(state[0], state[1], state[2]):
            return fn(*args, **kwargs)
    return run


class Fp8Meta:
    """Delayed-scaling state of one linear: slots x / w / dy, amax history [3, H], the amax being
    accumulated this iteration (fp32 bits, max-reduced by the cast kernels), scale and 1 / scale."""

    def __init__(self, device, history: int | None = None, margin: int | None = None):
        H = history or _Fp8State.history
        self.H = H
        self.margin = _Fp8State.margin if margin is None else margin
        self.hist = torch.zeros(3, H, dtype=torch.float32, device=device)
        self.cur = torch.zeros(3, dtype=torch.float32, device=device)
        self.scale = torch.ones(3, dtype=torch.float32, device=device)
        self.scale_inv = torch.ones(3, dtype=torch.float32, device=device)
        self.fresh = [True, True, True]          # first use of a slot: scale from the tensor's own amax

    def update(self, s0: int, s1: int, fmt: int):
        fmax = _FMT_MAX[fmt]
        mul = 2.0 ** (-self.margin)
        if self.hist.is_cuda:
            _lib.call("pdt_fp8_update_scales", self.hist.data_ptr(), self.cur.data_ptr(), self.scale.data_ptr(),
                      self.scale_inv.data_ptr(), self.H, s0, s1, fmax, mul, _lib.stream_handle(self.hist.device))
            return
        h = self.hist[s0:s1]
        h.copy_(torch.cat([self.cur[s0:s1, None], h[:, :-1]], dim=1))
        self.cur[s0:s1] = 0
        m = h.amax(dim=1)
        ok = (m > 0) & torch.isfinite(m)
        new = torch.where(ok, fmax / torch.where(ok, m, torch.ones_like(m)) * mul, self.scale[s0:s1])
        self.scale[s0:s1] = new
        self.scale_inv[s0:s1] = 1.0 / new

    def prepare(self, slot_tensors, fmt: int):
        """Before casting the slots' tensors: refresh their scales.  A slot's first use measures the tensor's
        own amax first (one read-only pass) so iteration 0 is not cast with scale 1.  An entry may give a
        callable instead of a tensor: it runs that amax-only pass itself (fused GELU casts)."""
        s0, s1 = slot_tensors[0][0], slot_tensors[-1][0] + 1
        for slot, t in slot_tensors:
            if self.fresh[slot]:
                if callable(t):
                    t()
                else:
                    cast_transpose(t, self, slot, fmt, want_q=False, want_t=False)
                self.fresh[slot] = False
        self.update(s0, s1, fmt)


def _ct_ok(x: torch.Tensor) -> bool:
    R, C = x.shape
    return x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.is_contiguous() and R % 64 == 0 \
        and C % 64 == 0 and x.data_ptr() % 16 == 0


def cast_transpose(x: torch.Tensor, meta: Fp8Meta, slot: int, fmt: int, want_q: bool = True, want_t: bool = True):
    """fp8(x * scale[slot]) as [R, C] and / or its transpose [C, R]; max-accumulates |x| into meta.cur[slot].
    Returns (q or None, qt or None) as torch fp8 tensors."""
    R, C = x.shape
    dt = _FMT_DTYPE[fmt]
    if _ct_ok(x):
        q = torch.empty(R, C, dtype=dt, device=x.device) if want_q else None
        qt = torch.empty(C, R, dtype=dt, device=x.device) if want_t else None
        _lib.call("pdt_fp8_cast_transpose", x.data_ptr(), _lib.ptr(q), _lib.ptr(qt), R, C, _lib.dtype_code(x.dtype),
                  fmt, meta.scale[slot:slot + 1].data_ptr(), meta.cur[slot:slot + 1].data_ptr(),
                  _lib.stream_handle(x.device))
        return q, qt
    # reference path (CPU tests, shapes the tile kernel does not take)
    xf = x.float()
    meta.cur[slot:slot + 1].copy_(torch.maximum(meta.cur[slot:slot + 1], xf.abs().amax().reshape(1)))
    if not (want_q or want_t):
        return None, None
    fmax = _FMT_MAX[fmt]
    q = (xf * meta.scale[slot]).clamp(-fmax, fmax).to(dt)
    return (q if want_q else None), (q.t().contiguous() if want_t else None)


def fp8_mm(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor, bias=None,
           out_dtype=torch.bfloat16) -> torch.Tensor:
    """(a * sa) @ (b * sb) (+ bias) with a row-major [M, K] and b column-major [K, N] fp8 operands."""
    if a.is_cuda:
        return torch._scaled_mm(a, b, scale_a=sa, scale_b=sb, bias=bias, out_dtype=out_dtype)
    y = (a.float() * sa) @ (b.float() * sb)
    if bias is not None:
        y = y + bias.float()
    return y.to(out_dtype)


class _Fp8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, meta: Fp8Meta):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        need_dw, need_dx = weight.requires_grad, x.requires_grad
        meta.prepare([(SLOT_X, x2), (SLOT_W, weight)], 0)
        xq, xt = cast_transpose(x2, meta, SLOT_X, 0, want_q=True, want_t=need_dw)
        wq, wt = cast_transpose(weight, meta, SLOT_W, 0, want_q=True, want_t=need_dx)
        sinv = meta.scale_inv.clone()            # the scales these casts used, for the backward GEMMs
        y = fp8_mm(xq, wq.t(), sinv[0:1], sinv[1:2], bias, out_dtype=x.dtype)
        ctx.save_for_backward(xt, wt, sinv)
        ctx.meta, ctx.has_bias, ctx.xshape, ctx.wdtype = meta, bias is not None, x.shape, weight.dtype
        return y            # 2-D: callers reshape OUTSIDE the Function (in-place RoPE on a view of it is legal)

    @staticmethod
    def backward(ctx, dy):
        xt, wt, sinv = ctx.saved_tensors
        meta = ctx.meta
        N = dy.shape[-1]
        dy2 = dy.reshape(-1, N)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        meta.prepare([(SLOT_DY, dy2)], 1)
        dyq, dyt = cast_transpose(dy2, meta, SLOT_DY, 1, want_q=need_dx, want_t=need_dw)
        sdy = meta.scale_inv[SLOT_DY:SLOT_DY + 1]
        dx = dw = db = None
        if need_dx:
            dx = fp8_mm(dyq, wt.t(), sdy, sinv[1:2], out_dtype=dy.dtype).view(ctx.xshape)
        if need_dw:
            dw = fp8_mm(dyt, xt.t(), sdy, sinv[0:1], out_dtype=ctx.wdtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            from .activations import _colsum, colsum_ok
            db = _colsum(dy2, ctx.wdtype) if dy2.is_cuda and colsum_ok(N) else dy2.sum(0).to(ctx.wdtype)
        return dx, dw, db, None


def fp8_linear(x: torch.Tensor, weight: torch.Tensor, bias, meta: Fp8Meta) -> torch.Tensor:
    y = _Fp8LinearFn.apply(x.reshape(-1, x.shape[-1]), weight, bias, meta)
    return y.view(*x.shape[:-1], weight.shape[0])


# ---------------------------------------------------------------------------------------------------------------
# GPT-2 MLP in fp8 with the GELU fused into the casts: c_fc's output goes bias + GELU -> fp8 (row + transposed)
# in one pass (the bf16 hidden is never written), and backward's dH -> dA = dH * GELU'(A) -> e5m2 (row +
# transposed) + the c_fc bias gradient in one pass.  Against the per-Linear fp8 path this drops a write and a
# read of the [tokens, 4 d] hidden in each direction.
# ---------------------------------------------------------------------------------------------------------------

def _gelu_tanh(u):
    return 0.5 * u * (1.0 + torch.tanh(0.7978845608028654 * (u + 0.044715 * u * u * u)))


def _gelu_tanh_grad(u):
    t = torch.tanh(0.7978845608028654 * (u + 0.044715 * u * u * u))
    return 0.5 * (1 + t) + 0.5 * u * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * u * u)


def bias_gelu_cast_transpose(a, bias, meta: Fp8Meta, slot: int, fmt: int, want_q=True, want_t=True):
    """fp8(gelu_tanh(a + bias) * scale) as [R, C] / [C, R]; amax of the GELU output into meta.cur[slot]."""
    R, C = a.shape
    if _ct_ok(a) and a.dtype == torch.bfloat16 and bias.dtype == torch.bfloat16:
        dt = _FMT_DTYPE[fmt]
        q = torch.empty(R, C, dtype=dt, device=a.device) if want_q else None
        qt = torch.empty(C, R, dtype=dt, device=a.device) if want_t else None
        _lib.call("pdt_fp8_bias_gelu_ct", a.data_ptr(), bias.data_ptr(), _lib.ptr(q), _lib.ptr(qt), R, C, fmt,
                  meta.scale[slot:slot + 1].data_ptr(), meta.cur[slot:slot + 1].data_ptr(), _lib.stream_handle(a.device))
        return q, qt
    return cast_transpose(_gelu_tanh(a.float() + bias.float()), meta, slot, fmt, want_q, want_t)


def bias_gelu_bwd_cast_transpose(dh, a, bias, meta: Fp8Meta, slot: int, fmt: int, want_q=True, want_t=True,
                                 want_db=True):
    """dA = dh * gelu_tanh'(a + bias) cast to fp8 as [R, C] / [C, R] (amax into meta.cur[slot]) and, with
    ``want_db``, dbias = column sums of dA (bias dtype).  Returns (q, qt, dbias)."""
    R, C = a.shape
    if _ct_ok(a) and _ct_ok(dh) and a.dtype == torch.bfloat16 and dh.dtype == torch.bfloat16 \
            and bias.dtype == torch.bfloat16:
        dt = _FMT_DTYPE[fmt]
        q = torch.empty(R, C, dtype=dt, device=a.device) if want_q else None
        qt = torch.empty(C, R, dtype=dt, device=a.device) if want_t else None
        db = torch.empty(C, dtype=bias.dtype, device=a.device) if want_db else None
        ws = torch.empty(int(_lib.require().pdt_fp8_gelu_bwd_ws_floats(R, C)), dtype=torch.float32, device=a.device)
        _lib.call("pdt_fp8_bias_gelu_bwd_ct", dh.data_ptr(), a.data_ptr(), bias.data_ptr(), _lib.ptr(q), _lib.ptr(qt),
                  _lib.ptr(db), ws.data_ptr(), R, C, fmt, meta.scale[slot:slot + 1].data_ptr(),
                  meta.cur[slot:slot + 1].data_ptr(), _lib.stream_handle(a.device))
        return q, qt, db
    da = dh.float() * _gelu_tanh_grad(a.float() + bias.float())
    q, qt = cast_transpose(da, meta, slot, fmt, want_q, want_t)
    return q, qt, (da.sum(0).to(bias.dtype) if want_db else None)


def fp8_gelu_mlp_ok(x, w1, b1, w2, b2) -> bool:
    ts = (x, w1, b1, w2, b2)
    if any(t is None or t.dtype != torch.bfloat16 for t in ts):
        return False
    M = x.shape[:-1].numel()
    return all(d % 64 == 0 for d in (M, w1.shape[0], w1.shape[1], w2.shape[0])) and w1.is_contiguous() \
        and w2.is_contiguous()


class _Fp8GeluMlpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, m1: Fp8Meta, m2: Fp8Meta):
        K = x.shape[-1]
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        need_dx = x.requires_grad
        m1.prepare([(SLOT_X, x2), (SLOT_W, w1)], 0)
        xq, xt = cast_transpose(x2, m1, SLOT_X, 0, want_q=True, want_t=w1.requires_grad)
        wq1, wt1 = cast_transpose(w1, m1, SLOT_W, 0, want_q=True, want_t=need_dx)
        s1 = m1.scale_inv.clone()
        a = fp8_mm(xq, wq1.t(), s1[0:1], s1[1:2], out_dtype=x.dtype)
        m2.prepare([(SLOT_X, lambda: bias_gelu_cast_transpose(a, b1, m2, SLOT_X, 0, False, False)),
                    (SLOT_W, w2)], 0)
        hq, ht = bias_gelu_cast_transpose(a, b1, m2, SLOT_X, 0, want_q=True, want_t=w2.requires_grad)
        wq2, wt2 = cast_transpose(w2, m2, SLOT_W, 0, want_q=True, want_t=True)
        s2 = m2.scale_inv.clone()
        y = fp8_mm(hq, wq2.t(), s2[0:1], s2[1:2], b2, out_dtype=x.dtype)
        ctx.save_for_backward(xt, wt1, a, b1, ht, wt2, s1, s2)
        ctx.m1, ctx.m2, ctx.xshape = m1, m2, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        xt, wt1, a, b1, ht, wt2, s1, s2 = ctx.saved_tensors
        m1, m2 = ctx.m1, ctx.m2
        N2 = dy.shape[-1]
        dy2 = dy.reshape(-1, N2)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        m2.prepare([(SLOT_DY, dy2)], 1)
        dyq, dyt = cast_transpose(dy2, m2, SLOT_DY, 1, want_q=True, want_t=ctx.needs_input_grad[3])
        sdy = m2.scale_inv[SLOT_DY:SLOT_DY + 1]
        dh = fp8_mm(dyq, wt2.t(), sdy, s2[1:2], out_dtype=dy.dtype)
        dw2 = fp8_mm(dyt, ht.t(), sdy, s2[0:1], out_dtype=torch.bfloat16) if ctx.needs_input_grad[3] else None
        db2 = None
        if ctx.needs_input_grad[4]:
            from .activations import _colsum, colsum_ok
            db2 = _colsum(dy2, torch.bfloat16) if dy2.is_cuda and colsum_ok(N2) else dy2.sum(0).to(torch.bfloat16)
        need_dx, need_dw1 = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        m1.prepare([(SLOT_DY, lambda: bias_gelu_bwd_cast_transpose(dh, a, b1, m1, SLOT_DY, 1, False, False, False))],
                   1)
        daq, dat, db1 = bias_gelu_bwd_cast_transpose(dh, a, b1, m1, SLOT_DY, 1, want_q=need_dx, want_t=need_dw1,
                                                     want_db=ctx.needs_input_grad[2])
        sda = m1.scale_inv[SLOT_DY:SLOT_DY + 1]
        dx = fp8_mm(daq, wt1.t(), sda, s1[1:2], out_dtype=dy.dtype).view(ctx.xshape) if need_dx else None
        dw1 = fp8_mm(dat, xt.t(), sda, s1[0:1], out_dtype=torch.bfloat16) if need_dw1 else None
        return dx, dw1, db1, dw2, db2, None, None


def fp8_gelu_mlp(x, w1, b1, w2, b2, m1: Fp8Meta, m2: Fp8Meta):
    """GPT-2 MLP  gelu_tanh(x W1^T + b1) W2^T + b2  with fp8 GEMMs and the GELU fused into the casts."""
    y = _Fp8GeluMlpFn.apply(x.reshape(-1, x.shape[-1]), w1, b1, w2, b2, m1, m2)
    return y.view(*x.shape[:-1], w2.shape[0])
