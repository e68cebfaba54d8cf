"""Linear layer with an MI355X-shaped backward:

* large bf16 weight gradients dW = dY^T X run on the hand MFMA GEMM ``csrc/kernels/gemm.hip`` (TT layout:
  both operands token-major, read transposed from LDS; 1.26-1.36 PFLOP/s on the GPT-2 1.3B shapes against
  hipBLASLt's 1.0-1.22, profiles/r3_gemm_variants.txt) where it is measured faster than hipBLASLt for the
  shape (timed once per shape); ``PDT_WGRAD_HIP=0/1`` forces hipBLASLt / the hand kernel;

* the bias gradient is reduced with the framework's column-sum kernel (2x the bandwidth of the generic
  reduction torch uses for ``grad_output.sum(0)``);
* SMALL weight gradients (GPT-2 124M: N x K <= 2.5M outputs) are split 4-8 ways over the tokens into one
  batched GEMM with fp32 output (1.4-2x, see ``_split_k``);
* TALL-SKINNY weight gradients -- dW = dY^T X with hundreds of thousands of rows but only tens to
  hundreds of columns (SwinIR-S: 294,912 tokens x C = 60..180) -- are split over the row dimension into
  a batched GEMM with fp32 output and summed: one [N x M] x [M x K] GEMM with M = 295k leaves a single
  64x64 tile per CU walking the whole K loop (8 TFLOP/s measured, profiles/r1_v5_swinir_*), while
  ~72 batches of 4096 rows fill the chip;
* autocast-aware (bf16 compute with fp32 master weights) without leaving the fused path.

``Linear`` subclasses nn.Linear, so parameters / state_dict keys are unchanged.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .activations import _colsum, colsum_ok
from .attention import stash_dx_colsum, take_bias_grad
from .blaslt import prefer_bgradb, wgrad_bgrad
from .fp8 import Fp8Meta, fp8_enabled, fp8_linear
from .gemm import gemm_tt, tt_ok, tt_splits
from .grad_slots import claim, is_sharded_param
from .narrow import narrow_linear, narrow_ok, narrow_wgrad, narrow_wgrad_ok
from .picks import timed_choice

_WGRAD_CHUNK = 4096
# PDT_DX_COLSUM_STASH=0: the attention backward sums dO itself instead of taking the consuming Linear's db W
_DX_STASH = os.environ.get("PDT_DX_COLSUM_STASH", "1") == "1"


# PDT_NT_HIP: "auto" (default: per shape, the hand NT GEMM where it timed >= 1 % faster than hipBLASLt on the shape's
# first uncaptured call -- since round 4 they trade places by shape and box: the 3-stage program wins the long-K /
# narrow products, hipBLASLt the attention projection), "1" (always where it applies), "0" (never)
HIP_NT = os.environ.get("PDT_NT_HIP", "auto")
_NT_CHOICE: dict = {}


def _nt_hip_ok(a2: torch.Tensor, w: torch.Tensor, bias) -> bool:
    from . import gemm as G
    # (G.nt_ok also requires 16-byte aligned operand pointers)
    return (HIP_NT != "0" and G.KERNEL["name"] == "asm" and a2.is_cuda and a2.dim() == 2 and a2.shape[0] >= 4096
            and a2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
            and (bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous() and bias.data_ptr() % 16 == 0))
            and G.nt_ok(a2, w) and a2.shape[1] // 64 >= 2 and w.shape[0] % 8 == 0)


# PDT_NT_LT: "auto" -- the library side of nt_matmul's choice is the faster of torch's hipBLASLt call (its
# heuristic's first algorithm) and ops.blaslt's tuned plan (16 heuristic candidates timed once per shape); "0"
# (default): torch's call only -- on the flagship the tuned plans tied torch's pick (150.3 / 150.2k vs 150.7 /
# 149.9k tokens/s interleaved, profiles/r5/r5e_nt_lt_ab.log)
LT_NT = os.environ.get("PDT_NT_LT", "0")
_LT_CHOICE: dict = {}


def _lt_linear(a2, w, bias):
    """a2 [M, K] @ w[N, K]^T (+ bias) on the tuned hipBLASLt plan, or None (no algorithm for the combination).
    Column-major: D[N, M] = W^T(op T on col-major [K, N]) . A(col-major [K, M])."""
    from . import blaslt as LT
    m, k = a2.shape
    n = w.shape[0]
    y = torch.empty(m, n, dtype=a2.dtype, device=a2.device)
    if not LT.lt_matmul(LT.EPI_BIAS if bias is not None else LT.EPI_NONE, 1, n, m, k, w, a2, y, bias):
        return None
    return y


def _library_linear(a2, w, bias, key):
    """hipBLASLt for a2 @ w^T (+ bias): torch's call, or the tuned plan where it was measured faster."""
    if LT_NT != "0" and a2.is_cuda and a2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 \
            and a2.is_contiguous() and w.is_contiguous() and (bias is None or bias.dtype == torch.bfloat16):
        c = _LT_CHOICE.get(key)
        if c is None and not torch.cuda.is_current_stream_capturing():
            c = _LT_CHOICE[key] = _lt_linear(a2, w, bias) is not None and \
                timed_choice(lambda: _lt_linear(a2, w, bias), lambda: F.linear(a2, w, bias), 0.99,
                             table=_LT_CHOICE, key=key, name="lt")
        if c:
            y = _lt_linear(a2, w, bias)
            if y is not None:
                return y
    return F.linear(a2, w, bias)


def nt_matmul(a2: torch.Tensor, w: torch.Tensor, bias=None) -> torch.Tensor:
    """a2 [M, K] @ w[N, K]^T (+ bias): the hand NT GEMM (ops.gemm.gemm_nt) or hipBLASLt, per shape as timed."""
    key = (tuple(a2.shape), tuple(w.shape), bias is not None, a2.device)
    if _nt_hip_ok(a2, w, bias):
        from . import gemm as G
        if HIP_NT == "1":
            return G.gemm_nt(a2, w, bias)
        c = _NT_CHOICE.get(key)
        if c is None and not torch.cuda.is_current_stream_capturing():
            c = _NT_CHOICE[key] = timed_choice(lambda: G.gemm_nt(a2, w, bias),
                                               lambda: _library_linear(a2, w, bias, key), 0.99,
                                               table=_NT_CHOICE, key=key, name="nt")
        if c:
            return G.gemm_nt(a2, w, bias)
    return _library_linear(a2, w, bias, key)


# PDT_NARROW: "auto" (default: per shape, the narrow HIP kernel where it timed faster than the library path),
# "1" (always where it applies), "0" (never)
NARROW = os.environ.get("PDT_NARROW", "auto")
_NARROW_CHOICE: dict = {}


def _prefer_narrow(x2: torch.Tensor, w: torch.Tensor, bias, role: str) -> bool:
    """The narrow-GEMM kernel (ops.narrow) for a forward x W^T + b ("fwd") or a data gradient dY W ("dgrad") of a
    narrow Linear, where it is measured faster than the library GEMM on the shape's first uncaptured call."""
    if NARROW == "0":
        return False
    # dgrad: dY [M, N] . W [N, K] -- the kernel's B operand is W^T [K, N]
    if not narrow_ok(x2, w, bias, transposed=role != "fwd"):
        return False
    if NARROW == "1":
        return True
    key = (role, tuple(x2.shape), tuple(w.shape), bias is not None, x2.device)
    c = _NARROW_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return True
        if role == "fwd":
            fa = lambda: narrow_linear(x2, w, bias)                                  # noqa: E731
            fb = lambda: F.linear(x2, w, bias)                                       # noqa: E731
        else:
            fa = lambda: narrow_linear(x2, w.t().contiguous(), None, w.dtype)        # noqa: E731
            fb = lambda: (torch.mm(x2, w), _colsum(x2, w.dtype) if colsum_ok(x2.shape[1]) else None)  # noqa: E731
        c = _NARROW_CHOICE[key] = timed_choice(fa, fb, table=_NARROW_CHOICE, key=key, name="narrow")
    return c


def _prefer_narrow_wgrad(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype) -> bool:
    """The narrow weight-gradient kernel (ops.narrow) for tall-skinny dW with both feature counts <= 192, where it
    is measured faster than the row-split library GEMM (PDT_NARROW as for the forward)."""
    if NARROW == "0" or not narrow_wgrad_ok(dy2, x2, out_dtype):
        return False
    if NARROW == "1":
        return True
    key = ("wgrad", tuple(dy2.shape), x2.shape[1], out_dtype, dy2.device)
    c = _NARROW_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return True
        c = _NARROW_CHOICE[key] = timed_choice(lambda: narrow_wgrad(dy2, x2, out_dtype),
                                               lambda: _library_wgrad(dy2, x2, out_dtype),
                                               table=_NARROW_CHOICE, key=key, name="narrow")
    return c


def _tall_skinny(m: int, n: int, k: int) -> bool:
    return m >= 16 * _WGRAD_CHUNK and max(n, k) <= 1024


def _split_k(m: int, n: int, k: int) -> int:
    """Token-dimension split for SMALL weight gradients (N x K <= 2.5M outputs: a few dozen 256 x 256
    output tiles for 256 CUs).  GPT-2 124M at 16 x 1024 tokens (profiles/r1_v10_gemm_small.jsonl):
    2304x768 134 -> 91 us (8-way), 768x768 95 -> 49 us (8-way), 3072x768 / 768x3072 151 -> 95 us (4-way);
    the 1.3B flagship's >= 2048x2048 gradients gain nothing and stay one GEMM."""
    nk = n * k
    if m < 8192 or nk > 2_500_000:
        return 1
    s = 8 if nk < 2_000_000 else 4
    while s > 1 and (m % s or m // s < 1024):
        s //= 2
    return s


# PDT_WGRAD_HIP: "auto" (default: per shape, the faster of the hand kernel and hipBLASLt, timed once on the
# shape's first uncaptured call), "1" (always the hand kernel where it applies), "0" (never)
HIP_WGRAD = os.environ.get("PDT_WGRAD_HIP", "auto")
_WGRAD_CHOICE: dict = {}


def _prefer_hip_wgrad(dy2: torch.Tensor, x2: torch.Tensor, ragged: bool = False) -> bool:
    """Hand kernel vs hipBLASLt for this weight-gradient shape.  Measured, not assumed: the two trade places
    by shape and by box (GPT-2 1.3B attention projection +12 %, fc1 +3 %, Llama-3 8B qkv -14 % on one box;
    the flagship gained 3 % on another, profiles/r2_wgrad_hip_vs_hipblaslt.jsonl)."""
    if HIP_WGRAD != "auto":
        return HIP_WGRAD == "1"
    key = (dy2.shape, x2.shape[1], dy2.device)
    c = _WGRAD_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return True
        # against the path wgrad() would otherwise take (split-K batched GEMM for small outputs, else one GEMM)
        hip = hip_wgrad_ragged if ragged else hip_wgrad
        c = _WGRAD_CHOICE[key] = timed_choice(lambda: hip(dy2, x2), lambda: _library_wgrad(dy2, x2, torch.bfloat16),
                                                    table=_WGRAD_CHOICE, key=key, name="wgrad")
    return c


def hip_wgrad_splits(m: int, n: int, k: int, cus: int = 256) -> int:
    """Token-dimension split of the HIP weight-gradient GEMM (``ops.gemm.tt_splits``): the slice count whose
    256x256-tile x slice workgroups fill whole waves of the 256 CUs best, >= 4096 tokens per slice; outputs
    of >= one wave of tiles are not split (the fp32 slab pass would cost more)."""
    return tt_splits(n, k, m, cus)


def hip_wgrad_ok(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype) -> bool:
    m, n = dy2.shape
    k = x2.shape[1]
    return (HIP_WGRAD != "0" and dy2.is_cuda and out_dtype == torch.bfloat16 and m >= 4096
            and tt_ok(dy2, x2, hip_wgrad_splits(m, n, k)))


def hip_wgrad(dy2: torch.Tensor, x2: torch.Tensor, splits: int | None = None, out: torch.Tensor | None = None):
    """dW [N, K] = dy2^T x2 on the hand MFMA GEMM (csrc/kernels/gemm.hip, TT layout: both operands token-major,
    fragments read transposed from LDS), bf16 out (into ``out`` when given)."""
    m, n = dy2.shape
    k = x2.shape[1]
    return gemm_tt(dy2, x2, splits or hip_wgrad_splits(m, n, k), out=out)


def _ragged_rows(n: int) -> int:
    """Rows of an N-row weight gradient the 256-row hand-kernel tiles cover (the rest go to hipBLASLt)."""
    return n // 256 * 256


def hip_wgrad_ragged_ok(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype) -> bool:
    """Weight gradients whose row count is not a multiple of 256 but large (GPT-2's tied LM head: 50,304 vocab
    rows): the leading 256-multiple on the hand kernel, a < 256-row remainder on hipBLASLt."""
    m, n = dy2.shape
    k = x2.shape[1]
    nm = _ragged_rows(n)
    return (HIP_WGRAD != "0" and dy2.is_cuda and out_dtype == torch.bfloat16 and m >= 4096 and nm >= 4096
            and nm < n and tt_ok(dy2[:, :nm], x2, hip_wgrad_splits(m, nm, k)))


def hip_wgrad_ragged(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    m, n = dy2.shape
    k = x2.shape[1]
    nm = _ragged_rows(n)
    if out is None:
        out = torch.empty(n, k, dtype=torch.bfloat16, device=dy2.device)
    gemm_tt(dy2[:, :nm], x2, hip_wgrad_splits(m, nm, k), out=out[:nm])
    if m % 16 == 0 and x2.is_contiguous():
        # the < 256-row remainder is a K = tokens, tiny-output product: 16 token slices as one batched GEMM
        # (0.40 -> 0.15 ms for the LM head's 128 rows, profiles/r4/r4_lm_head_paths_after.jsonl)
        rest = dy2[:, nm:].contiguous()
        c = m // 16
        out[nm:].copy_(torch.bmm(rest.view(16, c, n - nm).transpose(1, 2), x2.view(16, c, k),
                                 out_dtype=torch.float32).sum(0))
    else:
        torch.mm(dy2[:, nm:].t(), x2, out=out[nm:])
    return out


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype, out: torch.Tensor | None = None):
    """dW = dy2^T @ x2 ([M, N]^T [M, K] -> [N, K]) in ``out_dtype``; the hand MFMA kernel for large bf16
    shapes (a ragged row count split between it and hipBLASLt), row-split batched GEMM for tall-skinny M.
    ``out``: a contiguous [N, K] ``out_dtype`` tensor the result is written into (the GEMM's own output where
    the path allows, e.g. an FSDP unit's flat-gradient slot -- ops.grad_slots)."""
    m, n = dy2.shape
    k = x2.shape[1]
    if not dy2.is_cuda:
        r = torch.mm(dy2.t(), x2).to(out_dtype)
    elif hip_wgrad_ok(dy2, x2, out_dtype) and _prefer_hip_wgrad(dy2, x2):
        r = hip_wgrad(dy2, x2, out=out)
    elif hip_wgrad_ragged_ok(dy2, x2, out_dtype) and _prefer_hip_wgrad(dy2, x2, ragged=True):
        r = hip_wgrad_ragged(dy2, x2, out=out)
    elif _prefer_narrow_wgrad(dy2, x2, out_dtype):
        r = narrow_wgrad(dy2, x2, out_dtype)
    else:
        r = _library_wgrad(dy2, x2, out_dtype, out=out)
    if out is not None and r.data_ptr() != out.data_ptr():
        out.copy_(r)
        r = out
    return r


def _wgrad_result(w: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor):
    """A Linear backward's weight gradient: written into the parameter's FSDP flat-gradient slot when it has one
    (ops.grad_slots; returns None, autograd then carries no gradient for the weight), else returned."""
    slot = claim(w)
    if slot is None:
        return wgrad(dy2, x2, w.dtype)
    dst, acc = slot
    if acc:
        dst.add_(wgrad(dy2, x2, w.dtype))
    else:
        wgrad(dy2, x2, w.dtype, out=dst)
    return None


def _library_wgrad(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype, out: torch.Tensor | None = None):
    """dW on hipBLASLt: one GEMM, a token-split batched GEMM (small outputs) or the row-split tall-skinny form."""
    m, n = dy2.shape
    k = x2.shape[1]
    if not _tall_skinny(m, n, k):
        sk = _split_k(m, n, k)
        if sk == 1:
            if out is not None and out.dtype == dy2.dtype == x2.dtype:
                return torch.mm(dy2.t(), x2, out=out)
            return torch.mm(dy2.t(), x2).to(out_dtype)
        c = m // sk
        g = torch.bmm(dy2.view(sk, c, n).transpose(1, 2), x2.view(sk, c, k), out_dtype=torch.float32).sum(0)
        return g.to(out_dtype)
    s = m // _WGRAD_CHUNK
    main = s * _WGRAD_CHUNK
    a = dy2[:main].view(s, _WGRAD_CHUNK, n).transpose(1, 2)
    b = x2[:main].view(s, _WGRAD_CHUNK, k)
    g = torch.bmm(a, b, out_dtype=torch.float32).sum(0)
    if main < m:
        g += torch.mm(dy2[main:].t(), x2[main:], out_dtype=torch.float32)
    return g.to(out_dtype)


def transpose16(w: torch.Tensor) -> torch.Tensor:
    """w.t().contiguous() for a contiguous 16-bit GPU matrix with both dims % 64 == 0 (HIP LDS-tiled kernel)."""
    r, c = w.shape
    out = torch.empty(c, r, dtype=w.dtype, device=w.device)
    _lib.call("pdt_transpose16", w.data_ptr(), out.data_ptr(), r, c, _lib.stream_handle(w.device))
    return out


def _dgrad_via_transpose(m: int, n: int, k: int, w: torch.Tensor) -> bool:
    """dX = dY W ([M, N] x [N, K]) as F.linear(dY, W^T): hipBLASLt's NN-layout kernels for this product ran
    10-25 % below the forward's x W^T layout on the flagship shapes (qkv 0.79 -> 0.59 ms, fc2 0.89 -> 0.75 ms,
    tied LM head 4.97 -> 4.36 ms at 32 x 1024 tokens, profiles/r1_v11_gemm_dgrad_layout.jsonl); the weight
    transpose costs ~1 % of the GEMM.  GPT-2 124M's 0.6-2.4M-element weights gain too (901k -> 930-936k tokens/s,
    profiles/r2_gpt2_124m_dgrad_nt_threshold.log); SwinIR's (< 11k elements) keep the single mm."""
    return (w.is_cuda and w.dtype in (torch.bfloat16, torch.float16) and w.is_contiguous() and m >= 4096
            and n % 64 == 0 and k % 64 == 0 and n * k >= _DGRAD_T_MIN and n // 64 <= 65535 and w.data_ptr() % 16 == 0)


_DGRAD_T_MIN = int(os.environ.get("PDT_DGRAD_T_MIN", "500000"))    # smallest weight (elements) for the NT dgrad


BGRAD_IN_GEMM = os.environ.get("PDT_BGRAD_GEMM", "0") == "1"   # opt-in: no bench workload gains (r2)


def _bgrad_in_gemm(dy2: torch.Tensor, w: torch.Tensor) -> bool:
    """Plain single-GEMM weight gradients of bf16 Linears (not the split / row-split small-shape paths)."""
    m, n = dy2.shape
    k = w.shape[1]
    return (BGRAD_IN_GEMM and dy2.is_cuda and dy2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and not _tall_skinny(m, n, k) and _split_k(m, n, k) == 1 and n % 8 == 0 and k % 8 == 0 and colsum_ok(n))


def _as_output(t: torch.Tensor, shape) -> torch.Tensor:
    """A Function's forward output in its final shape WITHOUT being a view: autograd forbids in-place updates of
    view outputs created inside a custom Function (Llama's RoPE rotates the qkv projection in place)."""
    return torch.ops.aten._unsafe_view(t, shape)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, hm=None, in_hm=None):
        ctx.save_for_backward(x, weight)
        ctx.in_hm = in_hm
        ctx.has_bias = bias is not None
        # x is (a view of) a flash-attention output whose backward wants colsum(dX) (ops.attention._dout_colsum)
        base = x._base if x._base is not None else x
        ctx.dx_colsum = bias is not None and getattr(base, "_pdt_dx_colsum", False)
        x2 = x.reshape(-1, x.shape[-1])
        if hm is not None:      # linear_head_major checked the narrow kernel applies and was picked
            return _as_output(narrow_linear(x2, weight, bias, hm=hm)[0], (*x.shape[:-1], weight.shape[0]))
        if in_hm is not None:   # linear_from_head_major: x's buffer is head-major (the window attention's output)
            return _as_output(narrow_linear(x2, weight, bias, a_hm=in_hm)[0], (*x.shape[:-1], weight.shape[0]))
        if x2.is_contiguous() and _prefer_narrow(x2, weight, bias, "fwd"):
            return _as_output(narrow_linear(x2, weight, bias)[0], (*x.shape[:-1], weight.shape[0]))
        if x2.is_contiguous() and _nt_hip_ok(x2, weight, bias):
            return _as_output(nt_matmul(x2, weight, bias), (*x.shape[:-1], weight.shape[0]))
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        if ctx.in_hm is not None:
            return _LinearFn._backward_head_major(ctx, x, w, dy, dy2) + (None, None)
        dx = dw = db = None
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] and want_db and _bgrad_in_gemm(dy2, w):
            # weight AND bias gradient from one hipBLASLt GEMM (BGRADB epilogue) where that is measured faster
            # than the GEMM + column-sum pair for this shape (ops.blaslt.prefer_bgradb)
            x2 = x.reshape(-1, x.shape[-1])
            x2 = x2 if x2.is_contiguous() else x2.contiguous()
            if prefer_bgradb(dy2, x2, lambda: (wgrad(dy2, x2, w.dtype), _colsum(dy2, w.dtype))):
                r = wgrad_bgrad(dy2, x2)
                if r is not None:
                    dw, db = r
                    want_db = False
        if ctx.needs_input_grad[1] and dw is None:
            # (a concurrent dW on a second HIP stream measured 1 % slower on the flagship shapes,
            # profiles/r1_v11_wgrad_side_stream.log, and was removed)
            x2 = x.reshape(-1, x.shape[-1])
            if not x2.is_contiguous():
                x2 = x2.contiguous()
            dw = _wgrad_result(w, dy2, x2)
        dx2 = dbf = None
        if ctx.needs_input_grad[0] and _prefer_narrow(dy2, w, None, "dgrad"):
            # narrow data gradient dY W = dY (W^T)^T on the HIP kernel; the bias gradient colsum(dY) from its read
            # unless the kernel that produced dY already summed it (take_bias_grad)
            pre = take_bias_grad(dy2) if want_db else None
            dx2, cs = narrow_linear(dy2, w.t().contiguous(), None, w.dtype if (want_db and pre is None) else None)
            dx = dx2.view(*dy.shape[:-1], w.shape[1])
            if want_db:
                if pre is not None:
                    dbf, db = pre, pre.to(w.dtype)
                else:
                    db = cs
                want_db = False
        elif ctx.needs_input_grad[0]:
            if _dgrad_via_transpose(dy2.shape[0], w.shape[0], w.shape[1], w):
                dx2 = nt_matmul(dy2, transpose16(w))
            else:
                dx2 = torch.mm(dy2, w)
            dx = dx2.view(*dy.shape[:-1], w.shape[1])
        if want_db:
            db = take_bias_grad(dy2)      # summed by the kernel that produced dY (flash attention's backward)
            if db is not None:
                dbf, db = db, db.to(w.dtype)
            else:
                db = _colsum(dy2, w.dtype) if (dy2.is_cuda and colsum_ok(dy2.shape[1])) else dy2.sum(0).to(w.dtype)
        if ctx.dx_colsum and _DX_STASH and dx is not None and db is not None:
            # colsum(dX) = colsum(dY W) = db W: the attention backward's v-bias gradient without a pass over dX.
            # Stashed on the GEMM's own output, not on the view returned: the engine drops the Python object of
            # what a backward returns (a weak reference to it dies), the base's survives through the view
            dbf = dbf if dbf is not None and dbf.dtype == torch.float32 else db.float()
            stash_dx_colsum(dx2, dbf @ w.float())
        return dx, dw, db, None, None

    @staticmethod
    def _backward_head_major(ctx, x, w, dy, dy2):
        """x was read head-major (linear_from_head_major): the data gradient is written head-major as well (tagged
        for the window attention's backward), the weight gradient reads x head-major; off the narrow kernels x is
        put back token-major first."""
        n_tok, d = ctx.in_hm
        x2 = x.reshape(-1, x.shape[-1])
        dx = dw = db = None
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1]:
            if narrow_wgrad_ok(dy2, x2, w.dtype) and n_tok == 64:
                dw = narrow_wgrad(dy2, x2, w.dtype, x_hm_d=d)
            else:
                dw = wgrad(dy2, _token_major(x2, n_tok, d), w.dtype)
        if ctx.needs_input_grad[0]:
            wt = w.t().contiguous()
            if narrow_ok(dy2, wt):
                dx2, cs = narrow_linear(dy2, wt, None, w.dtype if want_db else None, hm=(n_tok, d))
                dx = dx2.view(*dy.shape[:-1], w.shape[1])
                dx._pdt_head_major = (n_tok, d)
                if want_db:
                    db, want_db = cs, False
            else:
                dx = torch.mm(dy2, w).view(*dy.shape[:-1], w.shape[1])
        if want_db:
            db = _colsum(dy2, w.dtype) if (dy2.is_cuda and colsum_ok(dy2.shape[1])) else dy2.sum(0).to(w.dtype)
        return dx, dw, db


def _token_major(x2: torch.Tensor, n_tok: int, d: int) -> torch.Tensor:
    """[M, C] token-major copy of a head-major buffer ([M / n_tok, C / d, n_tok, d])."""
    M, C = x2.shape
    return x2.reshape(M // n_tok, C // d, n_tok, d).permute(0, 2, 1, 3).reshape(M, C)


def _lin_residual_fwd(x2, w, b, r2):
    """x2 W^T (+ b) + r2 in one hipBLASLt GEMM (C = r2), else the GEMM and an add."""
    from .blaslt import linear_residual as _lt_residual
    if x2.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and r2.dtype == torch.bfloat16 \
            and (b is None or b.dtype == torch.bfloat16) and w.is_contiguous() and r2.is_contiguous():
        d = _lt_residual(x2, w, b, r2)
        if d is not None:
            return d
    return torch.addmm(r2, x2, w.t()) if b is None else F.linear(x2, w, b) + r2


class _LinearResidualFn(torch.autograd.Function):
    """out = x W^T (+ b) + r: the residual stream added by the GEMM that writes the projection (hipBLASLt's
    accumulate input), so the following norm reads one stream instead of summing two.  Backward: dr = dout (the
    same buffer), dW / dx as ``_LinearFn``, db from the following norm's pass (``take_bias_grad``) when it summed
    it, else a column sum."""

    @staticmethod
    def forward(ctx, x, weight, bias, r):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        base = x._base if x._base is not None else x
        ctx.dx_colsum = bias is not None and getattr(base, "_pdt_dx_colsum", False)
        n = weight.shape[0]
        x2 = x.reshape(-1, x.shape[-1])
        x2 = x2 if x2.is_contiguous() else x2.contiguous()
        r2 = r.reshape(-1, n)
        r2 = r2 if r2.is_contiguous() else r2.contiguous()
        if r2.data_ptr() % 16 == 0 and r2.dtype == x2.dtype and _prefer_narrow(x2, weight, bias, "fwd"):
            # narrow linears (SwinIR's MLP fc2): the residual added in the narrow GEMM's store
            return _as_output(narrow_linear(x2, weight, bias, residual=r2)[0], (*x.shape[:-1], n))
        return _as_output(_lin_residual_fwd(x2, weight, bias, r2), (*x.shape[:-1], n))

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
        dx = dx2 = dw = db = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            x2 = x2 if x2.is_contiguous() else x2.contiguous()
            dw = _wgrad_result(w, dy2, x2)
        dbf = None
        if ctx.needs_input_grad[0]:
            if _prefer_narrow(dy2, w, None, "dgrad"):
                # narrow data gradient, colsum(dY) (the bias gradient) from the same read unless already summed
                want = ctx.has_bias and (ctx.needs_input_grad[2] or ctx.dx_colsum)
                pre = take_bias_grad(dy2) if want else None
                dx2, cs = narrow_linear(dy2, w.t().contiguous(), None, torch.float32 if (want and pre is None) else None)
                dbf = pre if pre is not None else cs
            elif _dgrad_via_transpose(dy2.shape[0], w.shape[0], w.shape[1], w):
                dx2 = nt_matmul(dy2, transpose16(w))
            else:
                dx2 = torch.mm(dy2, w)
            dx = dx2.view(*dy.shape[:-1], w.shape[1])
        if ctx.has_bias and (ctx.needs_input_grad[2] or ctx.dx_colsum):
            if dbf is None:
                dbf = take_bias_grad(dy2)
            if dbf is None:
                dbf = _colsum(dy2, torch.float32) if (dy2.is_cuda and colsum_ok(dy2.shape[1])) else dy2.float().sum(0)
            db = dbf.to(w.dtype)
            if ctx.dx_colsum and _DX_STASH and dx2 is not None:   # (on the base: see _LinearFn)
                stash_dx_colsum(dx2, dbf.float() @ w.float())
            if not ctx.needs_input_grad[2]:
                db = None
        return dx, dw, db, (dy if ctx.needs_input_grad[3] else None)


def linear_residual(x, weight, bias, r):
    """x W^T (+ bias) + r with the add in the GEMM (``_LinearResidualFn``); plain ops off the GPU path."""
    if x.is_cuda and x.dtype == weight.dtype == r.dtype and x.dtype in (torch.bfloat16, torch.float32) \
            and (bias is None or bias.dtype == x.dtype) and not torch.is_autocast_enabled("cuda"):
        return _LinearResidualFn.apply(x, weight, bias, r)
    return linear(x, weight, bias) + r


FUSED_GELU = os.environ.get("PDT_FUSED_GELU", "1") == "1"


def linear_bias_gelu_ok(x, weight, bias) -> bool:
    """gelu_tanh(x W^T + b) in ONE hand-GEMM pass (``ops.gemm.gemm_nt_gelu``: bias + GELU in the epilogue, the
    GELU derivative kept for the backward) -- bf16, the hand kernel's tile grid, K >= 128."""
    from . import gemm as G
    if not (FUSED_GELU and G.KERNEL["name"] == "asm" and x.is_cuda and bias is not None):
        return False
    if torch.is_autocast_enabled("cuda") or x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16 \
            or bias.dtype != torch.bfloat16 or not weight.is_contiguous():
        return False
    m = x.numel() // x.shape[-1]
    n, k = weight.shape
    return (m % 256 == 0 and n % 256 == 0 and k % 64 == 0 and k >= 128 and x.shape[-1] == k
            and G.gemm_ok(G.L_NT, m, n, k, k, k) and weight.data_ptr() % 16 == 0)


class _LinearBiasGeluFn(torch.autograd.Function):
    """y = gelu_tanh(x W^T + b): forward on the hand NT GEMM with the bias + GELU epilogue (replaces hipBLASLt +
    the separate bias-GELU pass over the [tokens, 4d] hidden), which keeps gelu'(h) rather than h; backward = one
    multiply + bias-gradient sweep over that derivative (no transcendental), then the Linear's weight / data
    gradients."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from . import gemm as G
        x2 = x.reshape(-1, x.shape[-1])
        x2 = x2 if x2.is_contiguous() and x2.data_ptr() % 16 == 0 else x2.contiguous()
        y, d = G.gemm_nt_gelu(x2, weight, bias)
        ctx.save_for_backward(x2, weight, d)
        ctx.xshape = x.shape
        return _as_output(y, (*x.shape[:-1], weight.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        x2, w, d = ctx.saved_tensors
        dy2 = dy.reshape(d.shape)
        dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
        rows, n = d.shape
        lib = _lib.require()
        dpre = torch.empty_like(d)
        db = torch.empty(n, dtype=w.dtype, device=d.device)
        ws = torch.empty(lib.pdt_colsum_ws_floats(rows, n), dtype=torch.float32, device=d.device)
        # mode 2: d already is gelu'(pre-activation) -> dpre = dy * d and its column sums
        _lib.call("pdt_bias_gelu_bwd_db", dy2.data_ptr(), d.data_ptr(), None, dpre.data_ptr(),
                  db.data_ptr(), ws.data_ptr(), rows, n, _lib.dtype_code(d.dtype), _lib.dtype_code(db.dtype), 2, 0,
                  _lib.stream_handle(d.device))
        dw = _wgrad_result(w, dpre, x2) if ctx.needs_input_grad[1] else None
        dx = None
        if ctx.needs_input_grad[0]:
            if _dgrad_via_transpose(rows, w.shape[0], w.shape[1], w):
                dx = nt_matmul(dpre, transpose16(w))
            else:
                dx = torch.mm(dpre, w)
            dx = dx.view(*ctx.xshape)
        return dx, dw, (db if ctx.needs_input_grad[2] else None)


def linear_bias_gelu(x, weight, bias):
    """gelu_tanh(x W^T + b) (GPT-2's c_fc + GELU): one fused pass where ``linear_bias_gelu_ok``."""
    return _LinearBiasGeluFn.apply(x, weight, bias)


# default since round 5: the forward keeps gelu'(h) (the DGELU epilogue is a multiply), the epilogue no longer spills
# (spill reloads had put a vmcnt(0) in front of every main loop) and its round-0 / round-1 rows load under the main loop:
# DGELU 1,246 TFLOP/s vs 1,035 for the plain GEMM + sweep it replaces; flagship 147.3k vs 144.0k tokens/s
# (profiles/r5/r5_dgelu_gemm.jsonl, r5_dgelu_bench.log).  PDT_FUSED_DGELU=0 restores the sweep.
FUSED_DGELU = os.environ.get("PDT_FUSED_DGELU", "1") == "1"


def gelu_mlp_ok(x, w1, b1, w2, b2) -> bool:
    """The whole MLP (c_fc + GELU + c_proj) as ``gelu_mlp``: c_fc as ``linear_bias_gelu`` and c_proj's data
    gradient on the hand NT GEMM with the GELU-backward + c_fc bias-gradient epilogue."""
    return (FUSED_DGELU and linear_bias_gelu_ok(x, w1, b1) and w2.dtype == torch.bfloat16 and w2.is_contiguous()
            and b2 is not None and b2.dtype == torch.bfloat16 and w2.shape[1] == w1.shape[0]
            and w2.shape[0] % 64 == 0 and w2.shape[0] >= 128)


class _GeluMlpFn(torch.autograd.Function):
    """out = gelu_tanh(x W1^T + b1) W2^T + b2 (GPT-2's MLP).  Forward: c_fc + bias + GELU in one hand-GEMM pass,
    c_proj on hipBLASLt.  Backward: c_proj's data gradient, the GELU backward and c_fc's bias gradient in ONE hand-GEMM
    pass (DGELU epilogue: a multiply by the kept derivative) -- no separate sweep over the [tokens, 4d] hidden."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, r=None):
        from . import gemm as G
        x2 = x.reshape(-1, x.shape[-1])
        x2 = x2 if x2.is_contiguous() and x2.data_ptr() % 16 == 0 else x2.contiguous()
        y1, d1 = G.gemm_nt_gelu(x2, w1, b1)
        if r is None:
            out = F.linear(y1, w2, b2)
        else:   # + the residual stream, added by the c_proj GEMM itself (``linear_residual``)
            r2 = r.reshape(-1, w2.shape[0])
            out = _lin_residual_fwd(y1, w2, b2, r2 if r2.is_contiguous() else r2.contiguous())
        ctx.save_for_backward(x2, w1, d1, y1, w2)
        ctx.xshape = x.shape
        ctx.has_r = r is not None
        return _as_output(out, (*x.shape[:-1], w2.shape[0]))

    @staticmethod
    def backward(ctx, dout):
        from . import gemm as G
        x2, w1, d1, y1, w2 = ctx.saved_tensors
        d2 = dout.reshape(-1, dout.shape[-1])
        d2 = d2 if d2.is_contiguous() and d2.data_ptr() % 16 == 0 else d2.contiguous()
        dw2 = _wgrad_result(w2, d2, y1) if ctx.needs_input_grad[3] else None
        db2 = None
        if ctx.needs_input_grad[4]:
            db2 = take_bias_grad(d2)      # summed by the kernel that produced dY (the next LayerNorm's backward)
            db2 = db2.to(w2.dtype) if db2 is not None else _colsum(d2, w2.dtype)
        # c_proj dgrad (d2 W2) x GELU'(pre) (= d1, kept by the forward), and c_fc's bias gradient, in one pass
        dpre, db1 = G.gemm_nt_dgelu(d2, transpose16(w2), d1, bias_dtype=w1.dtype)
        dw1 = _wgrad_result(w1, dpre, x2) if ctx.needs_input_grad[1] else None
        dx = None
        if ctx.needs_input_grad[0]:
            if _dgrad_via_transpose(dpre.shape[0], w1.shape[0], w1.shape[1], w1):
                dx = nt_matmul(dpre, transpose16(w1))
            else:
                dx = torch.mm(dpre, w1)
            dx = dx.view(*ctx.xshape)
        dr = dout if ctx.has_r and ctx.needs_input_grad[5] else None
        return dx, dw1, (db1 if ctx.needs_input_grad[2] else None), dw2, db2, dr


def gelu_mlp(x, w1, b1, w2, b2, residual=None):
    """gelu_tanh(x W1^T + b1) W2^T + b2 (+ residual, added by the c_proj GEMM)."""
    return _GeluMlpFn.apply(x, w1, b1, w2, b2, residual)


def linear(x, weight, bias=None):
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            return linear(x.to(dt), weight.to(dt), None if bias is None else bias.to(dt))
    if (x.is_cuda or is_sharded_param(weight) or hasattr(x, "_pdt_recipe")) and x.dtype == weight.dtype and \
            x.dtype in (torch.bfloat16, torch.float32) and (bias is None or bias.dtype == x.dtype):
        # (an FSDP parameter takes this path on the CPU too: its backward writes dW into the unit's flat slot; so does
        # an input saved as a recompute recipe (utils.recompute): this Function saves x itself, not a view of it)
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


# PDT_HEAD_MAJOR_QKV=0: Swin's qkv projection always writes token-major (A/B of linear_head_major)
HEAD_MAJOR_QKV = os.environ.get("PDT_HEAD_MAJOR_QKV", "1") == "1"


def _has_hooks(module: nn.Module) -> bool:
    """Forward / pre-forward hooks on the module (or globally): the head-major paths call the GEMM directly, so they
    step aside for anything that expects to see ``module(x)``."""
    return bool(module._forward_hooks or module._forward_pre_hooks or nn.modules.module._global_forward_hooks
                or nn.modules.module._global_forward_pre_hooks)


def linear_head_major(module: "Linear", x: torch.Tensor, n_tok: int, head_dim: int) -> torch.Tensor:
    """``module(x)`` for a projection whose ONLY consumer is ops.window_attention (Swin's qkv): where the narrow
    GEMM computes it, the output buffer is written head-major ([windows, 3, heads, n_tok, d], ops.narrow) and the
    tensor is tagged ``_pdt_head_major = (n_tok, d)``, so the attention's staging loads read each head's token
    slices contiguously (no relayout pass).  The tensor keeps its logical [..., 3C] shape, and its gradient
    arrives token-major as usual (the Linear's backward never reads its output).  Anything else: ``module(x)``."""
    from .narrow import head_major_ok
    if HEAD_MAJOR_QKV and x.is_cuda and not fp8_enabled() and not _has_hooks(module):
        xc = x.to(torch.get_autocast_dtype("cuda")) if torch.is_autocast_enabled("cuda") else x
        w, b = module.weight, module.bias
        if torch.is_autocast_enabled("cuda"):
            w, b = w.to(xc.dtype), (None if b is None else b.to(xc.dtype))
        x2 = xc.reshape(-1, xc.shape[-1])
        if (xc.dtype == w.dtype and xc.dtype in (torch.bfloat16, torch.float32) and (b is None or b.dtype == xc.dtype)
                and x2.is_contiguous() and head_major_ok(x2.shape[0], w.shape[0], (n_tok, head_dim))
                and _prefer_narrow(x2, w, b, "fwd")):
            with torch.autocast("cuda", enabled=False):
                y = _LinearFn.apply(xc, w, b, (n_tok, head_dim))
            y._pdt_head_major = (n_tok, head_dim)
            return y
    return module(x)


def linear_from_head_major(module: "Linear", x: torch.Tensor) -> torch.Tensor:
    """``module(x)`` for x tagged ``_pdt_head_major = (n_tok, d)`` (ops.window_attention's output written head-major):
    the narrow GEMM reads the head-major buffer directly, and its backward writes the data gradient head-major for
    the attention's backward.  Untagged x: ``module(x)``; a tagged x the narrow path cannot take is put back
    token-major first."""
    hm = getattr(x, "_pdt_head_major", None)
    if hm is None:
        return module(x)
    n_tok, d = hm
    if _has_hooks(module):     # hooks see the module's usual call on a token-major input
        return module(_token_major(x.reshape(-1, x.shape[-1]), n_tok, d).view(x.shape))
    w, b = module.weight, module.bias
    if torch.is_autocast_enabled("cuda"):
        w, b = w.to(x.dtype), (None if b is None else b.to(x.dtype))
    x2 = x.reshape(-1, x.shape[-1])
    if (x.dtype == torch.bfloat16 and w.dtype == x.dtype and (b is None or b.dtype == x.dtype) and not fp8_enabled()
            and x2.is_contiguous() and narrow_ok(x2, w, b)):
        with torch.autocast("cuda", enabled=False):
            return _LinearFn.apply(x, w, b, None, hm)
    return module(_token_major(x2, n_tok, d).view(x.shape))


class Linear(nn.Linear):
    """nn.Linear on the framework GEMM paths; inside ``ops.fp8.fp8_autocast()`` its three GEMMs run in fp8
    with this module's delayed-scaling state (created on first fp8 use, not part of the state_dict)."""

    def _fp8_meta(self, x):
        if not (fp8_enabled() and x.dtype in (torch.bfloat16, torch.float16) and self.in_features % 16 == 0
                and self.out_features % 16 == 0):
            return None
        meta = self.__dict__.get("_fp8")
        if meta is None:
            meta = self.__dict__["_fp8"] = Fp8Meta(x.device)
        return meta

    def forward(self, x):
        return self.matmul(x, self.bias)

    def matmul(self, x, bias=None):
        """x W^T (+ bias): ``matmul(x)`` is the bias-free product for callers that fuse the bias into the
        following kernel (GPT-2's bias-GELU)."""
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            x = x.to(torch.get_autocast_dtype("cuda"))
        meta = self._fp8_meta(x)
        if meta is not None and x.shape[:-1].numel() % 16 == 0:
            w = self.weight if self.weight.dtype == x.dtype else self.weight.to(x.dtype)
            b = None if bias is None else bias.to(x.dtype)
            return fp8_linear(x, w, b, meta)
        return linear(x, self.weight, bias)
