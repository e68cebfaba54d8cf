"""Flash attention (causal / full, GQA) backed by the gfx950 MFMA kernels in csrc/kernels/flash_attn.hip.

Layout: q [B, Sq, H, D], k/v [B, Sk, Hkv, D] -- any strides with a contiguous head dim, so the
views of a fused qkv projection are consumed in place.  ``flash_attn_qkvpacked`` additionally writes
dq/dk/dv straight into one packed gradient buffer (no scatter/cat in backward).

CPU tensors use the exact-math reference (torch SDPA) -- used by the CPU tests only.
"""
from __future__ import annotations

import math

import weakref

import torch
import torch.nn.functional as F

from . import _lib
from ..utils import recompute as _rc


def _strides(t):
    return [t.stride(0), t.stride(1), t.stride(2)]


def _check(t, name):
    if t.dtype != torch.bfloat16:
        raise TypeError(f"flash_attn: {name} must be bf16 (got {t.dtype})")
    if t.stride(-1) != 1:
        raise ValueError(f"flash_attn: {name} head dim must be contiguous")
    if t.data_ptr() % 16 or any(s % 8 for s in t.stride()[:-1]):
        raise ValueError(f"flash_attn: {name} must be 16-byte aligned with strides multiple of 8")


def _fwd(q, k, v, causal, scale):
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    o = torch.empty((B, Sq, H, D), dtype=q.dtype, device=q.device)
    lse = torch.empty((B, H, Sq), dtype=torch.float32, device=q.device)
    strides = torch.tensor(_strides(q) + _strides(k) + _strides(v) + _strides(o), dtype=torch.int64)
    _lib.call("pdt_flash_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
              strides.data_ptr(), B, H, Hkv, Sq, Sk, D, float(scale), 1 if causal else 0,
              _lib.stream_handle(q.device))
    return o, lse


def _dout_colsum(do):
    """fp32 column sums of dO over (batch, query) rows -> [H*D]: stashed by the Linear whose data gradient dO is
    (``stash_dx_colsum``, computed there as db W without touching dO), else one column-sum pass."""
    cs = take_dx_colsum(do)
    if cs is not None:
        return cs
    from .activations import _colsum, colsum_ok
    d2 = do.reshape(-1, do.shape[-2] * do.shape[-1])
    if d2.is_contiguous() and colsum_ok(d2.shape[1]):
        return _colsum(d2, torch.float32)
    return d2.float().sum(0)


def _bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale, bias_grad=False):
    """dq, dk, dv; with ``bias_grad`` also returns the fp32 column sums of the stored dq | dk | dv rows
    ([H*D + 2*Hkv*D], the bias gradient of the packed qkv projection): the q part from per-workgroup partials of
    the dQ kernel, the k part exactly 0 and the v part from the column sums of dO (softmax identities, see
    pdt_flash_attn_bwd); None where the current kernel variant does not produce them."""
    B, Sq, H, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    delta = torch.empty((2, B, H, Sq), dtype=torch.float32, device=q.device)   # [delta | -lse*log2e]
    ws = db = cso = None
    if bias_grad:
        n = int(_lib.require().pdt_flash_attn_colsum_ws_floats(B, H, Hkv, Sq, Sk, D))
        if n > 0:
            ws = torch.empty(n, dtype=torch.float32, device=q.device)
            db = torch.empty((H + 2 * Hkv) * D, dtype=torch.float32, device=q.device)
            cso = _dout_colsum(do)
    do = do if (do.stride(-1) == 1 and all(s % 8 == 0 for s in do.stride()[:-1])) else do.contiguous()
    strides = torch.tensor(_strides(q) + _strides(k) + _strides(v) + _strides(o) + _strides(do) + _strides(dq)
                           + _strides(dk) + _strides(dv), dtype=torch.int64)
    _lib.call("pdt_flash_attn_bwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
              do.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), delta.data_ptr(), strides.data_ptr(),
              B, H, Hkv, Sq, Sk, D, float(scale), 1 if causal else 0, _lib.ptr(ws), _lib.ptr(db),
              _lib.dtype_code(torch.float32), _lib.ptr(cso), _lib.stream_handle(q.device))
    return db


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        for t, n in ((q, "q"), (k, "k"), (v, "v")):
            _check(t, n)
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        _bwd(q, k, v, o, lse, do, dq, dk, dv, ctx.causal, ctx.scale)
        return dq, dk, dv, None, None


class _FlashAttnPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, causal, scale, bias_grad):
        _check(qkv, "qkv")
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale, ctx.bias_grad = causal, scale, bias_grad
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        dqkv = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        db = _bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                  ctx.causal, ctx.scale, bias_grad=ctx.bias_grad)
        if db is not None:
            stash_bias_grad(dqkv, db)
        return dqkv, None, None, None


_BIAS_GRADS: dict = {}
_DX_COLSUMS: dict = {}


def _stash(table, grad, colsum):
    for key in [k for k, (ref, _, _) in table.items() if ref() is None]:
        del table[key]
    # a backward's RETURNED tensor loses its Python object once the engine takes it (a weak reference to it dies
    # before the consumer's backward runs); the base it views keeps its object, so hold that when it spans the
    # same elements
    base = grad._base
    if base is not None and base.data_ptr() == grad.data_ptr() and base.numel() == grad.numel():
        grad = base
    table[grad.untyped_storage().data_ptr()] = (weakref.ref(grad), colsum, grad._version)


def _take(table, t):
    ent = table.pop(t.untyped_storage().data_ptr(), None)
    if ent is None:
        return None
    src, colsum, version = ent[0](), ent[1], ent[2]
    if (src is None or src.untyped_storage().data_ptr() != t.untyped_storage().data_ptr()
            or src.numel() != t.numel() or colsum.numel() != t.shape[-1] * (t.shape[-2] if t.dim() == 4 else 1)
            or t.data_ptr() != src.data_ptr() or src._version != version or t._version != version):
        return None
    return colsum


def stash_bias_grad(grad, colsum):
    """Hand the column sums of the gradient buffer ``grad`` (computed by the kernel that wrote it) to the Linear
    whose output received that gradient: its backward takes them (``take_bias_grad``) instead of summing dY
    again.  Keyed by the buffer's storage; the entry holds the buffer weakly and dies with it, and records the
    buffer's version counter (shared by its views), so an in-place write between stash and take voids it."""
    _stash(_BIAS_GRADS, grad, colsum)


def take_bias_grad(dy):
    """The stashed column sums for ``dy`` (a 2-D [rows, N] view of a stashed gradient buffer, unmodified since
    the stash), once; else None (the caller sums dY itself)."""
    return _take(_BIAS_GRADS, dy) if dy.dim() == 2 else None


def stash_dx_colsum(dx, colsum):
    """Column sums of a Linear's data gradient ``dx`` (= db W, computed by that Linear from its bias gradient) for
    the attention backward that consumes dx as dO (``take_dx_colsum``): the v part of the qkv bias gradient."""
    _stash(_DX_COLSUMS, dx, colsum)


def take_dx_colsum(do):
    """The stashed fp32 [H*D] column sums of ``do`` ([B, S, H, D] or [rows, H*D] over a stashed buffer), once."""
    return _take(_DX_COLSUMS, do) if do.dim() in (2, 4) else None


_FRESH_GRADS = weakref.WeakValueDictionary()


def mark_fresh_grad(t):
    """Record that ``t`` is a gradient buffer this backward just allocated and hands to exactly one consumer,
    so that consumer may rewrite it in place (ops.rope's inverse rotation)."""
    _FRESH_GRADS[t.untyped_storage().data_ptr()] = t


def take_fresh_grad(t) -> bool:
    """True (once) if ``t`` views a buffer marked by ``mark_fresh_grad`` that is still alive.  A gradient that
    autograd accumulated from several consumers is a new buffer and reads False."""
    ptr = t.untyped_storage().data_ptr()
    src = _FRESH_GRADS.pop(ptr, None)
    return src is not None and src.untyped_storage().data_ptr() == ptr


class _FlashAttnGQAPackedFn(torch.autograd.Function):
    """q, k, v as head ranges of one [B, S, Hq + 2 Hkv, D] projection; backward writes the packed gradient."""

    @staticmethod
    def forward(ctx, qkv, hq, hkv, causal, scale):
        _check(qkv, "qkv")
        q, k, v = qkv[:, :, :hq], qkv[:, :, hq:hq + hkv], qkv[:, :, hq + hkv:]
        o, lse = _fwd(q, k, v, causal, scale)
        if _rc.active():     # selective recompute: o / lse saved as "run this forward again" (utils.recompute)
            recipe = _rc.Recipe(lambda: _fwd(q, k, v, causal, scale))
            _rc.tag(o, recipe, 0)
            _rc.tag(lse, recipe, 1)
        ctx.save_for_backward(qkv, o, lse)
        ctx.hq, ctx.hkv, ctx.causal, ctx.scale = hq, hkv, causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        hq, hkv = ctx.hq, ctx.hkv
        d = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        _bwd(qkv[:, :, :hq], qkv[:, :, hq:hq + hkv], qkv[:, :, hq + hkv:], o, lse, do, d[:, :, :hq],
             d[:, :, hq:hq + hkv], d[:, :, hq + hkv:], ctx.causal, ctx.scale)
        mark_fresh_grad(d)
        return d, None, None, None, None


def flash_attn_gqa_packed(qkv, n_q_heads: int, n_kv_heads: int, causal: bool = True, scale: float | None = None):
    """qkv [B, S, Hq + 2 Hkv, D] (q heads, then k, then v) -> o [B, S, Hq, D]; GQA (Hq % Hkv == 0)."""
    scale = 1.0 / math.sqrt(qkv.shape[-1]) if scale is None else scale
    hq, hkv = n_q_heads, n_kv_heads
    if not qkv.is_cuda:
        return _reference(qkv[:, :, :hq], qkv[:, :, hq:hq + hkv], qkv[:, :, hq + hkv:], causal, scale)
    return _FlashAttnGQAPackedFn.apply(qkv, hq, hkv, causal, scale)


def _reference(q, k, v, causal, scale):
    # [B, S, H, D] -> [B, H, S, D]; GQA by repeating kv heads
    H, Hkv = q.shape[2], k.shape[2]
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if Hkv != H:
        kt = kt.repeat_interleave(H // Hkv, dim=1)
        vt = vt.repeat_interleave(H // Hkv, dim=1)
    Sq, Sk = q.shape[1], k.shape[1]
    mask = None
    if causal:
        mask = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(diagonal=Sk - Sq)
    o = F.scaled_dot_product_attention(qt.float(), kt.float(), vt.float(), attn_mask=mask, scale=scale)
    return o.transpose(1, 2).to(q.dtype)


def flash_attn(q, k, v, causal: bool = True, scale: float | None = None):
    """softmax(q k^T * scale [+ causal mask]) v with q [B,Sq,H,D], k/v [B,Sk,Hkv,D]; returns [B,Sq,H,D]."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if not q.is_cuda:
        return _reference(q, k, v, causal, scale)
    return _FlashAttnFn.apply(q, k, v, causal, scale)


def flash_attn_qkvpacked(qkv, causal: bool = True, scale: float | None = None, bias_grad: bool = False):
    """qkv [B, S, 3, H, D] -> o [B, S, H, D].  ``bias_grad``: qkv is the output of a Linear with a bias (GPT-2's
    c_attn) -- the backward also produces that bias gradient (q part: the dQ kernel's column sums; k part: 0; v
    part: colsum(dO), stashed by a biased Linear consuming o -- GPT-2's c_proj -- as db W) and hands it to the
    Linear's backward (``take_bias_grad``), which then skips its own column-sum pass over dqkv."""
    scale = 1.0 / math.sqrt(qkv.shape[-1]) if scale is None else scale
    if not qkv.is_cuda:
        return _reference(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal, scale)
    o = _FlashAttnPackedFn.apply(qkv, causal, scale, bias_grad)
    if bias_grad:
        o._pdt_dx_colsum = True     # the Linear consuming o stashes colsum(dO) for this backward (ops.linear)
    return o


def set_kernel_variant(fwd: int = 0, bwd: int = 0) -> tuple:
    """Select the flash-attention kernels (0 keeps the current choice, -1 restores the default).
    fwd: 5 (default) 4 waves x 32 query rows per workgroup; 7 / 8 the same tile on 8-wave 256-row workgroups
    (3- / 2-deep LDS ring).  bwd (dQ kernel; dK/dV is always v3): 9 dQ v4 on 8-wave 256-row workgroups with a
    2-deep ring (default at head dim 128), 8 the same with a 3-deep ring, 3 dQ v3 on 4-wave 128-row workgroups
    (default at head dim 64).  Returns the pinned (fwd, bwd) pair (0 = default)."""
    r = _lib.require().pdt_flash_attn_set_variant(int(fwd), int(bwd))
    return r // 32, r % 32


def reset_kernel_variant() -> None:
    """Back to the default kernels and the per-shape block order."""
    set_kernel_variant(-1, -1)
    set_block_order(-2)


def set_block_order(order: int = -1) -> int:
    """Workgroup -> block order of the flash-attention kernels, a bitmask (bit 0 forward, bit 1 dK/dV, bit 2
    dQ): a set bit groups every (head, batch)'s blocks on one XCD, back to back, so the K/V (or Q/dO) re-reads
    hit that XCD's L2; a clear bit dispatches the longest causal blocks first across the chip.  -2 restores the
    per-shape default (forward grouped while one head's K/V fits comfortably in L2), -1 keeps the current
    setting.  Returns the setting in effect (-1 = per-shape default)."""
    return int(_lib.require().pdt_flash_attn_set_order(int(order)))


def supported(head_dim: int) -> bool:
    return head_dim in (64, 128)
