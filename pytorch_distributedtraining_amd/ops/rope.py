"""Rotary position embedding (rotate-half convention, Llama-3) with a gfx950 kernel.

cos/sin tables are precomputed once on the host side of the model (fp32 [S_max, D/2]) -- on-device
trig per element would turn this memory-bound op VALU-bound (cdna_hip_programming.md App. B).
"""
from __future__ import annotations

import torch

from . import _lib


def rope_tables(head_dim: int, max_seq: int, theta: float = 500000.0, device=None, scaling=None):
    """cos, sin fp32 tables of shape [max_seq, head_dim // 2]."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling is not None:
        inv = scaling(inv)
    pos = torch.arange(max_seq, dtype=torch.float64)
    f = torch.outer(pos, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def _rope_ref(x, cos, sin, pos0, sign):
    S, D = x.shape[1], x.shape[-1]
    c = cos[pos0:pos0 + S].view(1, S, 1, D // 2).to(torch.float32)
    s = sin[pos0:pos0 + S].view(1, S, 1, D // 2).to(torch.float32) * sign
    xf = x.float()
    a, b = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1).to(x.dtype)


def _launch(x, y, cos, sin, pos0, backward, heads=None):
    """Rotate heads [0, heads) of every position of x [B, S, Hx, D] into y (y may be x: in place)."""
    B, S, Hx, D = x.shape
    H = Hx if heads is None else heads
    _lib.call("pdt_rope", x.data_ptr(), y.data_ptr(), B * S * H, x.stride(2), x.stride(1), y.stride(2), y.stride(1),
              H, S, D, int(pos0), cos.data_ptr(), sin.data_ptr(), 1 if backward else 0, _lib.dtype_code(x.dtype),
              _lib.stream_handle(x.device))


def _rows_ok(t):
    B, S, H, D = t.shape
    return t.stride(3) == 1 and t.stride(1) == H * t.stride(2) and t.stride(0) == S * t.stride(1)


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos0):
        if not _rows_ok(x):
            x = x.contiguous()
        y = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        _launch(x, y, cos, sin, pos0, backward=False)
        ctx.save_for_backward(cos, sin)
        ctx.pos0 = pos0
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        dy = dy if _rows_ok(dy) else dy.contiguous()
        dx = torch.empty(dy.shape, dtype=dy.dtype, device=dy.device)
        _launch(dy, dx, cos, sin, ctx.pos0, backward=True)
        return dx, None, None, None


def apply_rope(x, cos, sin, pos0: int = 0):
    """x: [B, S, H, D] (rows of H*D contiguous); returns the rotated tensor (new storage)."""
    D = x.shape[-1]
    if not x.is_cuda or (D // 2) % 8 != 0 or x.dtype not in (torch.float32, torch.bfloat16):
        return _rope_ref(x, cos, sin, pos0, 1.0)
    # the kernel reads fp32 [>= pos0 + S, D/2] tables (a model cast to bf16 also casts its table buffers)
    if cos.dtype != torch.float32 or not cos.is_contiguous():
        cos = cos.float().contiguous()
    if sin.dtype != torch.float32 or not sin.is_contiguous():
        sin = sin.float().contiguous()
    if cos.shape != sin.shape or cos.dim() != 2 or cos.shape[1] != D // 2 or cos.shape[0] < pos0 + x.shape[1]:
        raise ValueError(f"apply_rope: tables {tuple(cos.shape)} do not cover positions {pos0}..{pos0 + x.shape[1]}"
                         f" x head_dim/2={D // 2}")
    return _RopeFn.apply(x, cos, sin, pos0)


def _tables_f32(cos, sin):
    if cos.dtype != torch.float32 or not cos.is_contiguous():
        cos = cos.float().contiguous()
    if sin.dtype != torch.float32 or not sin.is_contiguous():
        sin = sin.float().contiguous()
    return cos, sin


class _RopeQKInplaceFn(torch.autograd.Function):
    """RoPE on the q and k heads of a packed [B, S, (Hq + 2 Hkv) * D] projection output, in place; backward
    applies the inverse rotation in place on the packed gradient.  No separate q / k tensors exist in either
    direction, and the packed flash attention consumes the result (and produces the packed gradient).
    The projection output itself (not a view of it) is modified, so autograd needs no CopySlices copy."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, heads, head_dim, pos0):
        ctx.mark_dirty(qkv)
        B, S = qkv.shape[0], qkv.shape[1]
        x4 = qkv.view(B, S, -1, head_dim)
        _launch(x4, x4, cos, sin, pos0, backward=False, heads=heads)
        ctx.save_for_backward(cos, sin)
        ctx.heads, ctx.pos0, ctx.head_dim = heads, pos0, head_dim
        return qkv

    @staticmethod
    def backward(ctx, dqkv):
        from .attention import take_fresh_grad
        cos, sin = ctx.saved_tensors
        # In place only on a buffer the packed attention backward allocated for this node alone; any other
        # gradient (accumulated from several consumers, or a buffer shared with another node) gets a copy.
        if not (dqkv.is_contiguous() and take_fresh_grad(dqkv)):
            dqkv = dqkv.clone(memory_format=torch.contiguous_format)
        B, S = dqkv.shape[0], dqkv.shape[1]
        d4 = dqkv.view(B, S, -1, ctx.head_dim)
        _launch(d4, d4, cos, sin, ctx.pos0, backward=True, heads=ctx.heads)
        return dqkv, None, None, None, None, None


def apply_rope_qk_(qkv, n_q_heads: int, n_kv_heads: int, head_dim: int, cos, sin, pos0: int = 0):
    """In place: rotate the q and k heads (the first ``n_q_heads + n_kv_heads`` of ``head_dim`` each) of the
    packed projection ``qkv`` [B, S, (Hq + 2 Hkv) * head_dim]; returns it (CPU: a rotated copy)."""
    D = head_dim
    heads = n_q_heads + n_kv_heads
    if not qkv.is_cuda or (D // 2) % 8 != 0 or qkv.dtype not in (torch.float32, torch.bfloat16) or \
            not qkv.is_contiguous():
        B, S = qkv.shape[0], qkv.shape[1]
        x4 = qkv.reshape(B, S, -1, D)
        qk = _rope_ref(x4[:, :, :heads], cos, sin, pos0, 1.0)
        return torch.cat([qk, x4[:, :, heads:]], dim=2).reshape(qkv.shape)
    cos, sin = _tables_f32(cos, sin)
    if cos.shape[0] < pos0 + qkv.shape[1] or cos.shape[1] != D // 2:
        raise ValueError("apply_rope_qk_: tables do not cover the sequence / head_dim")
    return _RopeQKInplaceFn.apply(qkv, cos, sin, heads, D, pos0)
