"""Fused shifted-window attention for SwinIR / Swin blocks.

``window_attention(qkv, rel_bias, mask, num_heads, scale)`` computes, for every window and head,
``softmax(q kᵀ · scale + rel_bias[h] + mask[w]) v`` straight from the fused qkv projection
``[Bw, N, 3C]`` and returns ``[Bw, N, C]`` ready for the output projection.  On MI355X this is one
HIP kernel each way (``csrc/kernels/window_attn.hip``); the stock path would materialise the
expanded bias+mask ``[Bw, h, N, N]`` and the scores in HBM.  bf16 runs the bf16 MFMA kernels; fp32 (the reference's
own training precision) runs exact-f32 MFMA kernels (``v_mfma_f32_32x32x2_f32``), not a reduced-precision cast.  The CPU path is the plain PyTorch
formula (also the numerics reference in the GPU tests).
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.nn.functional as F

from . import _lib

_MASK_T_CACHE: dict = {}
USE_LABELS = os.environ.get("PDT_WIN_MASK_LABELS", "1") == "1"   # A/B switch: 0 = dense fp32 mask reads
MFMA_F32 = os.environ.get("PDT_WIN_F32_MFMA", "1") == "1"        # A/B switch: 0 = fp32 on the VALU kernels
# PDT_WIN_HEAD_MAJOR=0: the MFMA kernels read q / k / v / dO token-major in place (A/B of the head-major relayout)
HEAD_MAJOR = os.environ.get("PDT_WIN_HEAD_MAJOR", "1") == "1"


def _hm_ok(qkv, N, num_heads, d) -> bool:
    es = qkv.element_size()
    return (HEAD_MAJOR and d % 2 == 0 and (N * 3 * num_heads * d * es) % 16 == 0
            and N * 3 * num_heads * d * es <= 96 * 1024 and qkv.data_ptr() % 16 == 0)


def _mask_t(mask):
    """[nw, N(i), N(j)] -> [nw, N(j), N(i)] fp32, cached per (storage, version) -- masks are buffers."""
    key = (mask.data_ptr(), mask._version, tuple(mask.shape), mask.device)
    ent = _MASK_T_CACHE.get(key)
    if ent is None or ent[0]() is not mask:
        if len(_MASK_T_CACHE) > 64:
            _MASK_T_CACHE.clear()
        m = mask.float().contiguous()
        ent = (weakref.ref(mask), (m, m.transpose(1, 2).contiguous()))
        _MASK_T_CACHE[key] = ent
    return ent[1]


_LABEL_CACHE: dict = {}


def _mask_labels(mask):
    """Swin shift masks are -100 exactly where a query's and a key's image regions differ: return per-window
    region labels [nw, N] uint8 (label = first key of the token's region) when ``mask`` has that form, else None.
    The MFMA kernels then rebuild the mask from 64 label bytes per window instead of reading the fp32 mask.
    Derived once per mask buffer (one host check, in the first -- eager -- call)."""
    # keyed by address + version, and the entry holds a weak reference to the mask it was derived from: a new
    # mask allocated at a freed mask's address (same shape, version 0) is a miss, not stale labels
    key = (mask.data_ptr(), mask._version, tuple(mask.shape), mask.device)
    ent = _LABEL_CACHE.get(key)
    if ent is not None and ent[0]() is mask:
        return ent[1]
    if len(_LABEL_CACHE) > 64:
        _LABEL_CACHE.clear()
    m = mask.float()
    lab = (m == 0).float().argmax(-1)                                      # [nw, N]
    rebuilt = torch.where(lab[:, :, None] != lab[:, None, :], -100.0, 0.0)
    out = lab.to(torch.uint8).contiguous() if (mask.shape[-1] <= 64 and torch.equal(rebuilt, m)) else None
    _LABEL_CACHE[key] = (weakref.ref(mask), out)
    return out


def reference(qkv, rel_bias, mask, num_heads, scale):
    Bw, N, C3 = qkv.shape
    C = C3 // 3
    q, k, v = qkv.float().view(Bw, N, 3, num_heads, C // num_heads).permute(2, 0, 3, 1, 4)
    s = (q * scale) @ k.transpose(-1, -2) + rel_bias.float().unsqueeze(0)
    if mask is not None:
        nw = mask.shape[0]
        s = s.view(Bw // nw, nw, num_heads, N, N) + mask.float().view(1, nw, 1, N, N)
        s = s.view(Bw, num_heads, N, N)
    o = s.softmax(-1) @ v
    return o.transpose(1, 2).reshape(Bw, N, C).to(qkv.dtype)


class _WindowAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, rel_bias, mask, num_heads, scale, out_head_major=False):
        Bw, N, C3 = qkv.shape
        C = C3 // 3
        d = C // num_heads
        tag = getattr(qkv, "_pdt_head_major", None)
        qkv = qkv.contiguous()
        bias = rel_bias.float().contiguous()
        nw = mask.shape[0] if mask is not None else 1
        o = torch.empty((Bw, N, C), dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty((Bw, num_heads, N), dtype=torch.float32, device=qkv.device)
        lib = _lib.require()
        if qkv.dtype == torch.float32:
            # fp32 (the reference's precision): exact-f32 MFMA kernels (v_mfma_f32_32x32x2_f32), VALU as fallback
            ctx.mfma = "f32" if (MFMA_F32 and lib.pdt_win_attn_mfma32_ok(N, num_heads, d)) else None
        else:
            ctx.mfma = "bf16" if lib.pdt_win_attn_mfma_ok(N, num_heads, d, _lib.dtype_code(qkv.dtype)) else None
        if ctx.mfma:
            # MFMA kernels: dense bias [h, N(q), N(key)] and mask [nw, N, N], no transposed copies
            m = mask.float().contiguous() if mask is not None else None
            lab = _mask_labels(mask) if (mask is not None and USE_LABELS) else None
            st = _lib.stream_handle(qkv.device)
            # qkv already head-major (ops.linear.linear_head_major: the narrow GEMM wrote [Bw, 3, h, N, d]): every
            # staging load reads contiguous token slices.  Otherwise the forward writes a head-major copy of q / k / v
            # from the slices it stages anyway, for the backward's staging loads (kept in place of qkv, same size).
            given = tag is not None
            if given and tag != (N, d):
                raise RuntimeError(f"window_attention: head-major qkv tagged {tag}, expected {(N, d)}")
            ctx.hm = given or _hm_ok(qkv, N, num_heads, d)
            hm = torch.empty_like(qkv) if (ctx.hm and not given) else None
            # O head-major ([Bw, h, N, d]) for a projection that reads it so (ops.linear.linear_from_head_major); the
            # backward then needs the precomputed-delta path (ctx.hm)
            ctx.o_hm = bool(out_head_major) and ctx.hm and ctx.mfma == "bf16"
            _lib.call("pdt_win_attn_mfma_fwd" if ctx.mfma == "bf16" else "pdt_win_attn_mfma32_fwd", qkv.data_ptr(),
                      bias.data_ptr(), _lib.ptr(m), _lib.ptr(lab), nw,
                      o.data_ptr(), lse.data_ptr(), Bw, N, num_heads, d, float(scale), _lib.ptr(hm), int(given),
                      int(ctx.o_hm), st)
            ctx.save_for_backward(hm if hm is not None else qkv, bias, o, lse)
            ctx.mask = (m, lab, nw)
            ctx.h, ctx.scale, ctx.bias_dtype = num_heads, scale, rel_bias.dtype
            if ctx.o_hm:
                o._pdt_head_major = (N, d)
            return o
        if tag is not None:
            raise RuntimeError("window_attention: a head-major qkv (linear_head_major) needs the MFMA kernels")
        ctx.o_hm = False
        bias_t = bias.transpose(1, 2).contiguous()
        m, m_t = _mask_t(mask) if mask is not None else (None, None)
        _lib.call("pdt_win_attn_fwd", qkv.data_ptr(), bias_t.data_ptr(), _lib.ptr(m_t), nw, o.data_ptr(),
                  lse.data_ptr(), Bw, N, num_heads, d, float(scale), _lib.dtype_code(qkv.dtype),
                  _lib.stream_handle(qkv.device))
        ctx.save_for_backward(qkv, bias, bias_t, o, lse)
        ctx.mask = (m, m_t, nw)
        ctx.h, ctx.scale, ctx.bias_dtype = num_heads, scale, rel_bias.dtype
        return o

    @staticmethod
    def backward(ctx, do):
        dqkv, part = _WindowAttnFn._backward_parts(ctx, do)
        return dqkv, part.sum(0).to(ctx.bias_dtype), None, None, None, None

    @staticmethod
    def _backward_parts(ctx, do):
        """(dqkv, per-workgroup bias-gradient partials [G, h, N, N] fp32)."""
        if ctx.mfma:
            qkv, bias, o, lse = ctx.saved_tensors
            m, lab, nw = ctx.mask
            Bw, N, C3 = qkv.shape
            d = C3 // 3 // ctx.h
            G = _lib.require().pdt_win_attn_mfma_grid(Bw, ctx.h)
            dqkv = torch.empty_like(qkv)        # token-major (the projection's layout), also when qkv is head-major
            part = torch.empty((G, ctx.h, N, N), dtype=torch.float32, device=qkv.device)
            # dO head-major already when the projection's data gradient wrote it so (linear_from_head_major)
            g_hm = getattr(do, "_pdt_head_major", None) == (N, d)
            do = do.contiguous().to(qkv.dtype)
            st = _lib.stream_handle(qkv.device)
            delta = None
            if ctx.hm and do.data_ptr() % 16:
                do = do.clone()
            if g_hm and not ctx.hm:
                raise RuntimeError("window_attention: head-major dO needs the head-major backward")
            if ctx.hm:
                # dO head-major + delta = rowsum(dO o O) from one coalesced pass: the kernels stage neither O nor
                # token-major dO slices
                g = do if g_hm else torch.empty_like(do)
                delta = torch.empty((Bw, ctx.h, N), dtype=torch.float32, device=qkv.device)
                _lib.call("pdt_win_bwd_prep", do.data_ptr(), o.data_ptr(), None if g_hm else g.data_ptr(),
                          delta.data_ptr(), Bw, N, ctx.h, d, _lib.dtype_code(qkv.dtype), int(g_hm), int(ctx.o_hm), st)
                do = g
            _lib.call("pdt_win_attn_mfma_bwd" if ctx.mfma == "bf16" else "pdt_win_attn_mfma32_bwd", qkv.data_ptr(),
                      bias.data_ptr(), _lib.ptr(m), _lib.ptr(lab), nw, o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                      dqkv.data_ptr(), part.data_ptr(), Bw, N, ctx.h, d, float(ctx.scale), int(ctx.hm),
                      _lib.ptr(delta), st)
            return dqkv, part
        qkv, bias, bias_t, o, lse = ctx.saved_tensors
        m, m_t, nw = ctx.mask
        Bw, N, C3 = qkv.shape
        d = C3 // 3 // ctx.h
        lib = _lib.require()
        G = lib.pdt_win_attn_grid(Bw)
        dqkv = torch.empty_like(qkv)
        part = torch.empty((G, ctx.h, N, N), dtype=torch.float32, device=qkv.device)
        do = do.contiguous().to(qkv.dtype)
        _lib.call("pdt_win_attn_bwd", qkv.data_ptr(), bias.data_ptr(), bias_t.data_ptr(), _lib.ptr(m), _lib.ptr(m_t),
                  nw, o.data_ptr(), do.data_ptr(), lse.data_ptr(), dqkv.data_ptr(), part.data_ptr(), Bw, N, ctx.h,
                  d, float(ctx.scale), _lib.dtype_code(qkv.dtype), _lib.stream_handle(qkv.device))
        return dqkv, part


_CSR_CACHE: dict = {}


def _rel_csr(index, rows: int):
    """(idx int32 [N*N], off int32 [rows + 1], pos int32 [N*N]) for a relative-position index buffer: the entries
    that read each table row, in ascending order -- built once per index buffer (host, first call)."""
    key = (index.data_ptr(), index._version, tuple(index.shape), index.device, rows)
    ent = _CSR_CACHE.get(key)
    if ent is not None and ent[0]() is index:
        return ent[1]
    if len(_CSR_CACHE) > 64:
        _CSR_CACHE.clear()
    flat = index.reshape(-1).to(torch.int64).cpu()
    order = torch.argsort(flat, stable=True)
    counts = torch.bincount(flat, minlength=rows)
    off = torch.zeros(rows + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(counts, 0)
    dev = index.device
    out = (flat.to(torch.int32).to(dev), off.to(torch.int32).to(dev), order.to(torch.int32).to(dev))
    _CSR_CACHE[key] = (weakref.ref(index), out)
    return out


class _WindowAttnTableFn(torch.autograd.Function):
    """window_attention with the bias given as the Swin table [T, h] + index [N, N]: the dense fp32 bias is
    gathered by one kernel, and the backward turns the attention kernel's bias-gradient partials straight into
    the table gradient (csrc/kernels/rel_bias.hip) -- instead of index_select / permute / cast forward and
    sum / cast / zero-fill / index_add backward per block."""

    @staticmethod
    def forward(ctx, qkv, table, index, mask, num_heads, scale, out_head_major=False):
        N = qkv.shape[1]
        idx, off, pos = _rel_csr(index, table.shape[0])
        tab = table.contiguous()
        bias = torch.empty((num_heads, N, N), dtype=torch.float32, device=qkv.device)
        _lib.call("pdt_rel_bias_gather", tab.data_ptr(), idx.data_ptr(), bias.data_ptr(), num_heads, N * N,
                  _lib.dtype_code(tab.dtype), _lib.stream_handle(qkv.device))
        o = _WindowAttnFn.forward(ctx, qkv, bias, mask, num_heads, scale, out_head_major)
        ctx.table_meta = (table.shape[0], table.dtype, off, pos)
        return o

    @staticmethod
    def backward(ctx, do):
        rows, dt, off, pos = ctx.table_meta
        dqkv, part = _WindowAttnFn._backward_parts(ctx, do)
        G, h, N, _ = part.shape
        dtab = torch.empty((rows, h), dtype=dt, device=part.device)
        ws = torch.empty(h * N * N, dtype=torch.float32, device=part.device)
        _lib.call("pdt_rel_bias_scatter", part.data_ptr(), G, h, N * N, off.data_ptr(), pos.data_ptr(), rows,
                  dtab.data_ptr(), _lib.dtype_code(dt), ws.data_ptr(), _lib.stream_handle(part.device))
        return dqkv, dtab, None, None, None, None, None


def window_attention_table(qkv, table, index, mask, num_heads: int, scale: float, out_head_major: bool = False):
    """window_attention with rel_bias = table[index].permute(2, 0, 1) (Swin's relative-position table [T, h] and
    index buffer [N, N]), the gather and its backward fused into two small kernels on the GPU."""
    if (supported(qkv, num_heads) and table.dtype in (torch.float32, torch.bfloat16) and table.dim() == 2
            and table.shape[1] == num_heads and index.numel() == qkv.shape[1] ** 2):
        return _WindowAttnTableFn.apply(qkv, table, index, mask, num_heads, scale, out_head_major)
    N = qkv.shape[1]
    rel = table[index.reshape(-1)].view(N, N, num_heads).permute(2, 0, 1)
    return window_attention(qkv, rel, mask, num_heads, scale, out_head_major)


def head_major_ok(x, N: int, num_heads: int, d: int) -> bool:
    """Whether window_attention would run the MFMA kernels on a qkv of x's device / dtype (the only consumer that
    reads a head-major qkv, ops.linear.linear_head_major)."""
    if not (HEAD_MAJOR and x.is_cuda and _lib.available()):
        return False
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    lib = _lib.require()
    if dt == torch.bfloat16:
        return bool(lib.pdt_win_attn_mfma_ok(N, num_heads, d, _lib.dtype_code(dt)))
    return dt == torch.float32 and MFMA_F32 and bool(lib.pdt_win_attn_mfma32_ok(N, num_heads, d))


def supported(qkv, num_heads) -> bool:
    Bw, N, C3 = qkv.shape
    d = C3 // 3 // num_heads
    return (qkv.is_cuda and qkv.dtype in (torch.float32, torch.bfloat16) and N <= 64 and d <= 32
            and num_heads <= 16 and _lib.available())


def window_attention(qkv, rel_bias, mask, num_heads: int, scale: float, out_head_major: bool = False):
    """qkv [Bw, N, 3C]; rel_bias [h, N, N]; mask [nw, N, N] or None (window b uses mask b % nw).
    ``out_head_major``: the output MAY come back head-major ([Bw, h, N, d] in the [Bw, N, C] buffer), tagged
    ``_pdt_head_major`` -- only for a consumer that checks the tag (ops.linear.linear_from_head_major)."""
    if supported(qkv, num_heads):
        return _WindowAttnFn.apply(qkv, rel_bias, mask, num_heads, scale, out_head_major)
    if getattr(qkv, "_pdt_head_major", None) is not None:
        raise RuntimeError("window_attention: a head-major qkv (linear_head_major) needs the GPU kernels")
    if qkv.is_cuda:
        _lib.require()          # fail loudly on a GPU box without the kernels
    return reference(qkv, rel_bias, mask, num_heads, scale)


# ------------------------------------------------------------------------------------------------
# Fused shifted-window partition / reverse (+ residual): one row-permutation pass each way
# (csrc/kernels/conv.hip window_perm_kernel).
# ------------------------------------------------------------------------------------------------
def _perm(src, res, out_shape, H, W, ws, shift, reverse):
    C = src.shape[-1]
    if src.dtype not in (torch.bfloat16, torch.float32) or (res is not None and res.dtype != src.dtype):
        raise TypeError("fused window permutation takes bf16 or fp32 tensors of one dtype")
    out = torch.empty(out_shape, dtype=src.dtype, device=src.device)
    rows = src.numel() // C
    _lib.call("pdt_window_perm" if src.dtype == torch.bfloat16 else "pdt_window_perm_f32", src.data_ptr(), _lib.ptr(res), out.data_ptr(), rows, C, H, W, ws, shift,
              1 if reverse else 0, _lib.stream_handle(src.device))
    return out


class _PartitionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, H, W, ws, shift):
        B, L, C = x.shape
        ctx.geom = (B, H, W, ws, shift)
        return _perm(x.contiguous(), None, (B * (H // ws) * (W // ws), ws * ws, C), H, W, ws, shift, False)

    @staticmethod
    def backward(ctx, g):
        B, H, W, ws, shift = ctx.geom
        return _perm(g.contiguous(), None, (B, H * W, g.shape[-1]), H, W, ws, shift, True), None, None, None, None


class _ReverseAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, win, res, H, W, ws, shift):
        ctx.geom = (H, W, ws, shift)
        return _perm(win.contiguous(), res.contiguous(), res.shape, H, W, ws, shift, True)

    @staticmethod
    def backward(ctx, g):
        H, W, ws, shift = ctx.geom
        g = g.contiguous()
        B, L, C = g.shape
        dwin = _perm(g, None, (B * (H // ws) * (W // ws), ws * ws, C), H, W, ws, shift, False)
        return dwin, g, None, None, None, None


def fused_window_ok(x, H, W, ws, shift) -> bool:
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 3 and x.shape[1] == H * W and
            x.shape[2] % 4 == 0 and H % ws == 0 and W % ws == 0 and 0 <= shift < ws)


def window_partition_shifted(x, H, W, ws, shift):
    """[B, H*W, C] -> windows [B*nW, ws*ws, C] of torch.roll(x, (-shift, -shift)) in ONE pass."""
    return _PartitionFn.apply(x, H, W, ws, shift)


def window_reverse_shifted_add(windows, res, H, W, ws, shift):
    """res + roll(window_reverse(windows), (shift, shift)) as [B, H*W, C] in ONE pass."""
    return _ReverseAddFn.apply(windows, res, H, W, ws, shift)
