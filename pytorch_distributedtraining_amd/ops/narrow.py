"""Narrow linears (in / out features <= 192, hundreds of thousands of rows) on ``csrc/kernels/narrow_gemm.hip``:
bf16 on 16x16x32 bf16 MFMAs, fp32 (the reference's precision) on exact-f32 16x16x4 MFMAs.

SwinIR-S at the reference's Stoke config runs its attention projections on 294,912 tokens x C = 60 (qkv 60 -> 180,
proj 60 -> 60; Stoke-DDP.py:206-208).  Those products are bandwidth-bound, and a library GEMM tiled for compute
pays a macro tile's prologue / epilogue for two K-steps of MFMA work.  The HIP kernel keeps the weight in VGPRs,
streams 16-row blocks through LDS and writes contiguous output blocks; its data-gradient use also returns the
column sums of dY (the bias gradient) from the same read.  ``ops.linear`` times it against the library path per
shape (``ops.picks``) and takes the faster.
"""
from __future__ import annotations

import torch

from . import _lib


def narrow_ok(x2: torch.Tensor, w: torch.Tensor, bias=None, transposed: bool = False) -> bool:
    """Whether x2 @ w.T (+ bias) -- or x2 @ w with ``transposed`` (a data gradient dY W) -- fits the kernel."""
    n_out, k_in = (w.shape[1], w.shape[0]) if transposed else (w.shape[0], w.shape[1])
    dt = x2.dtype
    if not (x2.is_cuda and dt in (torch.bfloat16, torch.float32) and w.dtype == dt and x2.dim() == 2
            and w.dim() == 2 and x2.is_contiguous() and w.is_contiguous() and x2.shape[1] == k_in
            and x2.data_ptr() % 16 == 0 and x2.shape[0] >= 16384 and _lib.available()):
        return False
    if bias is not None and (bias.dtype != dt or not bias.is_contiguous()):
        return False
    lib = _lib.require()
    ok = lib.pdt_narrow_gemm_ok if dt == torch.bfloat16 else lib.pdt_narrow_gemm_f32_ok
    return bool(ok(x2.shape[0], k_in, n_out))


def head_major_ok(M: int, N: int, hm) -> bool:
    """Whether a head-major output (hm = (tokens per window, head dim)) fits: see narrow_linear."""
    n_tok, d = hm
    return n_tok > 0 and n_tok % 16 == 0 and M % n_tok == 0 and 2 <= d <= 32 and d % 2 == 0 and N % d == 0


def narrow_linear(x2: torch.Tensor, w: torch.Tensor, bias=None, colsum_dtype: torch.dtype | None = None, hm=None,
                  a_hm=None, residual=None):
    """(x2 @ w.T + bias, colsum(x2) in ``colsum_dtype`` or None) -- x2 [M, K], w [N, K], K, N <= 192.
    ``hm = (n_tok, d)``: the output buffer [M, N] is filled HEAD-MAJOR -- rows m = window w x n_tok + token t,
    columns c = segment s x d + dim -> element ((w N + s d) n_tok + t d + dim), i.e. Swin's qkv as
    [windows, 3, heads, n_tok, d] for the window attention's staging loads (ops.window_attention).
    ``a_hm = (n_tok, d)`` (bf16): x2's buffer is read head-major the same way (the window attention's output).
    ``residual`` [M, N] (x2's dtype, contiguous, 16-byte aligned, token-major output only): added in the store."""
    M, K = x2.shape
    N = w.shape[0]
    hm_n, hm_d = hm if hm is not None else (0, 0)
    a_n, a_d = a_hm if a_hm is not None else (0, 0)
    if a_n and x2.dtype != torch.bfloat16:
        raise ValueError("narrow_linear: a head-major input is bf16 only")
    if residual is not None and (hm is not None or residual.dtype != x2.dtype or not residual.is_contiguous()
                                 or tuple(residual.shape) != (M, N) or residual.data_ptr() % 16):
        raise ValueError("narrow_linear: residual must be a contiguous, 16-byte aligned [M, N] of x2's dtype")
    if x2.dtype == torch.float32:      # exact-f32 MFMA kernels (v_mfma_f32_16x16x4_f32)
        lib = _lib.require()
        y = torch.empty((M, N), dtype=torch.float32, device=x2.device)
        cs = ws = None
        if colsum_dtype is not None:
            cs = torch.empty(K, dtype=torch.float32, device=x2.device)
            ws = torch.empty((lib.pdt_narrow_gemm_f32_partials(M) + 64) * K, dtype=torch.float32, device=x2.device)
        _lib.call("pdt_narrow_gemm_f32", x2.data_ptr(), w.data_ptr(), _lib.ptr(bias), y.data_ptr(), M, K, N,
                  _lib.ptr(cs), _lib.ptr(ws), hm_n, hm_d, _lib.ptr(residual), _lib.stream_handle(x2.device))
        return y, (cs.to(colsum_dtype) if cs is not None else None)
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x2.device)
    cs = ws = None
    if colsum_dtype is not None:
        lib = _lib.require()
        cs = torch.empty(K, dtype=colsum_dtype, device=x2.device)
        ws = torch.empty((lib.pdt_narrow_gemm_partials(M, K, N) + 64) * K, dtype=torch.float32, device=x2.device)
    _lib.call("pdt_narrow_gemm", x2.data_ptr(), w.data_ptr(), _lib.ptr(bias), y.data_ptr(), M, K, N, _lib.ptr(cs),
              _lib.dtype_code(colsum_dtype) if colsum_dtype is not None else 0, _lib.ptr(ws), hm_n, hm_d, a_n, a_d,
              _lib.ptr(residual), _lib.stream_handle(x2.device))
    return y, cs


def narrow_wgrad_ok(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype) -> bool:
    """dW = dy2^T x2 with both operands token-major bf16 and both feature counts narrow (<= 192)."""
    dt = dy2.dtype
    if not (dy2.is_cuda and dt in (torch.bfloat16, torch.float32) and x2.dtype == dt and dy2.dim() == 2
            and x2.dim() == 2 and dy2.shape[0] == x2.shape[0] and dy2.is_contiguous() and x2.is_contiguous()
            and dy2.data_ptr() % 16 == 0 and x2.data_ptr() % 16 == 0 and dy2.shape[0] >= 16384
            and out_dtype in (torch.float32, torch.bfloat16) and _lib.available()):
        return False
    lib = _lib.require()
    ok = lib.pdt_narrow_wgrad_ok if dt == torch.bfloat16 else lib.pdt_narrow_wgrad_f32_ok
    return bool(ok(dy2.shape[0], dy2.shape[1], x2.shape[1]))


def narrow_wgrad(dy2: torch.Tensor, x2: torch.Tensor, out_dtype: torch.dtype, x_hm_d: int = 0) -> torch.Tensor:
    """dW [N, K] = dy2[M, N]^T x2[M, K] on the narrow weight-gradient kernel (transposed LDS reads, one fp32
    partial per workgroup, fixed-order reduce).  ``x_hm_d`` (bf16): x2's buffer is head-major with 64-token windows
    ([M / 64, K / x_hm_d, 64, x_hm_d], the window attention's output)."""
    if x_hm_d and (dy2.dtype != torch.bfloat16 or dy2.shape[0] % 64):
        raise ValueError("narrow_wgrad: a head-major x is bf16 with 64-token windows only")
    M, N = dy2.shape
    K = x2.shape[1]
    lib = _lib.require()
    ws = torch.empty(lib.pdt_narrow_wgrad_ws_floats(M, N, K), dtype=torch.float32, device=dy2.device)
    if dy2.dtype == torch.float32:
        out = torch.empty((N, K), dtype=torch.float32, device=dy2.device)
        _lib.call("pdt_narrow_wgrad_f32", dy2.data_ptr(), x2.data_ptr(), out.data_ptr(), M, N, K, ws.data_ptr(),
                  _lib.stream_handle(dy2.device))
        return out.to(out_dtype)
    out = torch.empty((N, K), dtype=out_dtype, device=dy2.device)
    _lib.call("pdt_narrow_wgrad", dy2.data_ptr(), x2.data_ptr(), out.data_ptr(), M, N, K, _lib.dtype_code(out_dtype),
              ws.data_ptr(), int(x_hm_d), _lib.stream_handle(dy2.device))
    return out
