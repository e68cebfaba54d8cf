"""Hand MFMA GEMMs with fused epilogues (``csrc/kernels/gemm.hip``).

* ``gemm_nt(a, b)``            a [M, K] @ b [N, K]^T  (Linear forward; dgrad against a transposed weight)
* ``gemm_nt(..., bias=)``      + bias
* ``gemm_nt_gelu(a, b, bias)`` -> (gelu_tanh(h), gelu_tanh'(h)) with h = a b^T + bias: GPT-2's c_fc in ONE
  pass; the backward keeps the derivative, not the pre-activation
* ``gemm_nt_dgelu(a, b, d)`` -> (g = (a b^T) * d, colsum(g)): c_proj's dgrad, the GELU backward (d is the
  derivative ``gemm_nt_gelu`` kept: a multiply, no transcendental in the epilogue) and c_fc's bias gradient in
  ONE pass
* ``gemm_tt(a, b)``            a [K, M]^T @ b [K, N]  (weight gradient dY^T X), optional token split

hipBLASLt has no gfx950 kernel for the GELU_AUX_BIAS / DGELU_BGRAD epilogues
(profiles/r2_hipblaslt_epilogue_probe.txt), so without these the bias + GELU work is two extra HBM passes
over the [tokens, 4d] hidden per layer ("fuse into a GEMM epilogue").
Shapes: M, N multiples of 256, K a multiple of 32 (``gemm_ok``); callers fall back to library GEMMs
otherwise.
"""
from __future__ import annotations

import os

import torch

from . import _lib

L_NT, L_TT = 0, 1
E_PLAIN, E_BIAS, E_GELU, E_DGELU = 0, 1, 2, 3


def gemm_ok(layout: int, m: int, n: int, k: int, lda: int, ldb: int, splits: int = 1) -> bool:
    return bool(_lib.require().pdt_gemm_ok(layout, m, n, k, lda, ldb, splits))


def _bf16_2d(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1 and t.data_ptr() % 16 == 0


def nt_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (_bf16_2d(a) and _bf16_2d(b) and a.shape[1] == b.shape[1]
            and gemm_ok(L_NT, a.shape[0], b.shape[0], a.shape[1], a.stride(0), b.stride(0)))


def tt_ok(a: torch.Tensor, b: torch.Tensor, splits: int = 1) -> bool:
    return (_bf16_2d(a) and _bf16_2d(b) and a.shape[0] == b.shape[0]
            and gemm_ok(L_TT, a.shape[1], b.shape[1], a.shape[0], a.stride(0), b.stride(0), splits))


# kernel generation: "asm" = the hand-scheduled main loop (gemm_asm_kernel, round 4), "hip" = the
# compiler-scheduled one (gemm_kernel, round 3)
KERNEL = {"name": os.environ.get("PDT_GEMM_KERNEL", "asm")}


def _launch(layout, epi, a, b, c, m, n, k, bias=None, aux=None, aux_out=None, dbias=None, ws=None, splits=1):
    # the hand-scheduled loop needs >= 2 K-steps per split and 16-byte epilogue rows; the compiler-scheduled
    # kernel takes the rest (same results: the MFMA order per accumulator is identical)
    asm = KERNEL["name"] == "asm" and k // splits >= 128 and c.stride(0) % 8 == 0
    fn = "pdt_gemm2_bf16" if asm else "pdt_gemm_bf16"
    _lib.call(fn, layout, epi, a.data_ptr(), b.data_ptr(), c.data_ptr(), m, n, k, a.stride(0),
              b.stride(0), c.stride(0), _lib.ptr(bias), _lib.ptr(aux), _lib.ptr(aux_out), _lib.ptr(dbias),
              _lib.ptr(ws), splits, _lib.stream_handle(a.device))


def gemm_nt(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """a [M, K] @ b[N, K]^T (+ bias[N]) -> bf16 [M, N]."""
    m, k = a.shape
    n = b.shape[0]
    c = torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    _launch(L_NT, E_BIAS if bias is not None else E_PLAIN, a, b, c, m, n, k, bias=bias)
    return c


def gemm_nt_gelu(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor):
    """(gelu_tanh(h), gelu_tanh'(h)) with h = bf16(a b^T + bias) -- both bf16 [M, N].  Value and derivative are
    taken of the ROUNDED pre-activation (what an unfused bf16 Linear + GELU differentiates); the derivative is
    what the backward needs (``gemm_nt_dgelu`` / the ``pdt_bias_gelu_bwd_db`` sweep in mode 2)."""
    m, k = a.shape
    n = b.shape[0]
    y = torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    d = torch.empty_like(y)
    _launch(L_NT, E_GELU, a, b, y, m, n, k, bias=bias, aux_out=d)
    return y, d


def gemm_nt_dgelu(a: torch.Tensor, b: torch.Tensor, d: torch.Tensor, bias_dtype=torch.bfloat16):
    """(g, db): g = (a b^T) * d bf16 [M, N] (d = the GELU derivative ``gemm_nt_gelu`` returned), db = g.sum(0)
    (fp32 partial per 256-row tile, reduced in a fixed two-level order)."""
    m, k = a.shape
    n = b.shape[0]
    g = torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    db = torch.empty(n, dtype=torch.bfloat16, device=a.device)
    ws = torch.empty((m // 256 + 64) * n, dtype=torch.float32, device=a.device)   # partials + 2nd reduce level
    _launch(L_NT, E_DGELU, a, b, g, m, n, k, aux=d, dbias=db, ws=ws)
    return g, db.to(bias_dtype)


def tt_splits(m: int, n: int, k: int, cus: int = 256) -> int:
    """Token split (1, 2, 4, 8, 16) whose tiles x slices fill whole waves of the CUs best (>= 4096 tokens
    per slice); outputs of at least one wave of tiles are not split (the fp32 slab pass costs more)."""
    tiles = (m // 256) * (n // 256)
    if tiles == 0:
        return 1
    if tiles >= cus:
        # a full wave already; split only to rescue a badly quantised last wave (GPT-2's LM-head weight gradient:
        # 1,568 tiles = 6.125 waves of 256 CUs run as 7; 2 slices = 12.25 -> 13 rounds, 4 slices 24.5 -> 25:
        # 87.5 / 94 / 98 % of the rounds busy, measured 16.2 / 15.3 / 14.8 ms, r4_lm_head_wgrad_ab.jsonl)
        eff1 = tiles / (-(-tiles // cus) * cus)
        best, best_eff = 1, eff1
        if eff1 < 0.9:
            for s in (2, 4):
                if k % (32 * s) or k // s < 4096:
                    break
                eff = s * tiles / (-(-(s * tiles) // cus) * cus)
                if eff > best_eff + 0.03:
                    best, best_eff = s, eff
        return best if best_eff > eff1 + 0.05 else 1
    best, best_eff = 1, 0.0
    for s in (1, 2, 4, 8, 16):
        if s > 1 and (k % (32 * s) or k // s < 4096):
            break
        wgs = tiles * s
        eff = wgs / (-(-wgs // cus) * cus)
        if eff > best_eff + 1e-9:
            best, best_eff = s, eff
    return best


def gemm_tt(a: torch.Tensor, b: torch.Tensor, splits: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """a[K, M]^T @ b[K, N] -> bf16 [M, N] (dW = dY^T X with a = dY, b = X); ``out``: a contiguous bf16 [M, N]
    to write into (e.g. the leading rows of a larger weight gradient)."""
    k, m = a.shape
    n = b.shape[1]
    s = splits or tt_splits(m, n, k)
    if out is not None:
        assert out.shape == (m, n) and out.dtype == torch.bfloat16 and out.is_contiguous()
    c = out if out is not None else torch.empty(m, n, dtype=torch.bfloat16, device=a.device)
    ws = torch.empty(s * m * n, dtype=torch.float32, device=a.device) if s > 1 else None
    _launch(L_TT, E_PLAIN, a, b, c, m, n, k, ws=ws, splits=s)
    return c
