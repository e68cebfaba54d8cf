"""hipBLASLt GEMMs with fused epilogues, called directly (csrc/kernels/blaslt.hip): per-shape plans, the
fastest of hipBLASLt's heuristic candidates picked by timing on a shape's first uncaptured call.

Used for the Linear weight gradient with the bias gradient reduced inside the same GEMM (epilogue BGRADB):
dW = dY^T X and db = colsum(dY) read dY once instead of twice, and the separate column-sum launches
(2 per biased Linear per step) disappear.  The probe in scripts/bench_lt_epilogues.py
(profiles/r2_hipblaslt_epilogue_probe.txt) shows which epilogues this hipBLASLt build has gfx950 algorithms
for: BIAS, GELU_BIAS and BGRADB (with B transposed) yes; GELU_AUX_BIAS, DGELU and DGELU_BGRAD no -- so the
GELU stays in the framework's own bias-GELU kernels.
"""
from __future__ import annotations

import torch

from . import _lib

EPI_NONE, EPI_BIAS, EPI_BGRADB = 0, 1, 6
_UNSUPPORTED: set = set()
TUNE = True


def lt_matmul(epi: int, trans: int, m: int, n: int, k: int, a, b, d, bias=None) -> bool:
    """Column-major D[m, n] = op(A) op(B) (trans bit 0: A^T, bit 1: B^T) with an epilogue; False if hipBLASLt
    has no algorithm for the combination (cached; the caller falls back)."""
    key = (epi, trans, m, n, k, d.dtype, None if bias is None else bias.dtype)
    if key in _UNSUPPORTED:
        return False
    rc = _lib.require().pdt_lt_matmul(epi, trans, m, n, k, a.data_ptr(), b.data_ptr(), d.data_ptr(), _lib.ptr(bias),
                                      _lib.dtype_code(bias.dtype) if bias is not None else 0, 0,
                                      _lib.dtype_code(d.dtype), 1 if TUNE else 0, _lib.stream_handle(d.device))
    if rc == -3:
        _UNSUPPORTED.add(key)
        return False
    _lib.check(rc, "pdt_lt_matmul")
    return True


def linear_residual(a2: torch.Tensor, w: torch.Tensor, bias, r2: torch.Tensor):
    """a2 [M, K] @ w[N, K]^T (+ bias) + r2 [M, N] in ONE hipBLASLt GEMM (the residual read in its epilogue, beta =
    1) into a new tensor, or None (no algorithm).  Column-major: D[N, M] = W^T(op T on col-major [K, N]) . A."""
    m, k = a2.shape
    n = w.shape[0]
    d = torch.empty(m, n, dtype=a2.dtype, device=a2.device)
    epi = EPI_BIAS if bias is not None else EPI_NONE
    key = ("c", epi, m, n, k, d.dtype, None if bias is None else bias.dtype)
    if key in _UNSUPPORTED:
        return None
    rc = _lib.require().pdt_lt_matmul_c(epi, 1, n, m, k, w.data_ptr(), a2.data_ptr(), r2.data_ptr(), d.data_ptr(),
                                        _lib.ptr(bias), _lib.dtype_code(bias.dtype) if bias is not None else 0,
                                        _lib.dtype_code(d.dtype), 1 if TUNE else 0, _lib.stream_handle(d.device))
    if rc == -3:
        _UNSUPPORTED.add(key)
        return None
    _lib.check(rc, "pdt_lt_matmul_c")
    return d


def wgrad_bgrad(dy2: torch.Tensor, x2: torch.Tensor):
    """(dW [N, K], db [N]) = (dY^T X, colsum dY) for contiguous bf16 dY [M, N], X [M, K] in ONE GEMM, or None."""
    m_rows, n = dy2.shape
    k = x2.shape[1]
    dw = torch.empty(n, k, dtype=dy2.dtype, device=dy2.device)
    db = torch.empty(n, dtype=dy2.dtype, device=dy2.device)
    # column-major: dW^T[K, N] = X^T(op N on col-major [K, M]) . dY(col-major [N, M], op T)
    if not lt_matmul(EPI_BGRADB, 2, k, n, m_rows, x2, dy2, dw, db):
        return None
    return dw, db


_CHOICE: dict = {}


def prefer_bgradb(dy2: torch.Tensor, x2: torch.Tensor, separate) -> bool:
    """Whether the one-GEMM BGRADB path beats ``separate()`` (GEMM + column-sum) for this shape -- timed once per
    shape on its first uncaptured call.  hipBLASLt's BGRADB kernels are 1.6x faster than the pair on GPT-2 124M's
    qkv gradient (32k x 2304 x 768) but 7-9x SLOWER on GPT-2 1.3B's qkv / fc2 (profiles/r2_bgradb_vs_separate.jsonl),
    so the choice must be measured, not assumed."""
    key = (dy2.shape, x2.shape[1], dy2.dtype, dy2.device)
    c = _CHOICE.get(key)
    if c is not None:
        return c
    if torch.cuda.is_current_stream_capturing():
        return False
    if wgrad_bgrad(dy2, x2) is None:
        _CHOICE[key] = False
        return False

    from .picks import timed_choice
    c = _CHOICE[key] = timed_choice(lambda: wgrad_bgrad(dy2, x2), separate, table=_CHOICE, key=key, name="bgradb")
    return c
