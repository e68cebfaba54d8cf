#!/usr/bin/env python
"""What does a residual read in the GEMM epilogue cost?  hipBLASLt D = A W^T (+ bias) against D = R + A W^T (beta = 1,
C = the residual stream), at GPT-2 1.3B's two residual-producing projections (attention c_proj 98,304 x 2,048 x
2,048; MLP c_proj 98,304 x 2,048 x 8,192), next to the fused residual-add + LayerNorm kernel the residual read
would shorten.  Median of interleaved rounds, one JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributedtraining_amd.ops.blaslt import linear_residual  # noqa: E402
from pytorch_distributedtraining_amd.ops.norms import add_norm, layer_norm  # noqa: E402

dev = torch.device("cuda")
T, C = 96 * 1024, 2048


def timeit(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


want = F.linear(a0 := torch.randn(4096, 2048, device=dev).bfloat16(), w0 := torch.randn(2048, 2048, device=dev).bfloat16() * 0.02,
                b0 := torch.randn(2048, device=dev).bfloat16()).float() + (r0 := torch.randn(4096, 2048, device=dev).bfloat16()).float()
got = linear_residual(a0, w0, b0, r0)
print(json.dumps({"check": "lt_bias_residual", "rel_err": float((got.float() - want).norm() / want.norm())}), flush=True)
for K in (2048, 8192):
    a = torch.randn(T, K, device=dev).bfloat16()
    w = (torch.randn(C, K, device=dev) * K ** -0.5).bfloat16()
    bias = torch.randn(C, device=dev).bfloat16()
    r = torch.randn(T, C, device=dev).bfloat16()
    g = torch.ones(C, device=dev).bfloat16()
    bb = torch.zeros(C, device=dev).bfloat16()
    arms = {"linear_bias": lambda: F.linear(a, w, bias),
            "addmm_residual": lambda: torch.addmm(r, a, w.t()),
            "lt_bias_residual": lambda: linear_residual(a, w, bias, r),
            "ln_plain": lambda: layer_norm(r, g, bb, 1e-5),
            "ln_residual_add": lambda: add_norm(r, r, g, bb, 1e-5, r_bias=bias)}
    res = {k: [] for k in arms}
    for _ in range(5):
        for k, fn in arms.items():
            res[k].append(timeit(fn))
    print(json.dumps({"shape": [T, C, K], **{k: round(sorted(v)[2] * 1e3, 1) for k, v in res.items()},
                      "unit": "us (median of 5 rounds)"}), flush=True)
