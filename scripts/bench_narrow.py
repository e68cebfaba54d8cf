#!/usr/bin/env python
"""Narrow linears at SwinIR-S Stoke shapes (294,912 tokens): the HIP narrow-GEMM kernel (ops.narrow) against the
library path ops.linear would otherwise take (F.linear forward; torch.mm + column sum for the data gradient)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributedtraining_amd.ops.activations import _colsum  # noqa: E402
from pytorch_distributedtraining_amd.ops.linear import _library_wgrad  # noqa: E402
from pytorch_distributedtraining_amd.ops.narrow import narrow_linear, narrow_wgrad  # noqa: E402


def t_ms(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


dev = torch.device("cuda")
M = 294912
for name, K, N, bias, role in [("qkv fwd", 60, 180, True, "fwd"), ("proj fwd", 60, 60, True, "fwd"),
                               ("qkv dgrad+db", 180, 60, False, "dgrad"), ("proj dgrad+db", 60, 60, False, "dgrad")]:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
    b = torch.randn(N, device=dev).bfloat16() if bias else None
    if role == "fwd":
        tn = t_ms(lambda: narrow_linear(x, w, b))
        tl = t_ms(lambda: F.linear(x, w, b))
    else:
        # x = dY [M, K], w = W^T [N, K] (the Linear's weight transposed): dX = dY W, and db = colsum(dY)
        tn = t_ms(lambda: narrow_linear(x, w, None, torch.bfloat16))
        wl = w.t().contiguous()
        tl = t_ms(lambda: (torch.mm(x, wl), _colsum(x, torch.bfloat16)))
    gb = (M * K + M * N) * 2 / 1e9
    extra = {}
    if role == "fwd" and N % 10 == 0:      # head-major output (Swin's qkv: 64-token windows, d = 10)
        extra["narrow_head_major_us"] = round(1000 * t_ms(lambda: narrow_linear(x, w, b, hm=(64, 10))), 1)
    if role == "dgrad":                    # without the fused column sum
        extra["narrow_no_colsum_us"] = round(1000 * t_ms(lambda: narrow_linear(x, w, None)), 1)
    print(json.dumps({"op": name, "M": M, "K": K, "N": N, "narrow_us": round(1000 * tn, 1),
                      "library_us": round(1000 * tl, 1), "narrow_TBps": round(gb / tn, 2),
                      "speedup": round(tl / tn, 2), **extra}), flush=True)
for name, N, K in [("qkv wgrad", 180, 60), ("proj wgrad", 60, 60)]:
    dy = torch.randn(M, N, device=dev).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    tn = t_ms(lambda: narrow_wgrad(dy, x, torch.bfloat16))
    tl = t_ms(lambda: _library_wgrad(dy, x, torch.bfloat16))
    gb = (M * K + M * N) * 2 / 1e9
    print(json.dumps({"op": name, "M": M, "K": K, "N": N, "narrow_us": round(1000 * tn, 1),
                      "library_us": round(1000 * tl, 1), "narrow_TBps": round(gb / tn, 2),
                      "speedup": round(tl / tn, 2)}), flush=True)
