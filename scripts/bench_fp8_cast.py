#!/usr/bin/env python
"""fp8 cast / cast+transpose bandwidth at the GPT-2 1.3B MLP-hidden shape (65,536 x 8,192 bf16): row only,
transposed only, both, GELU-fused both; GB/s counts bytes read + written."""
import json

import torch

from pytorch_distributedtraining_amd.ops import fp8 as F8

dev = "cuda"
R, C = 65536, 8192
x = torch.randn(R, C, device=dev).bfloat16()
a = torch.randn(R, C, device=dev).bfloat16()
b = torch.randn(C, device=dev).bfloat16()
meta = F8.Fp8Meta(dev)


def timed(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


cases = {
    "copy_bf16": (lambda: a.copy_(x), 4 * R * C),
    "row_only": (lambda: F8.cast_transpose(x, meta, 0, 0, True, False), 3 * R * C),
    "t_only": (lambda: F8.cast_transpose(x, meta, 0, 0, False, True), 3 * R * C),
    "row_and_t": (lambda: F8.cast_transpose(x, meta, 0, 0, True, True), 4 * R * C),
    "amax_only": (lambda: F8.cast_transpose(x, meta, 0, 0, False, False), 2 * R * C),
    "gelu_row_and_t": (lambda: F8.bias_gelu_cast_transpose(x, b, meta, 0, 0, True, True), 4 * R * C),
    "gelu_bwd_row_and_t": (lambda: F8.bias_gelu_bwd_cast_transpose(x, a, b, meta, 2, 1, True, True), 6 * R * C),
}
for k, (fn, nbytes) in cases.items():
    ms = timed(fn)
    print(json.dumps({"case": k, "ms": round(ms, 4), "TB_s": round(nbytes / ms / 1e9, 2)}), flush=True)
