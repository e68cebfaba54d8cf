#!/usr/bin/env python
"""Attention forward / backward time at equal causal FLOPs (B * S^2 fixed) but different per-workgroup work:
B96 S1024 vs B24 S2048 vs B6 S4096 (H16 D128).  A large per-FLOP gap at short S points at per-workgroup costs
(prologue loads, epilogue stores, launch turnover) rather than the main loops."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import attention as A  # noqa: E402

dev = torch.device("cuda")
H, D = 16, 128


def timed(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for B, S in ((96, 1024), (24, 2048), (6, 4096)):
    qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16)
    scale = D ** -0.5
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = A._fwd(q, k, v, True, scale)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    f = min(timed(lambda: A._fwd(q, k, v, True, scale)) for _ in range(3))
    b = min(timed(lambda: A._bwd(q, k, v, o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], True, scale))
            for _ in range(3))
    fl = 4.0 * B * H * S * S * D / 2
    print(json.dumps({"B": B, "S": S, "fwd_ms": round(f, 4), "bwd_ms": round(b, 4),
                      "fwd_tflops": round(fl / f / 1e9, 1), "bwd_tflops": round(2.5 * fl / b / 1e9, 1)}), flush=True)
    del qkv, o, lse, do, dqkv
