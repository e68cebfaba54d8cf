#!/usr/bin/env python
"""Per-call time of the fused window attention (forward, backward) at the SwinIR-S Stoke shape: 4,608 windows x
6 heads x 64 tokens, d = 10, shifted-window label mask.  PDT_KERNEL_LIB selects an experiment build."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.models.swinir import SwinTransformerBlock  # noqa: E402
from pytorch_distributedtraining_amd.ops.window_attention import window_attention  # noqa: E402

dev = torch.device("cuda")
mask = SwinTransformerBlock(60, (128, 128), 6, window_size=8, shift_size=4)._mask((128, 128)).to(dev)
res = {"lib": os.path.basename(os.environ.get("PDT_KERNEL_LIB", "default"))}
for dt in (torch.bfloat16, torch.float32):
    qkv = torch.randn(4608, 64, 180, device=dev, dtype=dt, requires_grad=True)
    rel = (0.02 * torch.randn(6, 64, 64, device=dev)).requires_grad_()
    dwo = torch.randn(4608, 64, 60, device=dev, dtype=dt)
    for m in (None, mask):
        for _ in range(3):
            ow = window_attention(qkv, rel, m, 6, 10 ** -0.5)
            torch.autograd.grad(ow, (qkv, rel), dwo)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf = tb = 0.0
        n = 20
        for _ in range(n):
            ev[0].record()
            ow = window_attention(qkv, rel, m, 6, 10 ** -0.5)
            ev[1].record()
            torch.autograd.grad(ow, (qkv, rel), dwo)
            ev[2].record()
            torch.cuda.synchronize()
            tf += ev[0].elapsed_time(ev[1])
            tb += ev[1].elapsed_time(ev[2])
        key = f"{str(dt)[6:]}_{'masked' if m is not None else 'plain'}"
        res[key] = {"fwd_us": round(1000 * tf / n, 1), "bwd_us": round(1000 * tb / n, 1)}
print(json.dumps(res))
