#!/usr/bin/env python
"""Window attention at the SwinIR-S Stoke shape (4,608 windows x 6 heads x 64 tokens, d = 10, the shifted block's
region-label mask), forward + backward in bf16 (MFMA 32x32x16) and fp32 (MFMA 32x32x2 f32), ITERS times -- the
target of rocprofv3 --pmc passes (scripts/sessions/gpu_r6_e.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.models.swinir import SwinTransformerBlock  # noqa: E402
from pytorch_distributedtraining_amd.ops.window_attention import window_attention  # noqa: E402

dev = torch.device("cuda")
it = int(os.environ.get("ITERS", "3"))
mask = SwinTransformerBlock(60, (128, 128), 6, window_size=8, shift_size=4)._mask((128, 128)).to(dev)
for dt in (torch.bfloat16, torch.float32):
    qkv = torch.randn(4608, 64, 180, device=dev, dtype=dt, requires_grad=True)
    rel = (0.02 * torch.randn(6, 64, 64, device=dev)).requires_grad_()
    dwo = torch.randn(4608, 64, 60, device=dev, dtype=dt)
    for _ in range(it):
        ow = window_attention(qkv, rel, mask, 6, 10 ** -0.5)
        torch.autograd.grad(ow, (qkv, rel), dwo)
torch.cuda.synchronize()
print("ok")
