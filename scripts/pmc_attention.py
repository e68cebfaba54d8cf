#!/usr/bin/env python
"""Run the flash-attention kernels on the GPT-2 1.3B shape a few times (target for rocprofv3 PMC runs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402

B, S, H, D = 8, 1024, 16, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
for _ in range(int(os.environ.get("ITERS", "5"))):
    o = flash_attn(q, k, v, causal=True)
    torch.autograd.grad(o, (q, k, v), do)
torch.cuda.synchronize()
print("ok")
