#!/usr/bin/env python
"""Attention backward kernel variants at the GPT-2 1.3B mb16 layer shape, for rocprofv3 --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops.attention import set_kernel_variant  # noqa: E402

B, S, H, D = 16, 1024, 16, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
for var in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,3").split(",")]:
    set_kernel_variant(bwd=var)
    for causal in (True,):
        o = flash_attn(q, k, v, causal=causal)
        for _ in range(5):
            torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
torch.cuda.synchronize()
print("done")
