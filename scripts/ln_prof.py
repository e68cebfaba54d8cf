#!/usr/bin/env python
"""LayerNorm backward at the GPT-2 1.3B mb16 shape (16384 x 2048, residual fused), for rocprofv3 --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops.norms import add_norm  # noqa: E402

rows, N = 16384, 2048
x = torch.randn(rows, N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
r = torch.randn(rows, N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
w = torch.ones(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
b = torch.zeros(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
y, s = add_norm(x, r, w, b)
dy, ds = torch.randn_like(y), torch.randn_like(s)
for _ in range(10):
    torch.autograd.grad((y, s), (x, w, b), (dy, ds), retain_graph=True)
torch.cuda.synchronize()
print("done")
