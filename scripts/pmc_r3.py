#!/usr/bin/env python
"""PMC target for round 3 (rocprofv3 --pmc passes via scripts/gpu_pmc.sh PROBE=scripts/pmc_r3.py): the flash-
attention kernels at the flagship shape (GPT-2 1.3B: B96 S1024 H16 D128 causal, default variants and block
order), the hand TT weight-gradient GEMM at the c_fc / c_proj shapes, and hipBLASLt's NT forward GEMM of c_fc,
each a few launches on random data."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402

it = int(os.environ.get("ITERS", "3"))
B, S, H, D = 96, 1024, 16, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    o = flash_attn(q, k, v, causal=True)
    torch.autograd.grad(o, (q, k, v), do)
del q, k, v, do, o
T = 96 * 1024
dy = torch.randn(T, 8192, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, 2048, device="cuda", dtype=torch.bfloat16)
w = (torch.randn(8192, 2048, device="cuda") / 45).bfloat16()
for _ in range(it):
    G.gemm_tt(dy, x)                 # dW of c_fc   [8192, 2048]
    G.gemm_tt(x, dy)                 # dW of c_proj [2048, 8192]
    torch.mm(x, w.t())               # c_fc forward on hipBLASLt
torch.cuda.synchronize()
print("ok")
