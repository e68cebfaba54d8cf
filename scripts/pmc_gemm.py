#!/usr/bin/env python
"""PMC target: the hand GEMM (csrc/kernels/gemm.hip) NT and TT, hipBLASLt NT and TN at an
8k^3 / flagship wgrad shape, 5 launches each on random data (rocprofv3 --pmc, scripts/summarize_pmc.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
a = torch.randn(8192, 8192, device=dev).bfloat16()
b = (torch.randn(8192, 8192, device=dev) / 90).bfloat16()
dy = torch.randn(32768, 2048, device=dev).bfloat16()
x = torch.randn(32768, 8192, device=dev).bfloat16()
for _ in range(5):
    G.gemm_nt(a, b)
    torch.mm(a, b.t())
    G.gemm_tt(dy, x)
    torch.mm(dy.t(), x)
torch.cuda.synchronize()
print("done")
