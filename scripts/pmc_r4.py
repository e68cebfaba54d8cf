#!/usr/bin/env python
"""PMC target for round 4 (rocprofv3 --pmc passes via scripts/gpu_pmc.sh PROBE=scripts/pmc_r4.py): the shipped
flash-attention kernels at the flagship shape (GPT-2 1.3B: B96 S1024 H16 D128 causal), the inline-asm GEMM at the
flagship's four MLP products (TT weight gradients of c_fc / c_proj, NT c_fc forward with the bias+GELU epilogue,
NT c_proj forward) and hipBLASLt's NT products at the same two forward shapes, each a few launches on random
data.  Rows of the summary are per kernel name, so the asm rows average its TT and NT launches; the TT-only and
NT-only runs (MODE=tt / MODE=nt) separate them."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402

it = int(os.environ.get("ITERS", "3"))
mode = os.environ.get("MODE", "all")
if mode in ("all", "attn"):
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
w2 = (torch.randn(2048, 8192, device="cuda") / 90).bfloat16()
b = torch.zeros(8192, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    if mode in ("all", "tt"):
        G.gemm_tt(dy, x)                 # dW of c_fc   [8192, 2048]
        G.gemm_tt(x, dy)                 # dW of c_proj [2048, 8192]
    if mode in ("all", "nt"):
        G.gemm_nt_gelu(x, w, b)          # c_fc forward + bias + GELU epilogue
        G.gemm_nt(dy, w2)                # c_proj forward (K = 8192)
    if mode in ("all", "nt", "dgelu"):
        G.gemm_nt_dgelu(x, w, dy)        # c_proj data gradient + GELU backward + c_fc bias gradient epilogue
    if mode in ("all", "lt"):
        torch.mm(x, w.t())               # c_fc forward on hipBLASLt
        torch.mm(dy, w2.t())             # c_proj forward on hipBLASLt
torch.cuda.synchronize()
print("ok")
