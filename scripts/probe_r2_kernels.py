#!/usr/bin/env python
"""Runs the round-2 hand kernels a few times each at their production shapes, for rocprofv3 --pmc passes:
fused SwinIR MLP fwd/bwd (294,912 tokens, 60 -> 120 -> 60), fp8 cast+transpose (GPT-2 1.3B activation
65,536 x 2048 and MLP hidden 65,536 x 8192), hand weight-gradient GEMM (fc2: 65,536 tokens, 2048 x 8192)."""
import torch

from pytorch_distributedtraining_amd.ops import fp8 as F8
from pytorch_distributedtraining_amd.ops.linear import hip_wgrad
from pytorch_distributedtraining_amd.ops.swin_mlp import fused_mlp

dev = "cuda"
torch.manual_seed(0)
T, C, H = 294912, 60, 120
x = torch.randn(T, C, device=dev).bfloat16().requires_grad_()
w1 = (0.1 * torch.randn(H, C, device=dev)).bfloat16().requires_grad_()
b1 = torch.zeros(H, device=dev).bfloat16().requires_grad_()
w2 = (0.1 * torch.randn(C, H, device=dev)).bfloat16().requires_grad_()
b2 = torch.zeros(C, device=dev).bfloat16().requires_grad_()
dy = torch.randn(T, C, device=dev).bfloat16()
for _ in range(5):
    fused_mlp(x, w1, b1, w2, b2, x).backward(dy)
meta = F8.Fp8Meta(dev)
for shape in ((65536, 2048), (65536, 8192)):
    a = torch.randn(*shape, device=dev).bfloat16()
    for _ in range(5):
        F8.cast_transpose(a, meta, 0, 0)
        F8.cast_transpose(a, meta, 2, 1)
dy2 = torch.randn(65536, 2048, device=dev).bfloat16()
x2 = torch.randn(65536, 8192, device=dev).bfloat16()
for _ in range(5):
    hip_wgrad(dy2, x2)
torch.cuda.synchronize()
print("probe done")
