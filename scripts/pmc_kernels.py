#!/usr/bin/env python
"""Run every hand-written hot kernel a few times at its production shape (target for rocprofv3 --pmc runs):
flash attention fwd+bwd (GPT-2 1.3B: B8 S1024 H16 D128 causal), MFMA window attention fwd+bwd (SwinIR-S:
4608 windows x 6 heads x 64 tokens, d 10, shift mask), fused BN+add+ReLU fwd+bwd (ResNet-50
[256, 256, 56, 56] bf16 channels-last), LayerNorm with fused residual (32768 x 2048) and fused AdamW (1.3B-
element shard)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops.batchnorm import BatchNormAct2d  # noqa: E402
from pytorch_distributedtraining_amd.ops.norms import add_norm  # noqa: E402
from pytorch_distributedtraining_amd.ops.window_attention import window_attention  # noqa: E402
from pytorch_distributedtraining_amd.optim import FusedAdamW  # noqa: E402

dev = torch.device("cuda")
it = int(os.environ.get("ITERS", "3"))
bf = torch.bfloat16
# flash attention
q, k, v = (torch.randn(8, 1024, 16, 128, device=dev, dtype=bf, requires_grad=True) for _ in range(3))
do = torch.randn(8, 1024, 16, 128, device=dev, dtype=bf)
# window attention (SwinIR-S block, shifted: mask)
qkv = torch.randn(4608, 64, 180, device=dev, dtype=bf, requires_grad=True)
rel = (0.02 * torch.randn(6, 64, 64, device=dev)).requires_grad_()
mask = torch.zeros(256, 64, 64, device=dev)
mask[:, :32, 32:] = -100.0
mask[:, 32:, :32] = -100.0
dwo = torch.randn(4608, 64, 60, device=dev, dtype=bf)
# fused BN + residual + ReLU
bn = BatchNormAct2d(256, act="relu").to(dev)
x = torch.randn(256, 256, 56, 56, device=dev, dtype=bf).to(memory_format=torch.channels_last).requires_grad_()
res = torch.randn(256, 256, 56, 56, device=dev, dtype=bf).to(memory_format=torch.channels_last)
# LayerNorm + residual
hs = torch.randn(32768, 2048, device=dev, dtype=bf, requires_grad=True)
hr = torch.randn(32768, 2048, device=dev, dtype=bf)
lw, lb = torch.ones(2048, device=dev, requires_grad=True), torch.zeros(2048, device=dev, requires_grad=True)
# AdamW over a 1.3B-element fp32 shard with bf16 grads
p = torch.nn.Parameter(torch.randn(1 << 30, device=dev) * 0.02)
p._pdt_grad = torch.randn(1 << 30, device=dev, dtype=bf) * 1e-3
p._pdt_lp_shard = torch.empty(1 << 30, device=dev, dtype=bf)
opt = FusedAdamW([p], lr=1e-4)
for _ in range(it):
    o = flash_attn(q, k, v, causal=True)
    torch.autograd.grad(o, (q, k, v), do)
    ow = window_attention(qkv, rel, mask, 6, 10 ** -0.5)
    torch.autograd.grad(ow, (qkv, rel), dwo)
    y = bn(x, residual=res)
    torch.autograd.grad(y, (x,), torch.ones_like(y))
    yn, _s = add_norm(hs, hr, lw, lb)
    torch.autograd.grad(yn, (hs,), torch.ones_like(yn))
    opt.step()
torch.cuda.synchronize()
print("ok")
