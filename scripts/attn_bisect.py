#!/usr/bin/env python
"""Per-gradient error of each attention-backward kernel generation vs an fp32 reference (debug aid)."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops.attention import set_kernel_variant  # noqa: E402


def ref(q, k, v, causal):
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    s = (qt @ kt.transpose(-1, -2)) / math.sqrt(q.shape[-1])
    if causal:
        m = torch.ones(q.shape[1], k.shape[1], dtype=torch.bool, device=q.device).tril(k.shape[1] - q.shape[1])
        s = s.masked_fill(~m, float("-inf"))
    return (s.softmax(-1) @ vt).transpose(1, 2)


torch.manual_seed(0)
for (B, S, H, D) in [(2, 256, 4, 64), (2, 256, 4, 128), (1, 200, 2, 128)]:
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    gr = torch.autograd.grad(ref(qr, kr, vr, True), (qr, kr, vr), do.float())
    for var in (2, 3, 5, 6):
        set_kernel_variant(bwd=var)
        o = flash_attn(q, k, v, causal=True)
        g = torch.autograd.grad(o, (q, k, v), do)
        errs = [((a.float() - b).norm() / b.norm()).item() for a, b in zip(g, gr)]
        # first bad key / query row for dk and dq
        bad_k = ((g[1].float() - gr[1]).abs().amax(dim=(0, 2, 3)) > 0.05).nonzero().flatten()[:8].tolist()
        bad_q = ((g[0].float() - gr[0]).abs().amax(dim=(0, 2, 3)) > 0.05).nonzero().flatten()[:8].tolist()
        print(f"B{B} S{S} H{H} D{D} v{var}: dq {errs[0]:.4f} dk {errs[1]:.4f} dv {errs[2]:.4f} "
              f"bad_k {bad_k} bad_q {bad_q}", flush=True)
