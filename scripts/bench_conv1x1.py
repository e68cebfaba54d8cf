#!/usr/bin/env python
"""ResNet-50 stride-1 1x1 convolutions at batch 256 (NHWC bf16): MIOpen (find mode) vs the same product as plain
GEMMs on the channels_last storage (fwd x W^T, dgrad dY W, wgrad dY^T X).  Per shape: fwd / bwd ms each way."""
import json

import torch
import torch.nn.functional as F

from pytorch_distributedtraining_amd.ops.linear import wgrad

torch.backends.cudnn.benchmark = True
dev = "cuda"
B = 256
SHAPES = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
          (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048), (7, 2048, 512)]


def timed(fn, it=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


for (hw, ci, co) in SHAPES:
    x = torch.randn(B, ci, hw, hw, device=dev).bfloat16().to(memory_format=torch.channels_last)
    w = (0.05 * torch.randn(co, ci, 1, 1, device=dev)).bfloat16()
    dy = torch.randn(B, co, hw, hw, device=dev).bfloat16().to(memory_format=torch.channels_last)
    xr = x.detach().requires_grad_()
    wr = w.detach().requires_grad_()

    def mi_fwd():
        return F.conv2d(x, w)

    def mi_bwd():
        y = F.conv2d(xr, wr)
        torch.autograd.grad(y, (xr, wr), dy)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
    w2 = w.view(co, ci)

    def gm_fwd():
        return x2 @ w2.t()

    def gm_bwd():
        return dy2 @ w2, wgrad(dy2, x2, torch.bfloat16)
    t_mf, t_gf = timed(mi_fwd), timed(gm_fwd)
    t_mb = timed(mi_bwd) - t_mf          # conv backward = autograd grad (includes a forward)
    t_gb = timed(gm_bwd)
    print(json.dumps({"hw": hw, "cin": ci, "cout": co, "miopen_fwd_ms": round(t_mf, 4), "gemm_fwd_ms": round(t_gf, 4),
                      "miopen_bwd_ms": round(t_mb, 4), "gemm_bwd_ms": round(t_gb, 4)}), flush=True)
