#!/usr/bin/env python
"""Perceptual (feat_loss) network variants at the SwinIR Stoke shape (18 x 3 x 256 x 256, bf16 autocast, output
gradient only): stock nn.Conv2d NCHW / channels_last, and the im2col + hipBLASLt Conv2d3x3 path."""
import json
import time

import torch

from pytorch_distributedtraining_amd.models.losses import PerceptualLoss
from pytorch_distributedtraining_amd.ops.conv import Conv2d3x3

torch.backends.cudnn.benchmark = True
dev = "cuda"


def variant(kind):
    m = PerceptualLoss().to(dev)
    if kind == "hip":
        for i, l in enumerate(m.features):
            if isinstance(l, torch.nn.Conv2d):
                c = Conv2d3x3(l.in_channels, l.out_channels).to(dev)
                c.load_state_dict(l.state_dict())
                c.requires_grad_(False)
                m.features[i] = c
    if kind in ("cl", "hip"):
        m = m.to(memory_format=torch.channels_last)
    return m


def run(kind, iters=10):
    m = variant(kind)
    out = torch.rand(18, 3, 256, 256, device=dev, requires_grad=True)
    tgt = torch.rand(18, 3, 256, 256, device=dev)
    if kind != "nchw":
        out = out.detach().to(memory_format=torch.channels_last).requires_grad_()
        tgt = tgt.to(memory_format=torch.channels_last)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = m(out, tgt)
        loss.backward()
        return loss
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        loss = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1000 / iters
    return ms, float(loss), out.grad.float().norm().item()


for k in ("nchw", "cl", "hip"):
    try:
        ms, l, g = run(k)
        print(json.dumps({"variant": k, "ms_fwd_bwd": round(ms, 3), "loss": round(l, 5), "grad_norm": round(g, 4)}),
              flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"variant": k, "error": repr(e)[:300]}), flush=True)
