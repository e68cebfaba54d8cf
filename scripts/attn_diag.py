#!/usr/bin/env python
"""Where does the causal forward disagree with an fp32 reference?  Per (batch, head) relative errors and
the worst rows, for each forward variant, on a given shape."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops.attention import set_kernel_variant  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="32,1024,16,16,128")
ap.add_argument("--fwd", default="2,4,5")
ap.add_argument("--batches", default="0,1,31")
a = ap.parse_args()
B, S, H, Hkv, D = (int(x) for x in a.shape.split(","))
torch.manual_seed(0)
q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16)
outs = {}
for f in (int(x) for x in a.fwd.split(",")):
    set_kernel_variant(fwd=f)
    with torch.no_grad():
        outs[f] = flash_attn(q, k, v, causal=True).float()
for b in (int(x) for x in a.batches.split(",")):
    qt, kt, vt = (t[b:b + 1].float().transpose(1, 2) for t in (q, k, v))
    kt, vt = kt.repeat_interleave(H // Hkv, 1), vt.repeat_interleave(H // Hkv, 1)
    sc = (qt @ kt.transpose(-1, -2)) / D ** 0.5
    sc = sc.masked_fill(~torch.ones(S, S, dtype=torch.bool, device="cuda").tril(), float("-inf"))
    oref = (sc.softmax(-1) @ vt).transpose(1, 2)[0]       # [S, H, D]
    for f, o in outs.items():
        ob = o[b]
        err = (ob - oref).norm(dim=-1) / oref.norm(dim=-1)   # [S, H]
        worst = err.max(0)
        bad_heads = [(h, round(float(worst.values[h]), 4), int(worst.indices[h])) for h in range(H)
                     if worst.values[h] > 0.02]
        rows_bad = int((err > 0.02).sum())
        print(f"b={b} fwd={f} rel={float((ob - oref).norm() / oref.norm()):.5f} rows>2%={rows_bad} bad_heads={bad_heads[:8]}",
              flush=True)
