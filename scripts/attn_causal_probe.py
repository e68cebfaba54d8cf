"""Causal vs full flash attention time (fwd, fwd+bwd) on the flagship shape and a long-sequence shape:
does causal skip its work proportionally?  (CUDA events)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops import flash_attn_qkvpacked  # noqa: E402


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for B, S in ((32, 1024), (8, 4096)):
    qkv = torch.randn(B, S, 3, 16, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    for causal in (False, True):
        o = flash_attn_qkvpacked(qkv, causal=causal)
        g = torch.randn_like(o)
        fwd = t(lambda: flash_attn_qkvpacked(qkv, causal=causal))
        both = t(lambda: flash_attn_qkvpacked(qkv, causal=causal).backward(g))
        print(json.dumps({"B": B, "S": S, "causal": causal, "fwd_ms": round(fwd, 3), "bwd_ms": round(both - fwd, 3)}),
              flush=True)
