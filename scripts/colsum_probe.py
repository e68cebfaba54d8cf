"""Time the HIP column sum against torch's sum(0) on SwinIR bias-gradient shapes (CUDA events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops.activations import _colsum  # noqa: E402


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for n in (60, 180, 120):
    x = torch.randn(294912, n, device="cuda", dtype=torch.bfloat16)
    print(json.dumps({"n": n, "hip_colsum_us": round(t(lambda: _colsum(x, torch.float32)), 1),
                      "torch_sum_us": round(t(lambda: x.sum(0).float()), 1)}), flush=True)
