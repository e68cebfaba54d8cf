#!/usr/bin/env python
"""GPT-2 1.3B tied LM head GEMMs at the flagship's 96 x 1024 tokens: forward logits (x W^T), the data gradient
as the framework runs it (dY against the transposed weight) and the weight gradient (hipBLASLt TN vs the hand TT
kernel on the 256-row-aligned part + hipBLASLt for the rest)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributedtraining_amd.ops.linear import hip_wgrad_ragged, transpose16  # noqa: E402

dev = torch.device("cuda")
T, C, V = 96 * 1024, 2048, 50304
x = torch.randn(T, C, device=dev, dtype=torch.bfloat16)
w = torch.randn(V, C, device=dev, dtype=torch.bfloat16) * 0.02
dy = torch.randn(T, V, device=dev, dtype=torch.bfloat16) * 1e-3


def timed(fn, iters=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


fl = 2.0 * T * C * V
wt = transpose16(w)
res = {}
for name, fn in (("fwd", lambda: F.linear(x, w)), ("dgrad_nt", lambda: F.linear(dy, wt)),
                 ("dgrad_nn", lambda: torch.mm(dy, w)), ("wgrad_lt", lambda: torch.mm(dy.t(), x)),
                 ("wgrad_hip_ragged", lambda: hip_wgrad_ragged(dy, x))):
    ms = min(timed(fn) for _ in range(3))
    res[name] = {"ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}
print(json.dumps(res), flush=True)
