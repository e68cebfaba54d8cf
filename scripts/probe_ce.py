#!/usr/bin/env python
"""Cross-entropy at the GPT-2 1.3B flagship head (98,304 x 50,304 bf16 logits): the fused forward+gradient kernel
against the two-pass forward / backward, median of 10 forward+backward pairs.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

import torch  # noqa: E402

CE = importlib.import_module("pytorch_distributedtraining_amd.ops.cross_entropy")   # (ops.cross_entropy is the function)

dev = torch.device("cuda")
R, V = 96 * 1024, 50304
t = torch.randint(0, V, (R,), device=dev)
base = torch.randn(R, V, device=dev).bfloat16()


def run(fused):
    CE.FWD_GRAD = fused
    ts = []
    for i in range(12):
        leaf = base.clone().requires_grad_()
        x = leaf * 1.0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        CE.cross_entropy(x, t, grad_in_forward=True).backward()
        e1.record()
        e1.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
        del leaf, x
    ts.sort()
    return round(ts[len(ts) // 2], 3)


print(json.dumps({"nth": os.environ.get("PDT_CE_FUSED_NTH", "1024"), "fused_ms": run(True), "two_pass_ms": run(False),
                  "note": "includes the multiply-by-1 copy into the leaf's gradient"}), flush=True)
