#!/usr/bin/env python
"""Attention backward at the flagship shape (B96 S1024 H16 D128 causal, packed qkv) with and without the
in-kernel bias-gradient column sums, against the separate column-sum pass they replace; interleaved rounds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import attention as A  # noqa: E402
from pytorch_distributedtraining_amd.ops.activations import _colsum  # noqa: E402

B, S, H, D = int(os.environ.get("B", "96")), 1024, 16, 128
dev = torch.device("cuda")
qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16)
scale = D ** -0.5
o, lse = A._fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], True, scale)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)


def bwd(bias):
    return A._bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                  True, scale, bias_grad=bias)


def sep():
    bwd(False)
    return _colsum(dqkv.view(B * S, 3 * H * D), torch.bfloat16)


def timed(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


res = {"plain": [], "fused": [], "separate": []}
for r in range(4):
    res["plain"].append(timed(lambda: bwd(False)))
    res["fused"].append(timed(lambda: bwd(True)))
    res["separate"].append(timed(sep))
print(json.dumps({k: round(min(v), 4) for k, v in res.items()} | {"B": B}), flush=True)
