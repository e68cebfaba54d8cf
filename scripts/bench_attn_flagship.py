#!/usr/bin/env python
"""Flash attention at the flagship layer shape (GPT-2 1.3B: B96 S1024 H16 D128 causal, packed qkv with the
c_attn bias gradient): forward and backward ms and TFLOP/s over interleaved rounds (one JSON line).  Under
`rocprofv3 --kernel-trace --stats` it gives the per-kernel split."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import attention as A  # noqa: E402

B, S, H, D = (int(os.environ.get(k, v)) for k, v in (("B", "96"), ("S", "1024"), ("H", "16"), ("D", "128")))
dev = torch.device("cuda")
torch.manual_seed(0)
qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16)
scale = D ** -0.5
do = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
dqkv = torch.empty_like(qkv)


def fwd():
    return A._fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], True, scale)


o, lse = fwd()


cso = do.float().reshape(B * S, H * D).sum(0)


def bwd():
    # the model's c_proj stashes colsum(dO) (db W) for the v part of the bias gradient: do the same here, so the
    # timed backward is the attention's own work (without it a column-sum pass over dO runs)
    if hasattr(A, "stash_dx_colsum"):
        A.stash_dx_colsum(do, cso)
    return A._bwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], o, lse, do, dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2],
                  True, scale, bias_grad=True)


def timeit(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


f_ms, b_ms = [], []
for _ in range(int(os.environ.get("ROUNDS", "5"))):
    f_ms.append(timeit(fwd))
    b_ms.append(timeit(bwd))
flops = 4 * B * H * S * S * D / 2
print(json.dumps({"shape": [B, S, H, D], "causal": True, "fwd_ms": round(min(f_ms), 4), "bwd_ms": round(min(b_ms), 4),
                  "fwd_tflops": round(flops / min(f_ms) / 1e9, 1), "bwd_tflops": round(2.5 * flops / min(b_ms) / 1e9, 1)}),
      flush=True)
