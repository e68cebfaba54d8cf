#!/usr/bin/env python
"""Linear weight+bias gradient at the GPT-2 1.3B flagship shapes (32 x 1024 tokens): hipBLASLt GEMM + the
framework's column-sum kernel vs ONE hipBLASLt GEMM with the BGRADB epilogue (ops.blaslt.wgrad_bgrad)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops.activations import _colsum  # noqa: E402
from pytorch_distributedtraining_amd.ops.blaslt import wgrad_bgrad  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    M = 32768
    for name, N, K in (("qkv", 6144, 2048), ("attn_proj", 2048, 2048), ("fc2", 2048, 8192), ("gpt2-124m qkv", 2304, 768)):
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        a = timeit(lambda: (torch.mm(dy.t(), x), _colsum(dy, torch.bfloat16)))
        b = timeit(lambda: wgrad_bgrad(dy, x))
        dw, db = wgrad_bgrad(dy, x)
        err = float(((dw.float() - torch.mm(dy.t().float(), x.float())).norm() / torch.mm(dy.t().float(), x.float()).norm()))
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "separate_ms": round(a, 4), "bgradb_ms": round(b, 4),
                          "speedup": round(a / b, 3), "dw_rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
