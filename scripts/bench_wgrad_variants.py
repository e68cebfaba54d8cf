"""Weight-gradient formulations dW[N, K] = dY[T, N]^T X[T, K] on the flagship (GPT-2 1.3B, T = 32768) and
Llama-3 8B (T = 8192) shapes, plus the Llama data-gradient layouts.  One JSON line per case.
Usage: python scripts/bench_wgrad_variants.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributedtraining_amd.ops.linear import transpose16  # noqa: E402

CASES = [("gpt2-1.3b", 32768, {"qkv": (6144, 2048), "proj": (2048, 2048), "fc1": (8192, 2048),
                               "fc2": (2048, 8192), "lm_head": (50304, 2048)}),
         ("llama3-8b", 8192, {"wqkv": (6144, 4096), "wo": (4096, 4096), "w13": (28672, 4096),
                              "w2": (4096, 14336), "output": (128256, 4096)})]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    for model, T, shapes in CASES:
        for name, (n, k) in shapes.items():
            x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
            dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
            w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * T * n * k
            cands = {
                "wgrad mm(dy.t, x)": lambda: torch.mm(dy.t(), x),
                "wgrad mm(x.t, dy) + transpose16": lambda: transpose16(torch.mm(x.t(), dy)),
                "wgrad mm(x.t, dy) only": lambda: torch.mm(x.t(), dy),
            }
            if model == "llama3-8b":
                cands["dgrad mm(dy, w)"] = lambda: torch.mm(dy, w)
                cands["dgrad linear(dy, transpose16(w))"] = lambda: F.linear(dy, transpose16(w))
                cands["fwd linear(x, w)"] = lambda: F.linear(x, w)
            for c, fn in cands.items():
                ms = timeit(fn)
                print(json.dumps({"model": model, "gemm": name, "case": c, "T": T, "N": n, "K": k,
                                  "ms": round(ms, 4), "pflops": round(fl / ms / 1e12, 3)}), flush=True)
            del x, dy, w


if __name__ == "__main__":
    main()
