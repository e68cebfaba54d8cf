"""Time every flagship GEMM (GPT-2 1.3B, 32 x 1024 tokens) in its three roles -- forward y = x W^T,
data gradient dx = dy W, weight gradient dW = dy^T x -- exactly as torch.nn.functional.linear /
ops.linear issue them.  Prints one JSON line per (shape, role) with ms and PFLOP/s.
Usage: python scripts/bench_gemm_roles.py [dgrad]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_distributedtraining_amd.ops.linear import transpose16  # noqa: E402

T = 32768
SHAPES = {"qkv": (6144, 2048), "proj": (2048, 2048), "fc1": (8192, 2048), "fc2": (2048, 8192),
          "lm_head": (50304, 2048)}
if len(sys.argv) > 1 and sys.argv[1] == "dgrad":
    ROLES = ("dgrad_mm", "dgrad_linear_wT", "transpose_w", "transpose16_w", "dgrad_framework", "fwd_linear")
else:
    ROLES = None


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
    for name, (n, k) in SHAPES.items():
        x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02
        b = torch.zeros(n, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
        wt = w.t().contiguous()
        fl = 2.0 * T * n * k
        roles = {
            "fwd_linear_bias": lambda: torch.nn.functional.linear(x, w, b),
            "fwd_linear": lambda: torch.nn.functional.linear(x, w),
            "dgrad_mm": lambda: torch.mm(dy, w),
            # same product through the forward (x W^T) layout on a pre-transposed weight copy
            "dgrad_linear_wT": lambda: torch.nn.functional.linear(dy, wt),
            "transpose_w": lambda: w.t().contiguous(),
            "transpose16_w": lambda: transpose16(w),
            "dgrad_framework": lambda: F.linear(dy, transpose16(w)),
            "wgrad_mm": lambda: torch.mm(dy.t(), x),
            "wgrad_mm_fp32out": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32),
        }
        for role, fn in roles.items():
            if ROLES and role not in ROLES:
                continue
            ms = timeit(fn)
            print(json.dumps({"gemm": name, "role": role, "M": T, "N": n, "K": k, "ms": round(ms, 4),
                              "pflops": round(fl / ms / 1e12, 3)}), flush=True)
        del x, w, dy


if __name__ == "__main__":
    main()
