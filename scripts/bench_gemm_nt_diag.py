#!/usr/bin/env python
"""Where does the hand NT GEMM (csrc/kernels/gemm.hip, Linear forward layout) lose to hipBLASLt at short K?
Times, per shape, the production plain kernel (diag 0), the same kernel without its epilogue stores (diag 4),
the persistent plain kernel (diag 5), the GELU-epilogue kernel and hipBLASLt (torch.mm against b^T) -- the GPT-2 1.3B c_fc shape (K = 2048) against
the c_proj shape (K = 8192) separates the per-tile (prologue / epilogue) cost from the main loop's."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import _lib  # noqa: E402
from pytorch_distributedtraining_amd.ops.gemm import gemm_nt_gelu  # noqa: E402

lib = _lib.require()
T = int(os.environ.get("TOK", str(96 * 1024)))
dev = torch.device("cuda")


def timed(fn, reps=3, iters=5):
    best = 1e30
    for _ in range(reps):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best


for N, K in ((8192, 2048), (2048, 8192), (6144, 2048), (2048, 2048)):
    a = torch.randn(T, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    bias = torch.randn(N, device=dev).bfloat16()
    c = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    st = _lib.stream_handle(dev)
    fl = 2.0 * T * N * K
    res = {"M": T, "N": N, "K": K}
    for d in (0, 4, 5):
        ms = timed(lambda: _lib.check(lib.pdt_gemm_diag_nt_bf16(d, a.data_ptr(), b.data_ptr(), c.data_ptr(), T, N, K, st),
                                      "diag"))
        res[f"diag{d}_ms"] = round(ms, 4)
        res[f"diag{d}_tflops"] = round(fl / ms / 1e9, 1)
    ms = timed(lambda: gemm_nt_gelu(a, b, bias))
    res["gelu_ms"], res["gelu_tflops"] = round(ms, 4), round(fl / ms / 1e9, 1)
    ms = timed(lambda: gemm_nt_gelu(a, b, bias, persist=True))
    res["gelu_persist_ms"], res["gelu_persist_tflops"] = round(ms, 4), round(fl / ms / 1e9, 1)
    ms = timed(lambda: torch.mm(a, b.t()))
    res["lt_ms"], res["lt_tflops"] = round(ms, 4), round(fl / ms / 1e9, 1)
    print(json.dumps(res), flush=True)
    del a, b, c
