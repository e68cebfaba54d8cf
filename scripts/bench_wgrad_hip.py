#!/usr/bin/env python
"""Hand MFMA weight-gradient GEMM (csrc/kernels/gemm_wgrad.hip) vs hipBLASLt (torch.mm(dY^T, X)) on the
flagship / Llama shapes: ms, PFLOP/s, and the error of each against an fp32 product.  One process, interleaved."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops import _lib  # noqa: E402
from pytorch_distributedtraining_amd.ops.linear import hip_wgrad, hip_wgrad_splits  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,2").split(",")]

SHAPES = [("gpt2-1.3b qkv", 65536, 6144, 2048), ("gpt2-1.3b proj", 65536, 2048, 2048),
          ("gpt2-1.3b fc1", 65536, 8192, 2048), ("gpt2-1.3b fc2", 65536, 2048, 8192),
          ("llama3-8b qkv", 8192, 6144, 4096), ("llama3-8b gate_up", 8192, 28672, 4096),
          ("llama3-8b down", 8192, 4096, 14336)]


def timed(fn, it=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


torch.manual_seed(0)
for name, m, n, k in SHAPES:
    dy = torch.randn(m, n, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    ref = (dy[:4096].float().t() @ x[:4096].float())
    s0 = hip_wgrad_splits(m, n, k)
    cands = sorted({s0, 1, 4} if m % 256 == 0 else {s0})
    errs = {}
    for v in VARIANTS:
        _lib.require().pdt_wgrad_set_variant(v)
        d = hip_wgrad(dy[:4096], x[:4096], splits=1)
        errs[v] = round(float((d.float() - ref).norm() / ref.norm()), 5)
        for s in cands:
            hip_wgrad(dy, x, splits=s)
    d_lt = (dy[:4096].t() @ x[:4096])
    err_lt = float((d_lt.float() - ref).norm() / ref.norm())
    res = {}
    for _ in range(3):
        for v in VARIANTS:
            _lib.require().pdt_wgrad_set_variant(v)
            for s in cands:
                res.setdefault(f"hip_v{v}_s{s}", []).append(timed(lambda: hip_wgrad(dy, x, splits=s)))
        res.setdefault("hipblaslt", []).append(timed(lambda: dy.t() @ x))
    fl = 2.0 * m * n * k
    out = {"shape": name, "M": m, "N": n, "K": k, "default_splits": s0, "rel_err_hip": errs,
           "rel_err_hipblaslt": round(err_lt, 5)}
    for key, v in res.items():
        ms = sorted(v)[len(v) // 2]
        out[key + "_pf"] = round(fl / ms / 1e12, 3)
    print(json.dumps(out), flush=True)
