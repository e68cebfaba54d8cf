#!/usr/bin/env python
"""Hand MFMA GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch):
correctness against fp32 torch, then interleaved timing rounds in one process (cdna_hip_programming.md §5.4
rule 24) at the GPT-2 1.3B flagship shapes (96 x 1024 tokens) on random data.  One JSON line per case."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402
from pytorch_distributedtraining_amd.ops.activations import bias_gelu  # noqa: E402

dev = torch.device("cuda")
TOK = int(os.environ.get("TOK", str(96 * 1024)))
ROUNDS = int(os.environ.get("ROUNDS", "5"))
ONLY = os.environ.get("ONLY", "")


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def out(**kw):
    print(json.dumps(kw), flush=True)


def timeit(fn, iters=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def check():
    torch.manual_seed(0)
    M, N, K = 2048, 1024, 1536
    a = torch.randn(M, K, device=dev).bfloat16()
    b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
    bias = torch.randn(N, device=dev).bfloat16()
    ref = a.float() @ b.float().t()
    out(case="check_nt_plain", rel=rel(G.gemm_nt(a, b), ref))
    out(case="check_nt_bias", rel=rel(G.gemm_nt(a, b, bias), ref + bias.float()))
    y, pre = G.gemm_nt_gelu(a, b, bias)
    out(case="check_nt_gelu", rel_pre=rel(pre, ref + bias.float()),
        rel_y=rel(y, torch.nn.functional.gelu(ref + bias.float(), approximate="tanh")))
    h = (torch.randn(M, N, device=dev)).bfloat16()
    g, db = G.gemm_nt_dgelu(a, b, h)
    hr = h.float().requires_grad_()
    torch.nn.functional.gelu(hr, approximate="tanh").backward(ref)
    out(case="check_nt_dgelu", rel_g=rel(g, hr.grad), rel_db=rel(db, hr.grad.sum(0)))
    at = torch.randn(K * 4, M // 2, device=dev).bfloat16()
    bt = torch.randn(K * 4, N, device=dev).bfloat16()
    reft = at.float().t() @ bt.float()
    for s in (1, 2, 4):
        out(case=f"check_tt_s{s}", rel=rel(G.gemm_tt(at, bt, splits=s), reft))


def bench():
    torch.manual_seed(1)
    d = 2048
    nt_shapes = {"qkv": (TOK, 3 * d, d), "attn_proj": (TOK, d, d), "fc": (TOK, 4 * d, d), "fc_proj": (TOK, d, 4 * d),
                 "sq8k": (8192, 8192, 8192)}
    for name, (M, N, K) in nt_shapes.items():
        if ONLY and ONLY not in name:
            continue
        a = torch.randn(M, K, device=dev).bfloat16()
        b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device=dev).bfloat16()
        fl = 2.0 * M * N * K
        res = {"hip": [], "lt": []}
        extra = name == "fc"
        if extra:
            res.update(hip_gelu=[], lt_gelu=[])
        for _ in range(ROUNDS):
            res["hip"].append(timeit(lambda: G.gemm_nt(a, b)))
            res["lt"].append(timeit(lambda: torch.mm(a, b.t())))
            if extra:
                res["hip_gelu"].append(timeit(lambda: G.gemm_nt_gelu(a, b, bias)))
                res["lt_gelu"].append(timeit(lambda: bias_gelu(torch.mm(a, b.t()), bias)))
        r = {k: min(v) for k, v in res.items()}
        out(case=f"nt_{name}", M=M, N=N, K=K, ms=r,
            tflops={k: round(fl / v / 1e9, 1) for k, v in r.items() if "gelu" not in k})
        del a, b
    # weight gradients dW [N_out, K_in] = dY[T, N_out]^T X[T, K_in]
    tt_shapes = {"qkv": (3 * d, d), "attn_proj": (d, d), "fc": (4 * d, d), "fc_proj": (d, 4 * d)}
    for name, (No, Ki) in tt_shapes.items():
        if ONLY and ONLY not in name:
            continue
        dy = torch.randn(TOK, No, device=dev).bfloat16()
        x = torch.randn(TOK, Ki, device=dev).bfloat16()
        fl = 2.0 * TOK * No * Ki
        res = {"hip": [], "lt": []}
        for _ in range(ROUNDS):
            res["hip"].append(timeit(lambda: G.gemm_tt(dy, x)))
            res["lt"].append(timeit(lambda: torch.mm(dy.t(), x)))
        r = {k: min(v) for k, v in res.items()}
        out(case=f"tt_{name}", M=No, N=Ki, K=TOK, splits=G.tt_splits(No, Ki, TOK), ms=r,
            tflops={k: round(fl / v / 1e9, 1) for k, v in r.items()})
        del dy, x


if __name__ == "__main__":
    t0 = time.time()
    if os.environ.get("CHECK", "1") == "1":
        check()
    if os.environ.get("BENCH", "1") == "1":
        bench()
    out(case="done", s=round(time.time() - t0, 1))
