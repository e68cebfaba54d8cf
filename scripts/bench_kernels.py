#!/usr/bin/env python
"""Per-kernel microbenchmarks on MI355X: our HIP kernels vs the stock PyTorch-ROCm op, same shapes
(GPT-2 1.3B training step shapes: 8 x 1024 tokens, d=2048, 16 heads x 128).  Prints one JSON line per
case: time (ms), achieved TFLOP/s or GB/s, and the speedup over torch."""
import argparse
import json
import math
import sys

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def report(name, ms, ref_ms=None, flops=None, bytes_=None):
    d = {"case": name, "ms": round(ms, 4)}
    if flops:
        d["TFLOPs"] = round(flops / ms / 1e9, 1)
    if bytes_:
        d["GBps"] = round(bytes_ / ms / 1e6, 1)
    if ref_ms:
        d["torch_ms"] = round(ref_ms, 4)
        d["speedup"] = round(ref_ms / ms, 2)
    print(json.dumps(d), flush=True)


def attn(B=8, S=1024, H=16, D=128, causal=True):
    from pytorch_distributedtraining_amd.ops import flash_attn
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    f = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
    o = flash_attn(q, k, v, causal=causal)
    ms_f = timeit(lambda: flash_attn(q, k, v, causal=causal))
    ms_b = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True))
    qt, kt, vt = (t.detach().transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
    ref = lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal)
    orf = ref()
    r_f = timeit(ref)
    dot = do.transpose(1, 2).contiguous()
    r_b = timeit(lambda: torch.autograd.grad(orf, (qt, kt, vt), dot, retain_graph=True))
    tag = f"B{B} S{S} H{H} D{D} {'causal' if causal else 'full'}"
    report(f"flash_attn fwd {tag}", ms_f, r_f, flops=f)
    report(f"flash_attn bwd {tag}", ms_b, r_b, flops=2.5 * f)


def attn_variants(B=16, S=1024, H=16, D=128):
    """dQ kernels of the backward side by side (GPT-2 1.3B mb16 layer shape): v3 (bwd 3) vs v4 (bwd 9)."""
    from pytorch_distributedtraining_amd.ops import flash_attn
    from pytorch_distributedtraining_amd.ops.attention import set_kernel_variant
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    for causal in (True, False):
        f = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
        o = flash_attn(q, k, v, causal=causal)
        grads = {}
        for var in (3, 9):
            set_kernel_variant(bwd=var)
            ms = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True))
            grads[var] = torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
            report(f"flash_attn bwd v{var} B{B} S{S} H{H} D{D} {'causal' if causal else 'full'}", ms, flops=2.5 * f)
        diff = max((a.float() - b.float()).abs().max().item() for a, b in zip(grads[3], grads[9]))
        print(json.dumps({"case": "bwd 3 vs 9 max abs diff", "causal": causal, "diff": diff}), flush=True)
    set_kernel_variant(bwd=-1)


def layernorm(rows=8192, N=2048):
    from pytorch_distributedtraining_amd.ops import layer_norm
    x = torch.randn(rows, N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn_like(x)
    y = layer_norm(x, w, b)
    yr = F.layer_norm(x, (N,), w, b)
    report(f"layernorm fwd {rows}x{N}", timeit(lambda: layer_norm(x, w, b)), timeit(lambda: F.layer_norm(x, (N,), w, b)),
           bytes_=2 * rows * N * 2)
    report(f"layernorm bwd {rows}x{N}", timeit(lambda: torch.autograd.grad(y, (x, w, b), dy, retain_graph=True)),
           timeit(lambda: torch.autograd.grad(yr, (x, w, b), dy, retain_graph=True)), bytes_=3 * rows * N * 2)


def adamw(n=164_000_000):
    from pytorch_distributedtraining_amd.ops import adamw_step
    p, m, v = (torch.randn(n, device="cuda") for _ in range(3))
    v.abs_()
    g = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    lp = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    ms = timeit(lambda: adamw_step([p], [g], [m], [v], lr=1e-4, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1,
                                   step=10, out_bf16=[lp]), iters=10)
    gf = g.float()
    ref = lambda: torch._fused_adamw_([p], [gf], [m], [v], [], [torch.tensor(10.0, device="cuda")], lr=1e-4,
                                      beta1=0.9, beta2=0.95, weight_decay=0.1, eps=1e-8, amsgrad=False, maximize=False)
    report(f"adamw flat {n/1e6:.0f}M (bf16 grad, bf16 copy-out)", ms, timeit(ref, iters=10), bytes_=n * (12 + 2 + 12 + 2))


def cross_entropy(rows=8192, V=50304):
    from pytorch_distributedtraining_amd.ops import cross_entropy as ce
    x = torch.randn(rows, V, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    t = torch.randint(0, V, (rows,), device="cuda")
    def ours():
        l = ce(x, t)
        l.backward()
    def ref():
        l = F.cross_entropy(x.float(), t)
        l.backward()
    report(f"cross_entropy fwd+bwd {rows}x{V}", timeit(ours, iters=10), timeit(ref, iters=10), bytes_=3 * rows * V * 2)


def bias_gelu(rows=32768, N=8192):
    from pytorch_distributedtraining_amd.ops import bias_gelu
    h = torch.randn(rows, N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn_like(h)
    def ours():
        y = bias_gelu(h, b)
        torch.autograd.grad(y, (h, b), dy)
    def ref():
        y = F.gelu(h + b, approximate="tanh")
        torch.autograd.grad(y, (h, b), dy)
    report(f"bias_gelu fwd+bwd {rows}x{N}", timeit(ours), timeit(ref), bytes_=5 * rows * N * 2)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    torch.manual_seed(0)
    cases = {"attn": lambda: (attn(), attn(S=2048, B=4), attn(D=64, H=12, B=8, S=1024), attn(causal=False)),
             "attnvar": attn_variants,
             "ln": layernorm, "adamw": adamw, "ce": cross_entropy, "gelu": bias_gelu}
    for k, fn in cases.items():
        if a.only and k not in a.only.split(","):
            continue
        try:
            fn()
        except Exception as e:  # keep going: report the failure
            print(json.dumps({"case": k, "error": repr(e)[:300]}), flush=True)
