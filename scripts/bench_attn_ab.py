#!/usr/bin/env python
"""A/B the flash-attention kernel generations in ONE process, interleaved rounds (cdna_hip_programming.md
§5.4 rule 24): forward and backward ms + TFLOP/s on the flagship (GPT-2 1.3B: B32 S1024 H16 D128 causal),
Llama-3 8B (B8 S1024 H32/8 D128 causal) and a long-sequence shape, plus the max |diff| of each variant's
output against the first one.  Usage: python scripts/bench_attn_ab.py --fwd 4,5 --bwd 3"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops import flash_attn  # noqa: E402
from pytorch_distributedtraining_amd.ops.attention import set_block_order, set_kernel_variant  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--fwd", default="4,5")
ap.add_argument("--bwd", default="3")
ap.add_argument("--order", default="0", help="workgroup block orders to try: 0 heavy-first, 1 XCD-grouped")
ap.add_argument("--shapes", default="", help="comma list of shape names (default: all)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
fwds = [int(x) for x in a.fwd.split(",")]
bwds = [int(x) for x in a.bwd.split(",")]
orders = [int(x) for x in a.order.split(",")]
SHAPES = [("gpt2-1.3b-b96", 96, 1024, 16, 16, 128, True), ("gpt2-1.3b", 32, 1024, 16, 16, 128, True), ("gpt2-1.3b-full", 32, 1024, 16, 16, 128, False),
          ("llama3-8b", 8, 1024, 32, 8, 128, True), ("long-4k", 8, 4096, 16, 16, 128, True),
          ("gpt2-124m", 64, 1024, 12, 12, 64, True)]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


torch.manual_seed(0)
for name, B, S, H, Hkv, D, causal in SHAPES:
    if a.shapes and name not in a.shapes.split(","):
        continue
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    flops = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
    combos = [(f, b, o) for o in orders for f in fwds for b in bwds]
    res = {c: {"fwd": [], "bwd": []} for c in combos}
    # fp32 reference on batch element 0 (all heads): each variant's max |err| and relative L2 error
    with torch.no_grad():
        qt, kt, vt = (t[:1].float().transpose(1, 2) for t in (q, k, v))
        kt, vt = kt.repeat_interleave(H // Hkv, 1), vt.repeat_interleave(H // Hkv, 1)
        sc = qt @ kt.transpose(-1, -2) / D ** 0.5
        if causal:
            sc = sc.masked_fill(~torch.ones(S, S, dtype=torch.bool, device="cuda").tril(), float("-inf"))
        oref = (sc.softmax(-1) @ vt).transpose(1, 2)
        del sc
    gref = None
    for c in combos:   # warm-up + numerics
        set_kernel_variant(c[0], c[1])
        set_block_order(c[2])
        with torch.no_grad():
            ofull = flash_attn(q, k, v, causal=causal)
            o = ofull[:1].float()
        # full-grid backward of every variant against the first one (races show up under full load)
        g = torch.autograd.grad(flash_attn(q, k, v, causal=causal), (q, k, v), do)
        if gref is None:
            gref, oref_full = g, ofull
        res[c]["o_full_max_diff_vs_first"] = round(float((ofull.float() - oref_full.float()).abs().max()), 5)
        res[c]["grad_max_rel_diff_vs_first"] = round(max(float((x.float() - y.float()).norm() / y.float().norm())
                                                     for x, y in zip(g, gref)), 6)
        del g
        err = (o - oref).abs()
        i = int(err.argmax())
        res[c]["o_max_err"] = round(float(err.max()), 5)
        res[c]["o_max_err_row"] = (i // (H * D)) % S
        res[c]["o_rel_err"] = round(float((o - oref).norm() / oref.norm()), 6)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for c in combos:
            set_kernel_variant(c[0], c[1])
            set_block_order(c[2])
            f = timed(lambda: flash_attn(q, k, v, causal=causal), a.iters)
            o = flash_attn(q, k, v, causal=causal)
            fb = timed(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), a.iters)
            res[c]["fwd"].append(f)
            res[c]["bwd"].append(fb)
    for c in combos:
        r = res[c]
        fm, bm = sorted(r["fwd"])[len(r["fwd"]) // 2], sorted(r["bwd"])[len(r["bwd"]) // 2]
        print(json.dumps({"shape": name, "fwd_variant": c[0], "bwd_variant": c[1], "order": c[2], "fwd_ms": round(fm, 4),
                          "fwd_tflops": round(flops / fm / 1e9, 1), "bwd_ms": round(bm, 4),
                          "bwd_tflops": round(2.5 * flops / bm / 1e9, 1),
                          **{k2: v2 for k2, v2 in r.items() if k2.startswith(("o_", "grad_"))}}), flush=True)
