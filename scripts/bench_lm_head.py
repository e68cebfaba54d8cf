#!/usr/bin/env python
"""GPT-2 1.3B tied LM head at the flagship shape (96 x 1024 tokens, 2048 -> 50,304 vocab): time each GEMM of
its forward / backward on the paths ``ops.linear`` can take, to find which kernels of the step's hipBLASLt rows
belong to the head.  One JSON line per measurement (ms, TFLOP/s)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402
from pytorch_distributedtraining_amd.ops import linear as L  # noqa: E402

M, D, V = 96 * 1024, 2048, 50304
dev = "cuda"
x = torch.randn(M, D, device=dev, dtype=torch.bfloat16)
w = (torch.randn(V, D, device=dev) / 45).bfloat16()
dl = (torch.randn(M, V, device=dev) / 100).bfloat16()
nm = V // 256 * 256


def t(fn, it=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it


def rep(name, ms, flops):
    print(json.dumps({"case": name, "ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1)}), flush=True)


full = 2.0 * M * D * V
if os.environ.get("LM_WGRAD_ONLY") == "1":       # the hand TT part alone, per token split (P3 via PDT_GEMM_P3)
    out = torch.empty(V, D, dtype=torch.bfloat16, device=dev)
    for sp in (1, 2, 4):
        rep(f"wgrad_asm_part_s{sp}_p3={os.environ.get('PDT_GEMM_P3', 'auto')}",
            t(lambda: G.gemm_tt(dl[:, :nm], x, sp, out=out[:nm])), 2.0 * M * D * nm)
    sys.exit(0)
wt = L.transpose16(w)
rep("fwd_F.linear", t(lambda: torch.nn.functional.linear(x, w)), full)
rep("dgrad_mm_NN", t(lambda: torch.mm(dl, w)), full)
rep("dgrad_F.linear_wT", t(lambda: torch.nn.functional.linear(dl, wt)), full)
rep("dgrad_asm_nt_wT", t(lambda: G.gemm_nt(dl, wt)), full)
rep("transpose16_w", t(lambda: L.transpose16(w)), 0)
rep("wgrad_library", t(lambda: L._library_wgrad(dl, x, torch.bfloat16)), full)
rep("wgrad_ragged_total", t(lambda: L.hip_wgrad_ragged(dl, x)), full)
s = L.hip_wgrad_splits(M, nm, D)
out = torch.empty(V, D, dtype=torch.bfloat16, device=dev)
rep(f"wgrad_ragged_asm_part_s{s}", t(lambda: G.gemm_tt(dl[:, :nm], x, s, out=out[:nm])), 2.0 * M * D * nm)
rep("wgrad_ragged_mm_rest", t(lambda: torch.mm(dl[:, nm:].t(), x, out=out[nm:])), 2.0 * M * D * (V - nm))
rep("wgrad_rest_library_split", t(lambda: L._library_wgrad(dl[:, nm:].contiguous(), x, torch.bfloat16)),
    2.0 * M * D * (V - nm))
rest = dl[:, nm:].contiguous()
rep("wgrad_rest_bmm16", t(lambda: torch.bmm(rest.view(16, M // 16, V - nm).transpose(1, 2), x.view(16, M // 16, D),
                                              out_dtype=torch.float32).sum(0)), 2.0 * M * D * (V - nm))
rep("rest_contiguous_copy", t(lambda: dl[:, nm:].contiguous()), 0)
print("choice", L._WGRAD_CHOICE, flush=True)
