#!/usr/bin/env python
"""Does a concurrent small kernel (what an RCCL collective is to the compute stream) delay a persistent kernel?

Persistent kernels here size their grid to one workgroup per CU with a static item list, and their workgroups
fill a CU (all VGPRs / LDS), so a CU held by another stream's kernel at launch time delays that workgroup's whole
item list.  Emulation on one GPU: S side streams each run torch.cuda._sleep (one spinning workgroup) for ~X us,
launched just before the GEMM on the main stream; the GEMM's main-stream time is compared with the GEMM alone,
for the persistent hand GEMM (asm) and hipBLASLt (one workgroup per tile).  One JSON line per case."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402

dev = torch.device("cuda")
M, N, K = 96 * 1024, 8192, 2048
a = torch.randn(M, K, device=dev).bfloat16()
b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
bias = torch.randn(N, device=dev).bfloat16()
main = torch.cuda.current_stream()
sides = [torch.cuda.Stream() for _ in range(int(os.environ.get("SIDES", "16")))]
SLEEP_CYC = int(os.environ.get("SLEEP_CYC", str(1_000_000)))   # ~0.4-0.7 ms at the loaded clock


def asm():
    old = G.KERNEL["name"]
    G.KERNEL["name"] = "asm"
    try:
        return G.gemm_nt(a, b, bias)
    finally:
        G.KERNEL["name"] = old


def lt():
    return torch.nn.functional.linear(a, b, bias)


def run(fn, contend, iters=10):
    times = []
    for _ in range(iters + 2):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if contend:
            for s in sides:
                with torch.cuda.stream(s):
                    torch.cuda._sleep(SLEEP_CYC)
        e0.record(main)
        fn()
        e1.record(main)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    times = sorted(times[2:])
    return times[len(times) // 2]


# the sleep kernel's own duration
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
torch.cuda._sleep(SLEEP_CYC)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"sleep_ms": round(e0.elapsed_time(e1), 3), "sides": len(sides)}), flush=True)
for name, fn in (("asm_bias", asm), ("hipblaslt_bias", lt)):
    t0 = run(fn, False)
    t1 = run(fn, True)
    print(json.dumps({"case": name, "shape": [M, N, K], "alone_ms": round(t0, 3), "with_side_kernels_ms": round(t1, 3),
                      "delay_ms": round(t1 - t0, 3)}), flush=True)
