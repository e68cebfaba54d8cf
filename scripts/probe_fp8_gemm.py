#!/usr/bin/env python
"""Probe: does torch._scaled_mm run OCP fp8 (e4m3fn / e5m2) GEMMs on this gfx950 stack, and how fast vs bf16?"""
import json
import torch

dev = "cuda"
torch.manual_seed(0)


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for (M, N, K) in ((32768, 6144, 2048), (32768, 2048, 8192), (32768, 8192, 2048)):
    a = torch.randn(M, K, device=dev)
    b = torch.randn(N, K, device=dev)
    ref = a @ b.t()
    one = torch.ones((), device=dev)
    for dta, dtb in ((torch.float8_e4m3fn, torch.float8_e4m3fn), (torch.float8_e5m2, torch.float8_e4m3fn)):
        try:
            aq, bq = a.to(dta), b.to(dtb)
            y = torch._scaled_mm(aq, bq.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            err = float((y.float() - ref).norm() / ref.norm())
            ms = timed(lambda: torch._scaled_mm(aq, bq.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
            print(json.dumps({"M": M, "N": N, "K": K, "a": str(dta), "b": str(dtb), "ok": True, "rel_err": round(err, 4),
                              "ms": round(ms, 4), "pflops": round(2 * M * N * K / ms / 1e12, 3)}), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"M": M, "N": N, "K": K, "a": str(dta), "b": str(dtb), "ok": False, "err": str(e)[:300]}),
                  flush=True)
    ab, bb = a.bfloat16(), b.bfloat16()
    ms = timed(lambda: ab @ bb.t())
    print(json.dumps({"M": M, "N": N, "K": K, "a": "bf16", "ms": round(ms, 4), "pflops": round(2 * M * N * K / ms / 1e12, 3)}),
          flush=True)
