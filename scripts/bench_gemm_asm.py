#!/usr/bin/env python
"""Hand-scheduled GEMM main loop (gemm_asm_kernel, csrc/kernels/gen_gemm_kloop.py) against the compiler-scheduled
kernel (gemm_kernel) and hipBLASLt: (1) correctness -- bitwise equal to gemm_kernel for the plain epilogue (same
MFMA order per accumulator), close to fp32 torch for every epilogue; (2) interleaved timing rounds in one process
at the GPT-2 1.3B flagship shapes (96 x 1024 tokens) on random data.  One JSON line per case."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import gemm as G  # noqa: E402

dev = torch.device("cuda")
TOK = int(os.environ.get("TOK", str(96 * 1024)))
ROUNDS = int(os.environ.get("ROUNDS", "5"))
ONLY = os.environ.get("ONLY", "")
MODE = os.environ.get("MODE", "check,bench")


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def out(**kw):
    print(json.dumps(kw), flush=True)


def with_kernel(name, fn):
    old = G.KERNEL["name"]
    G.KERNEL["name"] = name
    try:
        return fn()
    finally:
        G.KERNEL["name"] = old


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
    for (M, N, K) in ((512, 512, 128), (2048, 1024, 1536), (1024, 768, 4096), (1024, 768, 4160), (1024, 768, 8192)):
        a = torch.randn(M, K, device=dev).bfloat16()
        b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device=dev).bfloat16()
        ref = a.float() @ b.float().t()
        c_asm = with_kernel("asm", lambda: G.gemm_nt(a, b))
        c_hip = with_kernel("hip", lambda: G.gemm_nt(a, b))
        torch.cuda.synchronize()
        out(case="nt_plain", shape=[M, N, K], rel=rel(c_asm, ref), bitwise_eq_hip=bool(torch.equal(c_asm, c_hip)))
        out(case="nt_bias", shape=[M, N, K],
            rel=rel(with_kernel("asm", lambda: G.gemm_nt(a, b, bias)), ref + bias.float()))
        y, dd = with_kernel("asm", lambda: G.gemm_nt_gelu(a, b, bias))
        hr = (ref + bias.float()).requires_grad_()
        yr = torch.nn.functional.gelu(hr, approximate="tanh")
        yr.sum().backward()
        out(case="nt_gelu", shape=[M, N, K], rel_dgelu=rel(dd, hr.grad), rel_y=rel(y, yr.detach()))
        h = torch.randn(M, N, device=dev).bfloat16()
        hr = h.float().requires_grad_()
        torch.nn.functional.gelu(hr, approximate="tanh").sum().backward()
        dh = hr.grad.bfloat16()
        g, db = with_kernel("asm", lambda: G.gemm_nt_dgelu(a, b, dh))
        want = ref * dh.float()
        out(case="nt_dgelu", shape=[M, N, K], rel_g=rel(g, want), rel_db=rel(db, want.sum(0)))
        at = torch.randn(K * 2, M, device=dev).bfloat16()
        bt = torch.randn(K * 2, N, device=dev).bfloat16()
        reft = at.float().t() @ bt.float()
        for s in (1, 2, 4):
            if (2 * K) // s < 128 or (2 * K) % (64 * s):
                continue
            t_asm = with_kernel("asm", lambda: G.gemm_tt(at, bt, splits=s))
            t_hip = with_kernel("hip", lambda: G.gemm_tt(at, bt, splits=s))
            out(case=f"tt_s{s}", shape=[M, N, 2 * K], rel=rel(t_asm, reft), bitwise_eq_hip=bool(torch.equal(t_asm, t_hip)))
    # K-step counts 6..11: every tail phase of the 3-stage program (T - 3 mod 6) and of the 2-stage one, both
    # layouts, bitwise against the compiler-scheduled kernel (run with PDT_GEMM_P3=1 to force the 3-stage program)
    for T in range(6, 12):
        K = 64 * T
        a = torch.randn(512, K, device=dev).bfloat16()
        b = (torch.randn(768, K, device=dev) * K ** -0.5).bfloat16()
        c_asm = with_kernel("asm", lambda: G.gemm_nt(a, b))
        c_hip = with_kernel("hip", lambda: G.gemm_nt(a, b))
        at = torch.randn(K, 512, device=dev).bfloat16()
        bt = torch.randn(K, 768, device=dev).bfloat16()
        t_asm = with_kernel("asm", lambda: G.gemm_tt(at, bt, splits=1))
        t_hip = with_kernel("hip", lambda: G.gemm_tt(at, bt, splits=1))
        out(case="tails", k_steps=T, nt_bitwise_eq_hip=bool(torch.equal(c_asm, c_hip)),
            tt_bitwise_eq_hip=bool(torch.equal(t_asm, t_hip)))
    # full grid at a flagship shape: every element against the compiler-scheduled kernel
    M, N, K = TOK, 2048, 2048
    a = torch.randn(M, K, device=dev).bfloat16()
    b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
    c_asm = with_kernel("asm", lambda: G.gemm_nt(a, b))
    c_hip = with_kernel("hip", lambda: G.gemm_nt(a, b))
    out(case="nt_fullgrid_flagship", shape=[M, N, K], bitwise_eq_hip=bool(torch.equal(c_asm, c_hip)),
        max_abs=float((c_asm.float() - c_hip.float()).abs().max()))
    at = torch.randn(M, 2048, device=dev).bfloat16()
    bt = torch.randn(M, 2048, device=dev).bfloat16()
    t_asm = with_kernel("asm", lambda: G.gemm_tt(at, bt))
    t_hip = with_kernel("hip", lambda: G.gemm_tt(at, bt))
    out(case="tt_fullgrid_flagship", shape=[2048, 2048, M], bitwise_eq_hip=bool(torch.equal(t_asm, t_hip)),
        max_abs=float((t_asm.float() - t_hip.float()).abs().max()))


def bench():
    torch.manual_seed(1)
    d = 2048
    nt = {"qkv": (TOK, 3 * d, d), "attn_proj": (TOK, d, d), "fc": (TOK, 4 * d, d), "fc_proj": (TOK, d, 4 * d),
          "qkv_dgrad": (TOK, d, 3 * d), "sq8k": (8192, 8192, 8192)}
    for name, (M, N, K) in nt.items():
        if ONLY and ONLY not in name:
            continue
        a = torch.randn(M, K, device=dev).bfloat16()
        b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device=dev).bfloat16()
        fl = 2.0 * M * N * K
        arms = {"asm": lambda: with_kernel("asm", lambda: G.gemm_nt(a, b)),
                "hip": lambda: with_kernel("hip", lambda: G.gemm_nt(a, b)),
                "lt": lambda: a @ b.t()}
        if name != "sq8k":
            arms["asm_bias"] = lambda: with_kernel("asm", lambda: G.gemm_nt(a, b, bias))
            arms["lt_bias"] = lambda: torch.nn.functional.linear(a, b, bias)
        if name == "fc":
            arms["asm_gelu"] = lambda: with_kernel("asm", lambda: G.gemm_nt_gelu(a, b, bias))
            h = torch.rand(M, N, device=dev).bfloat16()
            arms["asm_dgelu"] = lambda: with_kernel("asm", lambda: G.gemm_nt_dgelu(a, b, h))
            # the unfused alternative of the DGELU epilogue: plain GEMM, then the derivative-mode sweep (dy * d and
            # its column sums) that _LinearBiasGeluFn.backward runs
            from pytorch_distributedtraining_amd.ops import _lib
            lib = _lib.require()
            dpre, dbias = torch.empty_like(h), torch.empty(N, device=dev, dtype=torch.bfloat16)
            ws = torch.empty(lib.pdt_colsum_ws_floats(M, N), dtype=torch.float32, device=dev)

            def plain_sweep():
                c = with_kernel("asm", lambda: G.gemm_nt(a, b))
                _lib.call("pdt_bias_gelu_bwd_db", c.data_ptr(), h.data_ptr(), None, dpre.data_ptr(), dbias.data_ptr(),
                          ws.data_ptr(), M, N, 1, 1, 2, 0, _lib.stream_handle(dev))
            arms["asm_plain+sweep"] = plain_sweep
        res = {k: [] for k in arms}
        for _ in range(ROUNDS):
            for k, fn in arms.items():
                res[k].append(timeit(fn))
        out(case="nt_" + name, shape=[M, N, K],
            **{k: round(fl / (min(v) * 1e-3) / 1e12, 1) for k, v in res.items()}, unit="TFLOP/s (best of rounds)")
    tt = {"qkv": (3 * d, d), "attn_proj": (d, d), "fc": (4 * d, d), "fc_proj": (d, 4 * d)}
    for name, (N, K) in tt.items():
        if ONLY and ONLY not in name:
            continue
        a = torch.randn(TOK, N, device=dev).bfloat16()
        b = torch.randn(TOK, K, device=dev).bfloat16()
        fl = 2.0 * TOK * N * K
        s = G.tt_splits(N, K, TOK)
        arms = {"asm": lambda: with_kernel("asm", lambda: G.gemm_tt(a, b, splits=s)),
                "hip": lambda: with_kernel("hip", lambda: G.gemm_tt(a, b, splits=s)),
                "lt": lambda: a.t() @ b}
        res = {k: [] for k in arms}
        for _ in range(ROUNDS):
            for k, fn in arms.items():
                res[k].append(timeit(fn))
        out(case="tt_" + name, shape=[N, K, TOK], splits=s,
            **{k: round(fl / (min(v) * 1e-3) / 1e12, 1) for k, v in res.items()}, unit="TFLOP/s (best of rounds)")


if __name__ == "__main__":
    if "check" in MODE:
        check()
    if "bench" in MODE:
        bench()
