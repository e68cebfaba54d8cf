#!/usr/bin/env python
"""Phase shares of the hand-scheduled GEMM (diagnostic build, gemm.hip DIAG stamps): per item the main loop
(prologue wait included) and the epilogue, in shader cycles, plus the gap between a workgroup's items; the clock
from s_memtime / s_memrealtime (100 MHz).  Shares only -- the stamps' waits change the kernel."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import _lib  # noqa: E402

dev = torch.device("cuda")
TOK = int(os.environ.get("TOK", str(96 * 1024)))


def run(name, layout, M, N, K, ek=0):
    if layout == 0:
        a = torch.randn(M, K, device=dev).bfloat16()
        b = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        lda, ldb = K, K
    else:
        a = torch.randn(K, M, device=dev).bfloat16()
        b = torch.randn(K, N, device=dev).bfloat16()
        lda, ldb = M, N
    c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    items = (M // 256) * (N // 256)
    st = torch.zeros(items, 8, dtype=torch.int64, device=dev)
    bias = torch.randn(N, device=dev).bfloat16()
    aux = torch.empty_like(c) if ek == 2 else None
    for _ in range(3):
        _lib.call("pdt_gemm_stamps_epi_bf16", layout, ek, a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, lda,
                  ldb, bias.data_ptr() if ek else None, aux.data_ptr() if aux is not None else None, st.data_ptr(),
                  _lib.stream_handle(dev))
    torch.cuda.synchronize()
    s = st.cpu().double()
    loop = s[:, 1] - s[:, 0]
    epi = s[:, 2] - s[:, 1]
    T = K // 64
    cus = min(256, items)
    # per workgroup: items id, id + grid, ...: gap = next item's start - this item's end
    grid = cus & ~7 if cus >= 8 else cus
    gaps = []
    for g in range(grid):
        ids = list(range(g, items, grid))
        for x, y in zip(ids, ids[1:]):
            gaps.append(float(s[y, 0] - s[x, 2]))
    # clock: cycles per realtime tick over the whole run of one workgroup
    ids = list(range(0, items, grid))
    clk = float((s[ids[-1], 0] - s[ids[0], 0]) / max(1.0, float(s[ids[-1], 3] - s[ids[0], 3])) * 100e6) if len(ids) > 1 else 0.0
    # inside the main loop: T0 asm start, T1 prologue wait done, T2 first K-step done, T3 tail entry
    pre = s[:, 4] - s[:, 0]
    pro = s[:, 5] - s[:, 4]
    k0 = s[:, 6] - s[:, 5]
    mid = (s[:, 7] - s[:, 6]) / max(1, T - 3)
    tail = (s[:, 1] - s[:, 7]) / 2
    later = torch.arange(items) >= grid          # items whose tiles 0 / 1 the previous item issued
    def med(x, sel=None):
        x = x if sel is None else x[sel]
        return float(x.median()) if x.numel() else None
    out_ph = {"pre_asm_cyc": med(pre), "prologue_wait_cyc_first_item": med(pro, ~later),
              "prologue_wait_cyc_later_items": med(pro, later), "kstep0_cyc": med(k0),
              "kstep0_cyc_later_items": med(k0, later), "steady_kstep_cyc": med(mid), "tail_kstep_cyc": med(tail)}
    out = {"case": name, "epi": ek, "shape": [M, N, K], "items": items, "k_steps": T, **out_ph,
           "loop_cyc_median": float(loop.median()), "loop_cyc_per_kstep": float(loop.median()) / T,
           "epi_cyc_median": float(epi.median()), "epi_cyc_p90": float(epi.quantile(0.9)),
           "gap_cyc_median": float(torch.tensor(gaps).median()) if gaps else None, "clock_hz": clk}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    d = 2048
    if os.environ.get("EPI_ONLY"):      # the c_fc shape with the plain, bias and GELU epilogues
        for e in (0, 1, 2):
            run(f"nt_fc_epi{e}", 0, TOK, 4 * d, d, e)
        sys.exit(0)
    run("nt_fc", 0, TOK, 4 * d, d)
    run("nt_fc_proj", 0, TOK, d, 4 * d)
    run("nt_attn_proj", 0, TOK, d, d)
    run("nt_sq8k", 0, 8192, 8192, 8192)
    run("tt_fc", 1, 4 * d, d, TOK)
    # the same products with operands small enough to stay in the 256 MB Infinity Cache across the repeated
    # launches: is the long-K steady K-step bound by HBM latency (A streamed once) or by the loop itself?
    run("tt_fc_k8k_cached", 1, 4 * d, d, 8192)
    run("nt_fc_proj_m8k_cached", 0, 8192, d, 4 * d)
