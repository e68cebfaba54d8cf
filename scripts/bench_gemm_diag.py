#!/usr/bin/env python
"""Where does the hand TT GEMM lose to peak?  Times csrc/kernels/gemm.hip's weight-gradient kernel at the GPT-2
1.3B c_fc shape (dW [8192, 2048] over 98,304 tokens) against diagnostic builds of the same main loop with one
component removed (pdt_gemm_diag_bf16; their outputs are garbage by construction): 1 = no LDS-DMA (MFMA +
LDS-read ceiling), 2 = DMA issued but never waited for (issue cost only), 3 = no LDS reads (MFMA + DMA)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.ops import _lib  # noqa: E402

lib = _lib.require()
T = int(os.environ.get("TOK", str(96 * 1024)))
dev = torch.device("cuda")
for M, N in ((8192, 2048), (2048, 8192), (6144, 2048)):
    a = torch.randn(T, M, device=dev).bfloat16()
    b = torch.randn(T, N, device=dev).bfloat16()
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = _lib.stream_handle(dev)
    res = {}
    for rnd in range(3):
        for d in (0, 1, 2, 3):
            def run():
                _lib.check(lib.pdt_gemm_diag_bf16(d, a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, T, st), "diag")
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            e1.synchronize()
            res.setdefault(d, []).append(e0.elapsed_time(e1) / 5)
    fl = 2.0 * M * N * T
    print(json.dumps({"M": M, "N": N, "K": T, **{f"diag{d}_tflops": round(fl / min(v) / 1e9, 1) for d, v in res.items()}}),
          flush=True)
    del a, b, c
