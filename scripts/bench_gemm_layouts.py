"""Weight-gradient GEMM formulations for the flagship shapes (GPT-2 1.3B, 32 x 1024 tokens per GPU):
dW[N, K] = dY[T, N]^T X[T, K].  Prints ms and TFLOP/s per formulation (hipBLASLt / rocBLAS choices differ
by operand layout).  Usage: python scripts/bench_gemm_layouts.py"""
import json
import sys

import torch

# default: flagship (GPT-2 1.3B, 32 x 1024 tokens); "small": GPT-2 124M DDP (16 x 1024 tokens)
if len(sys.argv) > 1 and sys.argv[1] == "small":
    T = 16384
    SHAPES = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (50304, 768)]
else:
    T = 32768
    SHAPES = [(6144, 2048), (2048, 2048), (8192, 2048), (2048, 8192), (50304, 2048)]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    for n, k in SHAPES:
        dy = torch.randn(T, n, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, k, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * n * k
        ref = torch.mm(dy.t(), x).float()
        cands = {
            "mm(dy.t, x)": lambda: torch.mm(dy.t(), x),
            "mm(x.t, dy).t": lambda: torch.mm(x.t(), dy).t(),
            "mm(dy.t, x) fp32out": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32),
            "bmm split2 fp32": lambda: torch.bmm(dy.view(2, T // 2, n).transpose(1, 2), x.view(2, T // 2, k),
                                                 out_dtype=torch.float32).sum(0),
            "dyT contiguous + mm": lambda: torch.mm(dy.t().contiguous(), x),
        }
        for sp in (4, 8):
            cands[f"bmm split{sp} fp32"] = (lambda sp=sp: torch.bmm(dy.view(sp, T // sp, n).transpose(1, 2),
                                                                    x.view(sp, T // sp, k),
                                                                    out_dtype=torch.float32).sum(0))
            cands[f"bmm split{sp} xT fp32"] = (lambda sp=sp: torch.bmm(x.view(sp, T // sp, k).transpose(1, 2),
                                                                       dy.view(sp, T // sp, n),
                                                                       out_dtype=torch.float32).sum(0).t())
        for name, fn in cands.items():
            try:
                out = fn()
                err = ((out.float() - ref).norm() / ref.norm()).item()
                ms = timeit(fn)
                print(json.dumps({"N": n, "K": k, "T": T, "form": name, "ms": round(ms, 4),
                                  "TFLOPs": round(fl / ms / 1e9, 1), "rel_err": round(err, 5)}), flush=True)
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"N": n, "K": k, "form": name, "error": str(ex)[:120]}), flush=True)


if __name__ == "__main__":
    main()
