#!/usr/bin/env python
"""Host cost of the reducers' gradient-readiness hooks (parallel/_readiness.py), one process, no collectives:
backward of a model with 330 parameter tensors (SwinIR-S's count) and trivial compute, with (a) no hooks,
(b) per-parameter Python post-accumulate hooks over the native ReadyTracker, (c) C++ AccumulateGrad post hooks
(csrc/hooks/reducer_hooks.cpp) that enter Python once per ready bucket.  Interleaved rounds, medians."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pytorch_distributedtraining_amd.parallel import _readiness as R  # noqa: E402

N, D, BUCKETS = 330, 64, 10
torch.manual_seed(0)
torch.set_num_threads(1)
ps = [torch.nn.Parameter(torch.randn(D)) for _ in range(N)]
x = torch.randn(D)
buckets = [list(range(N - 1 - i, -1, -BUCKETS)) for i in range(BUCKETS)]   # any partition works


def bwd_ms(rd, iters=40):
    ts = []
    for _ in range(iters):
        loss = torch.stack([(p * x).sum() for p in ps]).sum()
        t0 = time.perf_counter()
        loss.backward()
        ts.append(time.perf_counter() - t0)
        if rd is not None:
            rd.reset()        # what the engine's end-of-backward callback does
        for p in ps:
            p.grad = None
    return statistics.median(ts) * 1e3


calls = {"n": 0}


def on_first():
    calls["n"] += 1


def on_ready(b):
    calls["n"] += 1


res = {"none": [], "python": [], "native": [], "native_off": []}
for rnd in range(15):
    for kind in ("none", "python", "native", "native_off"):
        rd = None
        if kind != "none":
            os.environ["PDT_NATIVE_HOOKS"] = "0" if kind == "python" else "1"
            R._hooks_mod = None
            rd = R.Readiness(ps, buckets, on_first, on_ready)
            assert rd.kind == kind.split("_")[0], rd.kind
            rd.set_enabled(kind != "native_off")
        calls["n"] = 0
        t = bwd_ms(rd)
        if rd is not None:
            rd.reset()
            rd.remove()
        res[kind].append(t)
med = {k: round(statistics.median(v), 3) for k, v in res.items()}
print(f"backward ms, median of 15 rounds x 40 passes ({N} params, {BUCKETS} buckets): {med}")
print(f"hook overhead per backward: python {med['python'] - med['none']:.3f} ms, "
      f"native {med['native'] - med['none']:.3f} ms (disabled: {med['native_off'] - med['none']:.3f} ms)")
