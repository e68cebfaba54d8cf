#!/usr/bin/env python
"""Kernel-level breakdown of the ResNet-50 DDP bench step (BASELINE.json secondary headline).

rocprofv3 is not usable for this model: under its preloaded tool library MIOpen falls back to its naive
convolution kernels (profiles/README.md).  This script instead uses the in-process torch profiler (kineto
over the ROCm tracer) on the exact bench step -- same model, DDP wrapper, bf16 autocast, fused AdamW and
clip -- after the same MIOpen find warm-up, and checks that the profiled step's kernel time matches the
un-profiled step time (so no fallback happened).  Output: one JSON line per category (conv / BN+act /
GEMM / pooling / loss / optimizer / elementwise / copies) and the top kernels by device time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the MIOpen find/perf database recorded on MI355X (as bench.py): without it a fresh box spends minutes in find
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "tuning", "miopen"))
import torch  # noqa: E402

CATS = [  # (category, substrings of the lower-cased kernel name), first match wins
    ("bn_act", ("bn_", "batchnorm", "batch_norm")),
    ("optimizer", ("adamw", "multi_tensor", "clip", "norm_sq", "grad_norm")),
    ("gemm", ("cijk", "gemm_kernel", "matmul")),          # hipBLASLt: ResNet's channels-last 1x1 convs as GEMMs
    ("conv", ("conv", "igemm", "miopen", "winograd", "naive", "implicit", "wrw", "xdlops", "gridwise", "ck::",
              "device_grouped", "subtensorop")),
    ("loss", ("softmax", "nll", "cross_entropy")),
    ("pooling", ("pool",)),
    ("copy_cast", ("copy", "cast", "convert", "transpose", "fill", "memset", "memcpy")),
    ("elementwise", ("elementwise", "vectorized", "unrolled", "reduce", "add", "mul", "relu")),
]


def category(name: str) -> str:
    n = name.lower()
    for cat, keys in CATS:
        if any(k in n for k in keys):
            return cat
    return "other"


def main():
    from pytorch_distributedtraining_amd.models.resnet import resnet50
    from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_
    from pytorch_distributedtraining_amd.parallel.comm import Comm
    from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("gloo", rank=0, world_size=1)
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    mb = int(os.environ.get("MB", "256"))
    model = resnet50().to(dev).to(memory_format=torch.channels_last)
    # PDT_RESNET_AUTOCAST=0: the bf16 compute copy (bench.py's other arm) instead of fp32 weights under autocast
    autocast = os.environ.get("PDT_RESNET_AUTOCAST", "1") == "1"
    model = DistributedDataParallel(model, comm=Comm(), reduce_dtype=torch.bfloat16,
                                    compute_dtype=None if autocast else torch.bfloat16)
    params = model.optimizer_parameters()
    opt = FusedAdamW(params, lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    x = torch.randn(mb, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    if not autocast:
        x = x.bfloat16()
    y = torch.randint(0, 1000, (mb,), device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            loss = crit(model(x).float(), y)
        loss.backward()
        _, coef, _ = clip_grad_norm_(params, 1.0, comm=model.comm, sharded=False, apply=False)
        opt.step(grad_scale=coef)
        opt.zero_grad(set_to_none=True)

    for i in range(4):                       # MIOpen find + allocator warm-up
        step()
        torch.cuda.synchronize()
        print(json.dumps({"warmup_step": i}), flush=True)
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) * 1000 / n
    print(json.dumps({"autocast": autocast}), flush=True)
    print(json.dumps({"unprofiled_step_ms": round(step_ms, 3), "samples_per_s": round(mb * 1000 / step_ms, 1)}),
          flush=True)

    from torch.profiler import ProfilerActivity, profile
    steps = 3
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    kern = {}
    for ev in prof.events():
        if getattr(ev, "device_type", None) is None or str(ev.device_type) != "DeviceType.CUDA":
            continue
        us = ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
        k = kern.setdefault(ev.name, [0.0, 0])
        k[0] += us
        k[1] += 1
    total_us = sum(v[0] for v in kern.values()) / steps
    cats = {}
    for name, (us, cnt) in kern.items():
        c = category(name)
        e = cats.setdefault(c, [0.0, 0])
        e[0] += us / steps
        e[1] += cnt // steps
    print(json.dumps({"profiled_kernel_ms_per_step": round(total_us / 1000, 3),
                      "kernel_time_vs_unprofiled_step": round(total_us / 1000 / step_ms, 3)}), flush=True)
    for c, (us, cnt) in sorted(cats.items(), key=lambda kv: -kv[1][0]):
        print(json.dumps({"category": c, "ms_per_step": round(us / 1000, 3), "share": round(us / total_us, 4),
                          "launches_per_step": cnt}), flush=True)
    for name, (us, cnt) in sorted(kern.items(), key=lambda kv: -kv[1][0])[:40]:
        print(json.dumps({"kernel": name[:160], "category": category(name), "ms_per_step": round(us / steps / 1000, 3),
                          "calls_per_step": cnt // steps}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
