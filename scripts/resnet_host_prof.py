#!/usr/bin/env python
"""Host side of the ResNet-50 DDP bench step (BASELINE.json secondary): the bench's exact step (DDP, bf16
autocast, fused AdamW + clip) after the MIOpen find warm-up, then (1) the un-profiled ms/step, (2) the host's
own time per step (step() calls back to back with the device queue kept shallow by an event wait two steps
behind), (3) torch-profiler CPU self time per op over 3 steps -- where the host spends the time that leaves
the GPU idle between kernels."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "tuning", "miopen"))
import torch  # noqa: E402

from pytorch_distributedtraining_amd.models.resnet import resnet50  # noqa: E402
from pytorch_distributedtraining_amd.optim import FusedAdamW, clip_grad_norm_  # noqa: E402
from pytorch_distributedtraining_amd.parallel import Comm  # noqa: E402
from pytorch_distributedtraining_amd.parallel.ddp import DistributedDataParallel  # noqa: E402

dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
mb = int(os.environ.get("MB", "256"))
comm = Comm()
model = resnet50().to(dev).to(memory_format=torch.channels_last)
x = torch.randn(mb, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (mb,), device=dev)
model = DistributedDataParallel(model, comm=comm, reduce_dtype=torch.bfloat16)
params = model.optimizer_parameters()
opt = FusedAdamW(params, lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
crit = torch.nn.CrossEntropyLoss()


def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = crit(model(x).float(), y)
    loss.backward()
    _, coef, _ = clip_grad_norm_(params, 1.0, comm=comm, sharded=False, apply=False)
    opt.step(grad_scale=coef)
    opt.zero_grad(set_to_none=True)


for _ in range(3):
    step()
torch.cuda.synchronize()
n = 10
t0 = time.perf_counter()
for _ in range(n):
    step()
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / n * 1e3
# host-only time: keep at most ~1 step queued so the host never blocks on a full queue
evs = []
host = []
for _ in range(n):
    if len(evs) >= 1:
        evs.pop(0).synchronize()
    h0 = time.perf_counter()
    step()
    host.append((time.perf_counter() - h0) * 1e3)
    e = torch.cuda.Event()
    e.record()
    evs.append(e)
torch.cuda.synchronize()
print(json.dumps({"ms_per_step": round(gpu_ms, 3), "samples_per_s": round(mb / gpu_ms * 1e3, 1),
                  "host_ms_per_step_median": round(sorted(host)[len(host) // 2], 3)}), flush=True)
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU]) as p:
    for _ in range(3):
        step()
    torch.cuda.synchronize()
print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=45), flush=True)
