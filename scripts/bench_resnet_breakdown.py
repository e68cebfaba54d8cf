"""Where does a ResNet-50 bf16 training step go?  Times forward+backward of the model as is, with every
BatchNorm replaced by Identity, and additionally with every ReLU replaced by Identity (CUDA events;
rocprofv3 is not usable here: under the profiler MIOpen falls back to its naive convolution kernels).
Also times our SyncBatchNorm kernels vs nn.BatchNorm2d on the largest activation shape."""
import json
import sys
import os

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def swap(m, cls, new):
    for name, ch in list(m.named_children()):
        if isinstance(ch, cls):
            setattr(m, name, new())
        else:
            swap(ch, cls, new)
    return m


def time_step(model, x, y, iters=10):
    crit = nn.CrossEntropyLoss()

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(model(x), y)
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        step()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    from pytorch_distributedtraining_amd.models.resnet import resnet50
    dev = torch.device("cuda")
    x = torch.randn(256, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (256,), device=dev)
    res = {}
    m = resnet50().to(dev).to(memory_format=torch.channels_last)
    res["full_fused_bn"] = time_step(m, x, y)
    m = resnet50(fused_bn=False).to(dev).to(memory_format=torch.channels_last)
    res["full_stock_bn"] = time_step(m, x, y)
    m = swap(resnet50(fused_bn=False), nn.BatchNorm2d, nn.Identity).to(dev).to(memory_format=torch.channels_last)
    res["no_bn"] = time_step(m, x, y)
    m = swap(swap(resnet50(fused_bn=False), nn.BatchNorm2d, nn.Identity), nn.ReLU, nn.Identity).to(dev)
    res["no_bn_no_relu"] = time_step(m.to(memory_format=torch.channels_last), x, y)
    print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
    # BN layer alone on the largest activation: [256, 256, 56, 56] bf16 channels_last
    from pytorch_distributedtraining_amd.parallel.syncbn import SyncBatchNorm
    a = torch.randn(256, 256, 56, 56, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    from pytorch_distributedtraining_amd.ops.batchnorm import BatchNormAct2d
    for name, bn in (("nn.BatchNorm2d", nn.BatchNorm2d(256).to(dev)), ("pdt SyncBatchNorm", SyncBatchNorm(256).to(dev)),
                     ("pdt BatchNormAct2d(relu)", BatchNormAct2d(256, act="relu").to(dev))):
        a.requires_grad_(True)

        def f():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                o = bn(a) if isinstance(bn, BatchNormAct2d) else torch.relu(bn(a))
            o.backward(torch.ones_like(o))
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"bn_relu_fwd_bwd": name, "ms": round(s.elapsed_time(e) / 10, 3),
                          "bytes_per_pass_MB": a.numel() * 2 / 1e6}), flush=True)


if __name__ == "__main__":
    main()
