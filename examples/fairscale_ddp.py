#!/usr/bin/env python
"""Counterpart of the reference's Fairscale-DDP.py on this framework.

Same workload and options: N local processes (mp.spawn style, 127.0.0.1 + free port), the SR CNN
``Net(upscale_factor=2)``, MSELoss, AdamW(lr 1e-3, betas (0.9, 0.99), eps 1e-8, wd 1e-4) wrapped in
ZeRO-1 ``OSS`` + ZeRO-2 ``ShardedDataParallel``, DistributedSampler, loss printed every 25 iterations.
Fixed reference quirks: sampler replicas/rank come from the process group (not hard-coded 4), the split
is seeded identically on every rank, set_epoch is called, and the GPU path uses RCCL.
Data: synthetic LR/HR patches (--lr-size 256 -> HR 512 reproduces the reference shapes; smaller by
default so it runs on CPU in seconds).

    python examples/fairscale_ddp.py --world-size 4 --epochs 2            # CPU / gloo, like the reference
    python examples/fairscale_ddp.py --world-size 1 --gpu                 # one MI355X
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402

from pytorch_distributedtraining_amd.data import DeviceDataLoader, DistributedSampler, SyntheticSRDataset, random_split  # noqa: E402,E501
from pytorch_distributedtraining_amd.launch import spawn  # noqa: E402
from pytorch_distributedtraining_amd.models.srnet import Net  # noqa: E402
from pytorch_distributedtraining_amd.parallel.zero import OSS, ShardedDataParallel  # noqa: E402


def train(rank, world_size, args):
    gpu = args.gpu and torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(rank)
    dist.init_process_group("nccl" if gpu else "gloo", init_method="env://", rank=rank, world_size=world_size)
    dev = torch.device("cuda", rank) if gpu else torch.device("cpu")
    print(f"Rank {rank} initialized")

    full = SyntheticSRDataset(n=args.samples, lr_size=args.lr_size, scale=2)
    train_ds, val_ds = random_split(full, [0.99, 0.01], seed=0)
    sampler = DistributedSampler(train_ds, num_replicas=world_size, rank=rank, shuffle=True)
    loader = DeviceDataLoader(train_ds, batch_size=args.batch, sampler=sampler, device=dev, drop_last=True,
                              num_workers=args.workers)
    x0, y0 = next(iter(loader))
    if rank == 0:
        print("train batch", tuple(x0.shape), "->", tuple(y0.shape))

    model = Net(upscale_factor=2).to(dev)
    loss_fn = nn.MSELoss()
    base_optimizer_arguments = {"lr": 1e-3, "betas": (0.9, 0.99), "eps": 1e-8, "weight_decay": 1e-4}
    optimizer = OSS(params=model.parameters(), optim=torch.optim.AdamW if not gpu else None,
                    **base_optimizer_arguments)
    model = ShardedDataParallel(model, optimizer)

    for e in range(args.epochs):
        sampler.set_epoch(e)
        model.train()
        for it, (x, y) in enumerate(loader, 1):
            model.zero_grad()
            loss = loss_fn(model(x), y)
            loss.backward()
            optimizer.step()
            if it % 25 == 0 or it == len(loader):
                print(f"rank {rank} epoch {e} iter {it}/{len(loader)} loss {loss.item():.5f}", flush=True)
        print(f"rank {rank} epoch {e} done, loss {loss.item():.5f}")
    dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world-size", type=int, default=4)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch", type=int, default=40)
    ap.add_argument("--samples", type=int, default=400)
    ap.add_argument("--lr-size", type=int, default=32)
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    spawn(train, a.world_size, args=(a.world_size, a))
