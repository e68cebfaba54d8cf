#!/usr/bin/env python
"""Counterpart of the reference's Stoke-DDP.py on this framework's Trainer facade.

    python -m pytorch_distributedtraining_amd.launch --nproc-per-node 4 examples/stoke_ddp.py --batchSize 18
    python examples/stoke_ddp.py --cpu --nEpochs 1 --samples 32       # single process, CPU smoke

Same model and options as the reference: SwinIR-S x2 (910,152 params), perceptual feat_loss,
StokeOptimizer(AdamW lr 1e-3, betas (0.9, 0.99), eps 1e-8, wd), AMPConfig(init_scale=2**14),
DDPConfig(convert_to_sync_batch_norm=True), FairscaleOSSConfig(broadcast_fp16=True), ddp + OSS +
ShardedDDP, grad_accum_steps=2, ClipGradNormConfig(max_norm=grad_clip, norm_type=2), OneCycleLR +
ReduceLROnPlateau, per-epoch train / validate / save_checkpoint, EMA-loss printing, MAE/PSNR.
Differences (reference quirks NOT reproduced): seeded split identical on all ranks,
set_epoch called, ReduceLROnPlateau actually stepped with the val loss, --start-epoch resumes from the
latest checkpoint, --lr is honoured, metrics go to a rank-0 JSONL sink (W&B optional, never a
retry-forever login), validation metrics are averaged across ranks.  Precision defaults to bf16 on
MI355X (--fp16 amp selects fp16 + loss scaling with the AMPConfig above).  Data: synthetic LR/HR
patches unless --inputDir/--targetDir point at image folders (no network access here).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch import optim  # noqa: E402

from pytorch_distributedtraining_amd.data import DistributedSampler, PairedImageDataset, SyntheticSRDataset, random_split  # noqa: E402,E501
from pytorch_distributedtraining_amd.models import metrics  # noqa: E402
from pytorch_distributedtraining_amd.models.losses import feat_loss  # noqa: E402
from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2  # noqa: E402
from pytorch_distributedtraining_amd.trainer import (AMPConfig, ClipGradNormConfig, DDPConfig, DistributedOptions,  # noqa: E402,E501
                                                     FairscaleOSSConfig, StokeOptimizer, Trainer)
from pytorch_distributedtraining_amd.utils import checkpoint as ckpt  # noqa: E402
from pytorch_distributedtraining_amd.utils.dist import env_int  # noqa: E402
from pytorch_distributedtraining_amd.utils.logging import MetricsSink  # noqa: E402


def parse():
    p = argparse.ArgumentParser(description="SwinIR-S x2 DDP + ZeRO training (Stoke-DDP.py counterpart)")
    p.add_argument("--projectName", default="SwinIR-S-x2")
    p.add_argument("--batchSize", type=int, default=18)
    p.add_argument("--nEpochs", type=int, default=10)
    p.add_argument("--start-epoch", type=int, default=1)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--weight_decay", "--wd", type=float, default=1e-4)
    p.add_argument("--grad_clip", type=float, default=0.1)
    p.add_argument("--local_rank", "--local-rank", type=int, default=None)
    p.add_argument("--threads", type=int, default=0)
    p.add_argument("--inputDir", default=None)
    p.add_argument("--targetDir", default=None)
    p.add_argument("--samples", type=int, default=512, help="synthetic dataset size")
    p.add_argument("--lr-size", type=int, default=64, help="synthetic LR patch size (reference: 128)")
    p.add_argument("--fp16", default="bf16", choices=["bf16", "amp", "none"])
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--ckpt-dir", default="checkpoint/")
    p.add_argument("--metrics", default="runs/stoke_ddp_metrics.jsonl")
    p.add_argument("--wandb", action="store_true")
    p.add_argument("--pretrained", default=None,
                   help="SwinIR checkpoint to start from, e.g. model_zoo/002_lightweightSR_DIV2K_s64w8_SwinIR-S_x2.pth "
                        "({'params': sd} or a raw state dict, strict key match; Stoke-DDP.py:209-213)")
    return p.parse_args()


def train(loader, t: Trainer, sched1, epoch, sink):
    t.print_on_devices(f"Starting Epoch {epoch + 1}")
    t.model_access.train()
    loader.set_epoch(epoch)
    sum_loss, n = 0.0, 0
    for idx, (inputs, targets) in enumerate(loader):
        outputs = t.model(inputs)
        loss = t.loss(outputs, targets)
        t.backward(loss=loss)
        if t.step():            # scheduler advances per optimizer step (the reference stepped per micro-batch)
            sched1.step()
        if (idx + 1) % 10 == 0:
            t.print_ema_loss(prepend_msg=f"Step {idx + 1} -- EMA Loss")
        # lazy=True: a SyncedLoss -- the running sum stays on the device; the cross-rank mean and the host read
        # happen only when a log line reads it (Stoke-DDP.py:86 synced on every micro-batch; every rank reads it)
        sum_loss += t.detach_and_sync_loss(loss=loss, lazy=True) * t.grad_accum
        n += 1
        if (n + 1) % 50 == 0:
            sink.log({"train_loss": float(sum_loss / n), "epoch": epoch}, step=t.optimizer_steps)
    t.flush_prints()
    return float(sum_loss / max(n, 1))


def validate(loader, t: Trainer, epoch, sink):
    t.model_access.eval()
    vals = torch.zeros(4, dtype=torch.float64)
    with torch.no_grad():
        for inputs, targets in loader:
            outputs = t.model(inputs).float()
            vals += torch.tensor([float(t.loss(outputs, targets)), metrics.mae(outputs, targets),
                                  metrics.psnr(outputs, targets), 1.0], dtype=torch.float64)
    v = vals.to(t.device)
    t.comm.all_reduce(v, "sum")
    cnt = max(float(v[3]), 1.0)
    val_loss, mae, psnr = (float(v[i]) / cnt for i in range(3))
    sink.log({"val_loss": val_loss, "MAE": mae, "PSNR": psnr, "epoch": epoch}, step=t.optimizer_steps)
    t.print_on_devices(f"Current Average Validation Loss: {val_loss:.5f}, PSNR : {psnr:.3f}, MAE : {mae:.5f}")
    return val_loss


def main():
    opt = parse()
    if opt.local_rank is not None:
        os.environ.setdefault("LOCAL_RANK", str(opt.local_rank))
    world = env_int("WORLD_SIZE", 1)
    gpu = not opt.cpu and torch.cuda.is_available()

    amp_config = AMPConfig(init_scale=2.0 ** 14)
    ddp_config = DDPConfig(local_rank=env_int("LOCAL_RANK", 0), convert_to_sync_batch_norm=True)
    oss_config = FairscaleOSSConfig(broadcast_fp16=True)

    model = swinir_s_x2()
    if opt.pretrained:
        # every rank reads the file before the engines sync rank 0's weights (weights_only: no pickle exec)
        ckpt.load_pretrained(model, opt.pretrained, key="params", strict=True)
    optimizer = StokeOptimizer(optimizer=torch.optim.AdamW,
                               optimizer_kwargs={"lr": opt.lr, "betas": (0.9, 0.99), "eps": 1e-8,
                                                 "weight_decay": opt.weight_decay})
    dist_opt = DistributedOptions.ddp.value if world > 1 else None
    t = Trainer(model=model, verbose=True, optimizer=optimizer, loss=feat_loss, batch_size_per_device=opt.batchSize,
                gpu=gpu, fp16=None if opt.fp16 == "none" else opt.fp16, distributed=dist_opt,
                fairscale_oss=world > 1, fairscale_sddp=world > 1, grad_accum_steps=2,
                configs=[amp_config, ddp_config, oss_config],
                grad_clip=ClipGradNormConfig(max_norm=opt.grad_clip, norm_type=2.0))

    if opt.inputDir and opt.targetDir and os.path.isdir(opt.inputDir):
        full = PairedImageDataset(opt.inputDir, opt.targetDir)
    else:
        full = SyntheticSRDataset(n=opt.samples, lr_size=opt.lr_size, scale=2)
    train_ds, val_ds = random_split(full, [0.9, 0.1], seed=0)
    train_dl = t.DataLoader(dataset=train_ds, sampler=DistributedSampler(train_ds, t.world_size, t.rank),
                            num_workers=opt.threads, drop_last=True)
    val_dl = t.DataLoader(dataset=val_ds, sampler=DistributedSampler(val_ds, t.world_size, t.rank, shuffle=False),
                          num_workers=0)
    sched1 = optim.lr_scheduler.OneCycleLR(t.optimizer, max_lr=0.01, pct_start=0.9,
                                           steps_per_epoch=max(1, len(train_dl) // 2), epochs=opt.nEpochs)
    sched2 = optim.lr_scheduler.ReduceLROnPlateau(t.optimizer, mode="min", factor=0.2, patience=2, min_lr=5e-5)
    sink = MetricsSink(opt.metrics, wandb_project=opt.projectName if opt.wandb else None,
                       config={"epochs": opt.nEpochs, "batch_size": opt.batchSize, "lr": opt.lr,
                               "dataset": "synthetic" if not opt.inputDir else opt.inputDir, "architecture": "SwinIR-S"})

    start = 0
    if opt.start_epoch > 1:
        tag = ckpt.latest_checkpoint(opt.ckpt_dir)
        if tag is not None:
            extras = t.load(opt.ckpt_dir, tag) or {}
            start = int(extras.get("epoch", 0)) + 1
            t.print_on_devices(f"resumed from {tag} at epoch {start}")

    for epoch in range(start, opt.nEpochs):
        tl = train(train_dl, t, sched1, epoch, sink)
        vl = validate(val_dl, t, epoch, sink)
        sched2.step(vl)
        t.save(path=opt.ckpt_dir, name=f"model_{epoch}_{tl:.2f}_{vl:.2f}", extras={"epoch": epoch})
        t.print_on_devices(f"Epoch {epoch}: train loss {tl:.5f} val loss {vl:.5f}; checkpoint saved")
    sink.close()


if __name__ == "__main__":
    main()
