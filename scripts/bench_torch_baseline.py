#!/usr/bin/env python
"""Stock PyTorch-ROCm baseline for the flagship benchmark ("the comparison baseline is
stock PyTorch-ROCm DDP / FSDP over RCCL on the same MI355X node").

Same model shape (GPT-2 1.3B: L24, d2048, 16x128 heads, vocab 50304, seq 1024), same per-GPU batch,
same synthetic data and optimizer settings as ``bench.py``, but built only from stock components:
nn.Linear / nn.LayerNorm / F.scaled_dot_product_attention / F.gelu / F.cross_entropy,
torch.distributed.fsdp.FullyShardedDataParallel (FULL_SHARD, bf16 MixedPrecision) and
torch.optim.AdamW(fused=True) + torch.nn.utils.clip_grad_norm_.  Prints one JSON line like bench.py.
"""
import argparse
import contextlib
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


class Block(nn.Module):
    def __init__(self, d, h):
        super().__init__()
        self.h = h
        self.ln_1 = nn.LayerNorm(d)
        self.c_attn = nn.Linear(d, 3 * d)
        self.c_proj = nn.Linear(d, d)
        self.ln_2 = nn.LayerNorm(d)
        self.c_fc = nn.Linear(d, 4 * d)
        self.c_proj2 = nn.Linear(4 * d, d)

    def forward(self, x):
        B, S, C = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).view(B, S, 3, self.h, C // self.h).permute(2, 0, 3, 1, 4)
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, S, C)
        x = x + self.c_proj(y)
        return x + self.c_proj2(F.gelu(self.c_fc(self.ln_2(x)), approximate="tanh"))


class GPT(nn.Module):
    def __init__(self, V=50304, S=1024, d=2048, L=24, h=16):
        super().__init__()
        self.wte = nn.Embedding(V, d)
        self.wpe = nn.Embedding(S, d)
        self.h = nn.ModuleList([Block(d, h) for _ in range(L)])
        self.ln_f = nn.LayerNorm(d)
        for p in self.parameters():
            if p.dim() == 2:
                nn.init.normal_(p, 0, 0.02)

    def forward(self, idx, labels):
        x = self.wte(idx) + self.wpe(torch.arange(idx.shape[1], device=idx.device))
        for b in self.h:
            x = b(x)
        logits = F.linear(self.ln_f(x), self.wte.weight)
        return F.cross_entropy(logits.view(-1, logits.shape[-1]).float(), labels.reshape(-1))


class LlamaBlock(nn.Module):
    """Stock-torch Llama-3 block: nn.RMSNorm, fused qkv nn.Linear, torch RoPE, SDPA with GQA, SwiGLU."""

    def __init__(self, d=4096, h=32, hkv=8, ffn=14336):
        super().__init__()
        self.h, self.hkv, self.hd = h, hkv, d // h
        self.attention_norm = nn.RMSNorm(d, eps=1e-5)
        self.wqkv = nn.Linear(d, (h + 2 * hkv) * self.hd, bias=False)
        self.wo = nn.Linear(d, d, bias=False)
        self.ffn_norm = nn.RMSNorm(d, eps=1e-5)
        self.w13 = nn.Linear(d, 2 * ffn, bias=False)
        self.w2 = nn.Linear(ffn, d, bias=False)

    @staticmethod
    def rope(x, cos, sin):
        d = x.shape[-1] // 2
        a, b = x[..., :d], x[..., d:]
        return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

    def forward(self, x, cos, sin):
        B, S, D = x.shape
        qkv = self.wqkv(self.attention_norm(x)).view(B, S, self.h + 2 * self.hkv, self.hd)
        q = self.rope(qkv[:, :, :self.h], cos, sin).transpose(1, 2)
        k = self.rope(qkv[:, :, self.h:self.h + self.hkv], cos, sin).transpose(1, 2)
        v = qkv[:, :, self.h + self.hkv:].transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
        x = x + self.wo(o.transpose(1, 2).reshape(B, S, D))
        g, u = self.w13(self.ffn_norm(x)).chunk(2, -1)
        return x + self.w2(F.silu(g) * u)


class Llama(nn.Module):
    def __init__(self, V=128256, d=4096, L=32, S=1024):
        super().__init__()
        self.tok_embeddings = nn.Embedding(V, d)
        self.layers = nn.ModuleList([LlamaBlock(d) for _ in range(L)])
        self.norm = nn.RMSNorm(d, eps=1e-5)
        self.output = nn.Linear(d, V, bias=False)
        inv = 1.0 / (500000.0 ** (torch.arange(0, 128, 2, dtype=torch.float64) / 128))
        f = torch.outer(torch.arange(S, dtype=torch.float64), inv)
        self.register_buffer("cos", f.cos().float().view(1, S, 1, 64), persistent=False)
        self.register_buffer("sin", f.sin().float().view(1, S, 1, 64), persistent=False)
        for p in self.parameters():
            if p.dim() == 2:
                nn.init.normal_(p, 0, 0.02)

    def forward(self, idx, labels):
        x = self.tok_embeddings(idx)
        S = idx.shape[1]
        cos, sin = self.cos[:, :S].to(x.dtype), self.sin[:, :S].to(x.dtype)
        for b in self.layers:
            x = torch.utils.checkpoint.checkpoint(b, x, cos, sin, use_reentrant=False)
        logits = self.output(self.norm(x))
        return F.cross_entropy(logits.view(-1, logits.shape[-1]).float(), labels.reshape(-1))


def lm_fsdp(a, dev, world, rank, kind):
    """Stock torch FSDP (FULL_SHARD, bf16 MixedPrecision) + fused torch AdamW + clip_grad_norm_ for the
    GPT-2 1.3B (``gpt2-fsdp``) and Llama-3 8B + activation checkpointing (``llama3-fsdp``) configs;
    ``gpt2-ddp`` = GPT-2 124M under stock DDP."""
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP, MixedPrecision, ShardingStrategy
    from torch.distributed.fsdp.wrap import ModuleWrapPolicy
    from torch.nn.parallel import DistributedDataParallel as DDP
    torch.manual_seed(0)
    if kind == "llama3-fsdp":
        mb, vocab, name = a.micro_batch or 8, 128000, "Llama-3 8B FSDP + act-ckpt"
        with torch.device(dev):
            model = Llama(S=a.seq)
        wrap = {LlamaBlock}
        opt_kw = dict(lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    elif kind == "gpt2-ddp":
        mb, vocab, name = a.micro_batch or 16, 50257, "GPT-2 124M DDP"
        with torch.device(dev):
            model = GPT(S=a.seq, d=768, L=12, h=12)
        wrap = None
        opt_kw = dict(lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    else:
        mb, vocab, name = a.micro_batch or 32, 50257, "GPT-2-1.3B FSDP"
        with torch.device(dev):
            model = GPT(S=a.seq)
        wrap = {Block}
        opt_kw = dict(lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    n = sum(p.numel() for p in model.parameters())
    if wrap is None:
        model = DDP(model, device_ids=[dev.index])              # fp32 params + bf16 autocast
        opt = torch.optim.AdamW(model.parameters(), fused=True, **opt_kw)
    else:
        model = FSDP(model, sharding_strategy=ShardingStrategy.FULL_SHARD, auto_wrap_policy=ModuleWrapPolicy(wrap),
                     mixed_precision=MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16), device_id=dev,
                     use_orig_params=False, limit_all_gathers=True)
        opt = torch.optim.AdamW(model.parameters(), fused=True, **opt_kw)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    batches = [torch.randint(0, vocab, (mb, a.seq + 1), device=dev, generator=g) for _ in range(4)]

    def step(i):
        b = batches[i % 4]
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=wrap is None):
            loss = model(b[:, :-1], b[:, 1:])
        loss.backward()
        if wrap is None:
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        else:
            model.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dt, loss = timed(step, a, dev)
    tps = world * mb * a.seq * a.steps / dt
    if rank == 0:
        print(f"[torch-baseline] {name} params={n/1e9:.3f}B loss={loss.item():.4f} step={1000*dt/a.steps:.1f}ms",
              file=sys.stderr)
        print(json.dumps({"metric": f"tokens/sec {name} (whole node) -- stock PyTorch-ROCm baseline",
                          "value": round(tps, 2), "unit": "tokens/s", "n_gpus": world, "steps": a.steps,
                          "ms_per_step": round(1000 * dt / a.steps, 3), "micro_batch_per_gpu": mb,
                          "seq_len": a.seq}))


def resnet18_cpu(a, dev, world, rank):
    """Stock torch DDP over gloo on CPU, ResNet-18 fp32 (BASELINE.json config 1), same shapes as
    ``bench.py --workload resnet18-cpu``."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pytorch_distributedtraining_amd.models.resnet import resnet18
    from torch.nn.parallel import DistributedDataParallel as DDP
    mb = a.micro_batch or 16
    model = DDP(resnet18(fused_bn=False).to(memory_format=torch.channels_last))
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4)
    x = torch.randn(mb, 3, 224, 224).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (mb,))

    def step(i):
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dt, loss = timed(step, a, dev)
    if rank == 0:
        print(json.dumps({"metric": "samples/sec ResNet-18 DDP CPU/gloo (whole node) -- stock PyTorch baseline",
                          "value": round(world * mb * a.steps / dt, 2), "unit": "samples/s", "n_ranks": world,
                          "steps": a.steps, "ms_per_step": round(1000 * dt / a.steps, 3), "micro_batch_per_rank": mb}))


def resnet50_ddp(a, dev, world, rank):
    """Stock torch DDP (25 MiB buckets) + bf16 autocast + torch fused AdamW + clip_grad_norm_ on the
    same ResNet-50 / batch / synthetic data as ``bench.py --workload resnet50-ddp``."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pytorch_distributedtraining_amd.models.resnet import resnet50  # plain nn.Conv2d / nn.BatchNorm2d
    from torch.nn.parallel import DistributedDataParallel as DDP
    mb = a.micro_batch or 256
    model = resnet50(fused_bn=False).to(dev).to(memory_format=torch.channels_last)   # nn.BatchNorm2d + nn.ReLU
    model = DDP(model, device_ids=[dev.index])
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4, fused=True)
    x = torch.randn(mb, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (mb,), device=dev)

    def step(i):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dt, loss = timed(step, a, dev)
    sps = world * mb * a.steps / dt
    if rank == 0:
        print(f"[torch-baseline] resnet50 loss={loss.item():.4f} step={1000*dt/a.steps:.1f}ms", file=sys.stderr)
        print(json.dumps({"metric": "samples/sec ResNet-50 DDP (whole node) -- stock PyTorch-ROCm baseline",
                          "value": round(sps, 2), "unit": "samples/s", "n_gpus": world, "steps": a.steps,
                          "ms_per_step": round(1000 * dt / a.steps, 3), "micro_batch_per_gpu": mb,
                          "stack": "torch DDP + autocast bf16 + MIOpen + fused torch AdamW"}))


def swinir_stoke(a, dev, world, rank):
    """Stock torch counterpart of ``bench.py --workload swinir-stoke``: the same SwinIR-S x2 parameters with
    nn.LayerNorm + SDPA window attention, torch DDP (no_sync on the non-boundary micro-step), bf16 autocast,
    fused torch AdamW, clip_grad_norm_(0.1), 2 x 18 LR 128x128 patches per optimizer step."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from pytorch_distributedtraining_amd.models.swinir import swinir_s_x2, to_stock_torch
    from torch.nn.parallel import DistributedDataParallel as DDP
    mb, accum = a.micro_batch or 18, 2
    model = to_stock_torch(swinir_s_x2().to(dev))
    ddp = DDP(model, device_ids=[dev.index])
    opt = torch.optim.AdamW(ddp.parameters(), lr=1e-3, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-4, fused=True)
    g = torch.Generator(device=dev).manual_seed(2000 + rank)
    data = [(torch.rand(mb, 3, 128, 128, device=dev, generator=g), torch.rand(mb, 3, 256, 256, device=dev, generator=g))
            for _ in range(accum)]

    if a.loss == "feat":
        from pytorch_distributedtraining_amd.models.losses import PerceptualLoss   # stock nn.Conv2d / ReLU / MaxPool
        crit = PerceptualLoss().to(dev)
    else:
        crit = lambda o, t: F.mse_loss(o.float(), t)   # noqa: E731

    def step(i):
        for j, (x, y) in enumerate(data):
            ctx = ddp.no_sync() if j < accum - 1 else contextlib.nullcontext()
            with ctx:
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.precision == "bf16"):
                    loss = crit(ddp(x), y) / accum
                loss.backward()
        torch.nn.utils.clip_grad_norm_(ddp.parameters(), 0.1)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dt, loss = timed(step, a, dev)
    sps = world * mb * accum * a.steps / dt
    if rank == 0:
        print(f"[torch-baseline] swinir loss={loss.item():.4f} step={1000*dt/a.steps:.1f}ms", file=sys.stderr)
        print(json.dumps({"metric": "samples/sec SwinIR-S x2 DDP (whole node) -- stock PyTorch-ROCm baseline",
                          "value": round(sps, 2), "unit": "samples/s", "n_gpus": world, "steps": a.steps,
                          "ms_per_step": round(1000 * dt / a.steps, 3), "micro_batch_per_gpu": mb,
                          "loss": a.loss, "dtype": a.precision,
                          "stack": "torch DDP + autocast + SDPA + nn.LayerNorm + fused torch AdamW"}))


def timed(step, a, dev):
    for i in range(a.warmup):
        step(i)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(i)
    sync()
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    return float(dt.item()), loss


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="gpt2-fsdp",
                    choices=["gpt2-fsdp", "gpt2-ddp", "llama3-fsdp", "resnet50-ddp", "swinir-stoke",
                             "resnet18-cpu"])
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--micro-batch", type=int, default=None)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--loss", default="feat", choices=["feat", "mse"])
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    if a.workload == "resnet18-cpu":
        dist.init_process_group("gloo", rank=rank, world_size=world)
        resnet18_cpu(a, torch.device("cpu"), world, rank)
        dist.destroy_process_group()
        return
    torch.cuda.set_device(lr)
    dev = torch.device("cuda", lr)
    # same MIOpen find mode as bench.py for the convolution workloads (fair comparison)
    torch.backends.cudnn.benchmark = os.environ.get("PDT_CONV_BENCHMARK", "1") == "1"
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    if a.workload in ("resnet50-ddp", "swinir-stoke"):
        (resnet50_ddp if a.workload == "resnet50-ddp" else swinir_stoke)(a, dev, world, rank)
        dist.destroy_process_group()
        return
    if a.workload in ("llama3-fsdp", "gpt2-ddp"):
        lm_fsdp(a, dev, world, rank, a.workload)
        dist.destroy_process_group()
        return
    a.micro_batch = a.micro_batch or 16
    from torch.distributed.fsdp import FullyShardedDataParallel as FSDP, MixedPrecision, ShardingStrategy
    from torch.distributed.fsdp.wrap import ModuleWrapPolicy
    torch.manual_seed(0)
    with torch.device(dev):
        model = GPT(S=a.seq)
    n = sum(p.numel() for p in model.parameters())
    model = FSDP(model, sharding_strategy=ShardingStrategy.FULL_SHARD, auto_wrap_policy=ModuleWrapPolicy({Block}),
                 mixed_precision=MixedPrecision(torch.bfloat16, torch.bfloat16, torch.bfloat16), device_id=dev,
                 use_orig_params=False, limit_all_gathers=True)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, fused=True)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    batches = [torch.randint(0, 50257, (a.micro_batch, a.seq + 1), device=dev, generator=g) for _ in range(4)]

    def step(i):
        b = batches[i % 4]
        loss = model(b[:, :-1], b[:, 1:])
        loss.backward()
        model.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    dt, loss = timed(step, a, dev)
    tps = world * a.micro_batch * a.seq * a.steps / dt
    if rank == 0:
        print(f"[torch-baseline] params={n/1e9:.3f}B loss={loss.item():.4f} step={1000*dt/a.steps:.1f}ms",
              file=sys.stderr)
        print(json.dumps({"metric": "tokens/sec GPT-2-1.3B FSDP (whole node) -- stock PyTorch-ROCm baseline",
                          "value": round(tps, 2), "unit": "tokens/s", "n_gpus": world, "steps": a.steps,
                          "ms_per_step": round(1000 * dt / a.steps, 3), "micro_batch_per_gpu": a.micro_batch,
                          "seq_len": a.seq, "stack": "torch FSDP + SDPA + nn.LayerNorm + fused torch AdamW"}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
