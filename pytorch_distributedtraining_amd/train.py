"""Config-driven training entry point: one process per GPU, any BASELINE.json workload
through the Stoke-style ``Trainer`` on synthetic data of the workload's shape.

    python -m pytorch_distributedtraining_amd.train --config configs/resnet18_ddp_cpu.yaml
    python -m pytorch_distributedtraining_amd.launch --nproc-per-node 8 -m pytorch_distributedtraining_amd.train \
        --config configs/gpt2_1.3b_fsdp.yaml

Accepts both ``--local-rank`` and ``--local_rank`` (the reference's parser only knew the latter while
torch.distributed.launch passes the former).  Prints rank-0 progress lines with the
synced loss and whole-job throughput, writes JSONL metrics when ``metrics_path`` is set, saves Stoke-layout
checkpoints every ``checkpoint_every`` optimizer steps and at the end when ``checkpoint_dir`` is set, and
resumes from the newest one found there (``resume``, default on) -- which is what makes a launcher restart
(``launch --max-restarts``) after a rank failure continue the run instead of starting over.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

from .run_config import RunConfig, apply_env_overrides, load_config


def build_model(cfg: RunConfig):
    """-> (model, kind) with kind in {"lm", "cls", "sr"}."""
    m = cfg.model
    if m.startswith("gpt2"):
        from .models import build_gpt2
        return build_gpt2(m, n_positions=max(1024, cfg.seq_len),
                          activation_checkpointing=cfg.activation_checkpointing), "lm"
    if m.startswith("llama"):
        from .models.llama import build_llama
        return build_llama(m, max_seq_len=max(cfg.seq_len, 2048),
                           activation_checkpointing=cfg.activation_checkpointing), "lm"
    if m.startswith("resnet"):
        from .models import resnet
        return getattr(resnet, m)(num_classes=cfg.num_classes), "cls"
    if m.startswith("swinir"):
        from .models.swinir import swinir_s_x2
        return swinir_s_x2(), "sr"
    if m == "srnet":
        from .models.srnet import Net
        return Net(upscale_factor=2), "sr"
    raise ValueError(f"unknown model {m}")


def make_batch(cfg: RunConfig, kind: str, device, gen):
    b = cfg.batch_size_per_device
    if kind == "lm":
        vocab = 128000 if cfg.model.startswith("llama3-8b") else (1024 if "tiny" in cfg.model else 50257)
        t = torch.randint(0, vocab, (b, cfg.seq_len + 1), device=device, generator=gen)
        return t[:, :-1], t[:, 1:]
    if kind == "cls":
        x = torch.randn(b, 3, cfg.image_size, cfg.image_size, device=device, generator=gen)
        if device.type == "cuda":
            x = x.to(memory_format=torch.channels_last)
        return x, torch.randint(0, cfg.num_classes, (b,), device=device, generator=gen)
    s = cfg.image_size
    return (torch.rand(b, 3, s, s, device=device, generator=gen),
            torch.rand(b, 3, 2 * s, 2 * s, device=device, generator=gen))


def loss_fn(cfg: RunConfig, kind: str):
    if kind == "lm":
        return lambda out, _tgt: out                      # the model returns the fused CE loss
    if kind == "cls" or cfg.loss == "ce":
        return lambda out, tgt: F.cross_entropy(out.float(), tgt)
    if cfg.loss == "feat":
        from .models.losses import feat_loss
        return feat_loss
    return lambda out, tgt: F.mse_loss(out.float(), tgt)


def run(cfg: RunConfig) -> dict:
    from .trainer import ClipGradNormConfig, DDPConfig, FairscaleFSDPConfig, StokeOptimizer, Trainer
    from .utils.logging import MetricsSink, ThroughputMeter
    from .utils.profiling import StepTimer

    gpu = cfg.gpu and torch.cuda.is_available()
    torch.manual_seed(cfg.seed)
    if cfg.gpu and cfg.conv_benchmark:
        torch.backends.cudnn.benchmark = True   # MIOpen find: +12 % on ResNet-50 (profiles/r1_v9_miopen_modes.log)
    model, kind = build_model(cfg)
    if gpu and kind == "cls":
        model = model.to(memory_format=torch.channels_last)
    ddp_cfg = DDPConfig(backend=cfg.backend if gpu else "gloo", bucket_cap_mb=cfg.bucket_cap_mb,
                        first_bucket_mb=cfg.first_bucket_mb, convert_to_sync_batch_norm=cfg.sync_batchnorm,
                        local_rank=int(os.environ.get("LOCAL_RANK", "0")) if gpu else None)
    configs = [ddp_cfg, FairscaleFSDPConfig(activation_checkpointing=cfg.activation_checkpointing)]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    distributed = cfg.distributed if (world > 1 or cfg.distributed == "fsdp") else None
    opt = StokeOptimizer(optimizer=torch.optim.AdamW, optimizer_kwargs=dict(cfg.optimizer))
    precision = None if cfg.precision == "fp32" else "bf16" if cfg.precision == "fp8" else cfg.precision
    tr = Trainer(model, optimizer=opt, loss=loss_fn(cfg, kind), batch_size_per_device=cfg.batch_size_per_device,
                 grad_accum_steps=cfg.grad_accum_steps,
                 grad_clip=ClipGradNormConfig(max_norm=cfg.grad_clip) if cfg.grad_clip else None, gpu=gpu,
                 fp16=precision if gpu else None, distributed=distributed,
                 fairscale_oss=cfg.fairscale_oss and distributed is not None,
                 fairscale_sddp=cfg.fairscale_sddp and distributed is not None,
                 fairscale_fsdp=distributed == "fsdp", configs=configs, verbose=False,
                 fp8=cfg.precision == "fp8" and gpu)
    dev = tr.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(cfg.seed + 1000 * tr.rank)
    batches = [make_batch(cfg, kind, dev, gen) for _ in range(max(1, cfg.grad_accum_steps))]
    sink = MetricsSink(cfg.metrics_path, config=cfg.to_dict()) if tr.rank == 0 and cfg.metrics_path else None

    def opt_step():
        loss = None
        for x, y in batches:
            out = tr.model(x, labels=y) if kind == "lm" else tr.model(x)
            loss = tr.loss(out, y)
            tr.backward(loss)
            tr.step()
        return loss

    # auto-resume: continue from the newest Stoke-layout checkpoint in checkpoint_dir --
    # after a launcher restart (--max-restarts) the group picks up where the last save left it
    start = 0
    if cfg.checkpoint_dir and cfg.resume:
        from .utils.checkpoint import latest_checkpoint
        tag = latest_checkpoint(cfg.checkpoint_dir) if os.path.isdir(cfg.checkpoint_dir) else None
        if tag is not None:
            extras = tr.load(cfg.checkpoint_dir, tag) or {}
            start = int(extras.get("step", 0))
            tr.print(f"[train] resumed from {tag} at step {start}")
    total = cfg.warmup + cfg.steps

    def maybe_save(step):
        if cfg.checkpoint_dir and cfg.checkpoint_every and step % cfg.checkpoint_every == 0 and step < total:
            tr.save(cfg.checkpoint_dir, name=f"{cfg.name}-s{step}", extras={"step": step})

    for step in range(start, min(cfg.warmup, total)):
        opt_step()
        maybe_save(step + 1)
    if gpu:
        torch.cuda.synchronize(dev)
    tr.barrier()
    if gpu:
        torch.cuda.reset_peak_memory_stats(dev)
    inner = getattr(tr.model, "module", tr.model)
    flops = inner.flops_per_token(cfg.seq_len) * cfg.seq_len if kind == "lm" and hasattr(inner, "flops_per_token") \
        else None
    meter = ThroughputMeter(tr.world_size, flops_per_sample=flops)   # whole-job samples/s (+ TFLOP/s for LMs)
    timer = StepTimer(enabled=gpu and cfg.log_every > 0)              # per-step GPU time from HIP events
    meter.start()
    t0 = meter.t0
    last, loss = None, None
    first = max(start, cfg.warmup)
    for step in range(first, total):
        with timer.phase("optimizer_step"):
            loss = opt_step()
        meter.add(cfg.batch_size_per_device * cfg.grad_accum_steps)
        i = step - cfg.warmup
        maybe_save(step + 1)
        if (i + 1) % cfg.log_every == 0 or step + 1 == total:
            last = float(tr.detach_and_sync_loss(loss))       # one host sync per log line only
            rate = meter.rate()
            rec = {"step": step + 1, "loss": last, "samples_per_s": rate["samples_per_s"]}
            if kind == "lm":
                rec["tokens_per_s"] = rate["samples_per_s"] * cfg.seq_len
                if "tflops_per_s" in rate:
                    rec["tflops_per_s_per_rank"] = rate["tflops_per_s"] / tr.world_size
            if gpu:
                rec["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
            tr.print(json.dumps(rec))
            if sink:
                sink.log(rec, step=step + 1)
    if gpu:
        torch.cuda.synchronize(dev)
    tr.barrier()
    dt = time.perf_counter() - t0
    n = max(1, total - first)
    samples = n * cfg.batch_size_per_device * cfg.grad_accum_steps * tr.world_size
    result = {"name": cfg.name, "model": cfg.model, "world_size": tr.world_size, "steps": cfg.steps,
              "resumed_from": start, "ms_per_step": 1000 * dt / n, "samples_per_s": samples / dt, "loss": last}
    if kind == "lm":
        result["tokens_per_s"] = samples * cfg.seq_len / dt
    st = timer.summary().get("optimizer_step")
    if st:
        result["gpu_ms_per_step"] = round(st["mean_ms"], 3)
    if gpu:
        result["peak_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    if cfg.checkpoint_dir:
        result["checkpoint"] = tr.save(cfg.checkpoint_dir, name=f"{cfg.name}-final", extras={"step": total})
    if sink:
        sink.log({"final": result})
        sink.close()
    return result


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--batch-size", type=int, default=None, dest="batch_size_per_device")
    ap.add_argument("--local-rank", "--local_rank", type=int, default=None, dest="local_rank")
    a = ap.parse_args(argv)
    if a.local_rank is not None:
        os.environ.setdefault("LOCAL_RANK", str(a.local_rank))
    cfg = apply_env_overrides(load_config(a.config, steps=a.steps, batch_size_per_device=a.batch_size_per_device))
    res = run(cfg)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(res, default=str), flush=True)
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # pragma: no cover
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
