"""Run configurations for the BASELINE.json workloads (SURVEY.md §5.6 "YAML/JSON run configs for the five
BASELINE.json configs" + "env overrides for comm tuning").

A ``RunConfig`` names the model, the engine combination (the reference's Stoke flags: distributed /
fairscale_oss / fairscale_sddp, plus fsdp), precision, batch / accumulation / clipping (Stoke-DDP.py:159,
247-253), optimizer kwargs (Stoke-DDP.py:226-235) and the DDP bucket sizing.  ``load_config`` reads YAML
(safe loader) or JSON; ``apply_env_overrides`` lets a launcher retune communication without editing files:

    PDT_BUCKET_MB, PDT_FIRST_BUCKET_MB   DDP bucket cap / first bucket (MiB)
    PDT_XGMI=1|auto, PDT_XGMI_ONESHOT_KB route eligible collectives through the xGMI peer kernels (auto: by
                                        size class, PDT_XGMI_MIN_KB / PDT_XGMI_MAX_KB)
    PDT_BATCH, PDT_STEPS, PDT_PRECISION  quick sweeps
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class RunConfig:
    name: str = "run"
    model: str = "resnet18"                 # resnet18/50, gpt2-124m/1.3b, llama3-8b/1b/tiny, swinir-s-x2, srnet
    distributed: Optional[str] = "ddp"      # None | "ddp" | "fsdp"
    fairscale_oss: bool = False             # ZeRO-1 (Fairscale OSS)
    fairscale_sddp: bool = False            # ZeRO-2 (Fairscale ShardedDDP)
    precision: str = "bf16"                 # bf16 | fp8 (bf16 + fp8 linear GEMMs) | amp (fp16 + loss scaling) | fp32
    gpu: bool = True
    backend: str = "nccl"                   # RCCL on ROCm; gloo for CPU runs
    batch_size_per_device: int = 32
    grad_accum_steps: int = 1
    grad_clip: Optional[float] = 1.0
    seq_len: int = 1024                     # language models
    image_size: int = 224                   # classifiers; SR models: LR patch size
    num_classes: int = 1000
    loss: str = "auto"                      # auto | mse | feat (perceptual) | ce
    optimizer: Dict[str, Any] = field(default_factory=lambda: {"lr": 1e-4, "betas": (0.9, 0.95), "eps": 1e-8,
                                                                "weight_decay": 0.1})
    activation_checkpointing: bool = False
    bucket_cap_mb: float = 64.0
    first_bucket_mb: float = 8.0
    sync_batchnorm: bool = False
    conv_benchmark: bool = True             # MIOpen find per conv shape (torch.backends.cudnn.benchmark)
    steps: int = 10
    warmup: int = 2
    log_every: int = 10
    checkpoint_dir: Optional[str] = None
    checkpoint_every: int = 0               # optimizer steps between checkpoints (0: only at the end)
    resume: bool = True                     # continue from the newest checkpoint in checkpoint_dir
    metrics_path: Optional[str] = None
    seed: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def load_config(path: str, **overrides) -> RunConfig:
    """YAML (yaml.safe_load) or JSON file -> RunConfig; unknown keys raise."""
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text)
    data.update({k: v for k, v in overrides.items() if v is not None})
    names = {f.name for f in dataclasses.fields(RunConfig)}
    unknown = set(data) - names
    if unknown:
        raise ValueError(f"{path}: unknown config keys {sorted(unknown)}")
    if "optimizer" in data and "betas" in data["optimizer"]:
        data["optimizer"] = dict(data["optimizer"], betas=tuple(data["optimizer"]["betas"]))
    return RunConfig(**data)


def apply_env_overrides(cfg: RunConfig, env=None) -> RunConfig:
    env = os.environ if env is None else env
    upd = {}
    if env.get("PDT_BUCKET_MB"):
        upd["bucket_cap_mb"] = float(env["PDT_BUCKET_MB"])
    if env.get("PDT_FIRST_BUCKET_MB"):
        upd["first_bucket_mb"] = float(env["PDT_FIRST_BUCKET_MB"])
    if env.get("PDT_BATCH"):
        upd["batch_size_per_device"] = int(env["PDT_BATCH"])
    if env.get("PDT_STEPS"):
        upd["steps"] = int(env["PDT_STEPS"])
    if env.get("PDT_PRECISION"):
        upd["precision"] = env["PDT_PRECISION"]
    return dataclasses.replace(cfg, **upd) if upd else cfg


# PDT_XGMI=auto: the mesh takes the latency class up to this size, RCCL the rest.  A default from the size-class
# arithmetic of SURVEY.md §5.8, unmeasured on a multi-GPU node (the mesh has only run as ranks sharing one GPU),
# which is also why PDT_XGMI defaults to off
XGMI_AUTO_MAX_KB = 1024


def xgmi_mode(env=None) -> str:
    """PDT_XGMI: "0" (RCCL only, default), "1" / "all" (every eligible collective on the xGMI mesh), "auto"
    (size classes: small payloads on the mesh, bulk on RCCL)."""
    env = os.environ if env is None else env
    v = env.get("PDT_XGMI", "0").strip().lower()
    if v in ("1", "all", "true", "on"):
        return "all"
    if v == "auto":
        return "auto"
    return "off"


def xgmi_kwargs(env=None) -> Dict[str, Any]:
    """XGMIComm tuning from the environment (PDT_XGMI_ONESHOT_KB, PDT_XGMI_SLOT_MB, PDT_XGMI_TIMEOUT_S, and the
    size class PDT_XGMI_MIN_KB / PDT_XGMI_MAX_KB -- the latter defaulting to 1 MiB under PDT_XGMI=auto)."""
    env = os.environ if env is None else env
    kw = {}
    if env.get("PDT_XGMI_MIN_KB"):
        kw["min_bytes"] = int(float(env["PDT_XGMI_MIN_KB"]) * 1024)
    if env.get("PDT_XGMI_MAX_KB"):
        kw["max_bytes"] = int(float(env["PDT_XGMI_MAX_KB"]) * 1024)
    elif xgmi_mode(env) == "auto":
        kw["max_bytes"] = XGMI_AUTO_MAX_KB * 1024
    if env.get("PDT_XGMI_ONESHOT_KB"):
        kw["oneshot_max_bytes"] = int(float(env["PDT_XGMI_ONESHOT_KB"]) * 1024)
    if env.get("PDT_XGMI_SLOT_MB"):
        kw["slot_bytes"] = int(float(env["PDT_XGMI_SLOT_MB"]) * (1 << 20))
    if env.get("PDT_XGMI_TIMEOUT_S"):
        kw["timeout_us"] = int(float(env["PDT_XGMI_TIMEOUT_S"]) * 1e6)
    return kw
