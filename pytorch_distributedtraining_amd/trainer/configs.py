"""Typed configuration objects of the training facade (Stoke-compatible names and defaults).

Reference call sites: AMPConfig(init_scale=2**14) Stoke-DDP.py:182-184; DDPConfig(local_rank,
convert_to_sync_batch_norm=True) :190-193; FairscaleOSSConfig(broadcast_fp16=True) :197-199;
ClipGradNormConfig(max_norm, norm_type=2.0) :253; StokeOptimizer(optimizer, optimizer_kwargs)
:226-235; DistributedOptions.ddp / FP16Options.amp :247-248; DeepspeedConfig / DeepspeedZeROConfig
imported :18 (here they map onto the framework's own ZeRO engines).  Defaults follow SURVEY.md B1.cfg
except where the MI355X defaults differ (DDP bucket caps picked from 7-xGMI-link arithmetic -- documented per
field; defaults, unmeasured on a multi-GPU node).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Sequence, Type

import torch


class DistributedOptions(enum.Enum):
    ddp = "ddp"          # data parallel (bucketed all-reduce)
    fsdp = "fsdp"        # fully sharded (ZeRO-3) flat-parameter engine
    deepspeed = "deepspeed"  # accepted for config compatibility: routed to the native ZeRO engines


class FP16Options(enum.Enum):
    amp = "amp"          # fp16 autocast + dynamic loss scaling (GradScaler)
    bf16 = "bf16"        # bf16 compute (MI355X default: no loss scaling needed)
    apex_O1 = "apex_O1"  # accepted for compatibility: treated as amp
    apex_O2 = "apex_O2"  # accepted for compatibility: treated as bf16 master-weight training
    deepspeed = "deepspeed"


@dataclass
class AMPConfig:
    init_scale: float = 2.0 ** 16
    growth_factor: float = 2.0
    backoff_factor: float = 0.5
    growth_interval: int = 2000


@dataclass
class DDPConfig:
    local_rank: Optional[int] = None
    backend: str = "nccl"                 # RCCL on ROCm; 'gloo' for CPU runs
    init_method: str = "env://"
    bucket_cap_mb: float = 64.0           # torch default 25; larger buckets should keep xGMI ring steps
                                          # bandwidth-bound (arithmetic; unmeasured on a multi-GPU node)
    first_bucket_mb: float = 8.0          # torch default 1
    broadcast_buffers: bool = True
    find_unused_parameters: bool = False
    convert_to_sync_batch_norm: bool = False
    no_sync: bool = True                  # skip the all-reduce on non-boundary micro-steps
    timeout_s: float = 1800.0
    reduce_dtype: Optional[torch.dtype] = None   # e.g. torch.bfloat16 to compress fp32 gradients


@dataclass
class FairscaleOSSConfig:
    broadcast_fp16: bool = False


@dataclass
class FairscaleSDDPConfig:
    broadcast_buffers: bool = True
    sync_models_at_startup: bool = True
    reduce_buffer_size: int = 2 ** 23
    reduce_fp16: bool = False


@dataclass
class FairscaleFSDPConfig:
    sharding_strategy: str = "full_shard"          # or "shard_grad_op" (ZeRO-2 flat)
    param_dtype: torch.dtype = torch.bfloat16
    reduce_dtype: torch.dtype = torch.bfloat16
    wrap_classes: Sequence[Type] = ()              # default: model.block_class
    forward_prefetch: bool = True
    backward_prefetch: bool = True
    activation_checkpointing: bool = False


FSDPConfig = FairscaleFSDPConfig
OSSConfig = FairscaleOSSConfig
SDDPConfig = FairscaleSDDPConfig


@dataclass
class ClipGradNormConfig:
    max_norm: float
    norm_type: float = 2.0


@dataclass
class ClipGradConfig:
    clip_value: float


@dataclass
class StokeOptimizer:
    optimizer: Any
    optimizer_kwargs: Dict[str, Any] = field(default_factory=dict)


@dataclass
class DeepspeedZeROConfig:
    stage: int = 0


@dataclass
class DeepspeedConfig:
    zero_optimization: DeepspeedZeROConfig = field(default_factory=DeepspeedZeROConfig)


def find_config(configs, cls):
    for c in configs or ():
        if isinstance(c, cls):
            return c
    return None
