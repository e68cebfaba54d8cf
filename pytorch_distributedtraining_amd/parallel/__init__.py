"""Parallel engines over RCCL / xGMI (and gloo for CPU)."""
from .comm import Comm, Handle, default_comm
from .fsdp import FullyShardedDataParallel, MixedPrecision, ShardingStrategy

__all__ = ["Comm", "Handle", "default_comm", "FullyShardedDataParallel", "MixedPrecision", "ShardingStrategy"]
