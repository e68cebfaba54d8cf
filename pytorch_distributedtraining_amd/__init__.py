"""pytorch_distributedtraining_amd -- an MI355X-native (gfx950 / CDNA4) distributed training framework.

Capabilities of rushi-the-neural-arch/PyTorch-DistributedTraining (Stoke facade over DDP, Fairscale
OSS / ShardedDDP, SyncBN, AMP, grad accumulation / clipping, checkpointing) plus FSDP, re-designed
MI355X-first: PyTorch-ROCm for the framework layer, hand-written HIP kernels (``ops``) for the hot
path, RCCL over xGMI (``parallel``) for the collectives, and a C++ host runtime (``_pdt_runtime``).
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401
