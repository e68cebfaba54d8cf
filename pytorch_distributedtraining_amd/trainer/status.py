"""Validation of a facade option combination (the role of Stoke's status object)."""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Optional


class StatusError(ValueError):
    pass


@dataclass
class TrainerStatus:
    gpu: bool
    distributed: Optional[str]
    fp16: Optional[str]
    oss: bool
    sddp: bool
    fsdp: bool
    grad_accum_steps: int
    batch_size_per_device: int
    world_size: int = 1

    def validate(self):
        if self.grad_accum_steps < 1:
            raise StatusError("grad_accum_steps must be >= 1")
        if self.batch_size_per_device < 1:
            raise StatusError("batch_size_per_device must be >= 1")
        if self.sddp and not self.oss:
            raise StatusError("fairscale_sddp (ZeRO-2) requires fairscale_oss (ZeRO-1): ShardedDataParallel reduces "
                              "each gradient to the rank owning its optimizer shard")
        if (self.oss or self.sddp) and self.distributed is None:
            raise StatusError("fairscale_oss / fairscale_sddp require distributed='ddp'")
        if self.fsdp and (self.oss or self.sddp):
            raise StatusError("fsdp already shards optimizer state and gradients; do not combine with oss/sddp")
        if self.fp16 in ("amp", "apex_O1") and not self.gpu:
            raise StatusError("fp16 AMP requires gpu=True (use bf16 or fp32 on CPU)")
        if self.distributed not in (None, "ddp", "fsdp", "deepspeed"):
            raise StatusError(f"unknown distributed option {self.distributed!r}")
        if self.fp16 not in (None, "amp", "bf16", "apex_O1", "apex_O2", "deepspeed"):
            raise StatusError(f"unknown fp16 option {self.fp16!r}")
        return self

    @property
    def effective_batch_size(self) -> int:
        return self.batch_size_per_device * self.grad_accum_steps * self.world_size

    def as_dict(self):
        d = asdict(self)
        d["effective_batch_size"] = self.effective_batch_size
        return d
