"""Optimizer-side components: fused AdamW, fused grad clipping, loss scaling."""
from .clip import clip_grad_norm_, grad_norm_sq
from .fused_adamw import FusedAdamW
from .grad_scaler import GradScaler

__all__ = ["FusedAdamW", "clip_grad_norm_", "grad_norm_sq", "GradScaler"]
