"""Hand-written gfx950 (MI355X / CDNA4) kernels exposed as PyTorch ops.

Every op dispatches GPU tensors to ``lib/libpdt_kernels.so`` (HIP, MFMA/LDS-tiled where the op is
matmul-shaped) and fails loudly if that library is missing; CPU tensors use the reference math.
"""
from . import _lib
from .activations import bias_gelu, swiglu
from .attention import flash_attn, flash_attn_qkvpacked
from .cross_entropy import cross_entropy
from .fp8 import dequantize_fp8, fp8_autocast, quantize_fp8, scale_from_amax
from .multi_tensor import TensorTable, adamw_step, cast_f32_to_bf16, clip_coef, l2norm_sq, scale_
from .norms import LayerNorm, RMSNorm, layer_norm, rms_norm
from .rope import apply_rope, rope_tables


def native_available() -> bool:
    return _lib.available()


__all__ = [
    "bias_gelu", "swiglu", "flash_attn", "flash_attn_qkvpacked", "cross_entropy", "quantize_fp8",
    "dequantize_fp8", "fp8_autocast", "scale_from_amax", "TensorTable", "adamw_step", "cast_f32_to_bf16", "clip_coef",
    "l2norm_sq", "scale_", "LayerNorm", "RMSNorm", "layer_norm", "rms_norm", "apply_rope", "rope_tables",
    "native_available",
]
