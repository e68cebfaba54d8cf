"""ctypes binding of ``lib/libpdt_kernels.so`` (the gfx950 HIP kernels).

The library is loaded lazily, after ``import torch``, so its ``libamdhip64.so.7`` dependency resolves
to the HIP runtime torch already mapped (one runtime, one set of streams).  Every entry point takes
raw device pointers plus the current HIP stream handle and returns a ``hipError_t``.

Policy: a GPU tensor ALWAYS goes through the HIP kernels -- if the library is missing on a GPU box
the op raises (no silent eager fallback).  CPU tensors use the PyTorch reference math; that path
exists for the CPU unit tests and the gloo multi-process tests.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

# PDT_KERNEL_LIB points at another build of the library (A/B of two kernel builds on one box)
_LIB_PATH = os.environ.get("PDT_KERNEL_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libpdt_kernels.so")
_lock = threading.Lock()
_lib = None
_load_error: Exception | None = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_float = ctypes.c_float

# name -> argtypes (restype is always c_int)
_SIGS = {
    "pdt_adamw_mt": [c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_float, c_float, c_float,
                     c_float, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_step_inc": [c_void_p, c_void_p, c_void_p],
    "pdt_lt_probe": [c_int, c_int, c_int64, c_int64, c_int64, c_int, c_int, c_int],
    "pdt_lt_matmul": [c_int, c_int, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                      c_void_p, c_int, c_int, c_void_p],
    "pdt_lt_matmul_c": [c_int, c_int, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_int, c_int, c_int, c_void_p],
    "pdt_embedding_bwd": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int64, c_int, c_int64, c_void_p],
    "pdt_l2norm_mt": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "pdt_clip_coef": [c_void_p, c_float, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_scale_mt": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "pdt_cast_f32_bf16_mt": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "pdt_copy_mt": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "pdt_add_mt": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "pdt_norm_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                     c_int, c_float, c_int, c_int, c_int, c_void_p],
    "pdt_norm_bwd_workspace_floats": [c_int, c_int],
    "pdt_norm_fwd_win": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                         c_float, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_norm_bwd_win": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                         c_void_p],
    "pdt_norm_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_colsum_ws_floats": [c_int, c_int],
    "pdt_bias_gelu_bwd_db": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                             c_int, c_int, c_int, c_void_p],
    "pdt_colsum": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p],
    "pdt_bias_gelu_fwd": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_bias_gelu_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_swiglu_fwd": [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p],
    "pdt_swiglu_bwd": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p],
    "pdt_rope": [c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int, c_int, c_int, c_int,
                 c_void_p, c_void_p, c_int, c_int, c_void_p],
    "pdt_fp8_quant": [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p],
    "pdt_fp8_dequant": [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p],
    "pdt_fp8_cast_transpose": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               c_void_p],
    "pdt_fp8_update_scales": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float,
                              c_void_p],
    "pdt_fp8_gelu_bwd_ws_floats": [c_int, c_int],
    "pdt_fp8_bias_gelu_ct": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "pdt_fp8_bias_gelu_bwd_ct": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                 c_int, c_void_p, c_void_p, c_void_p],
    "pdt_cast_f32_bf16": [c_void_p, c_void_p, c_int64, c_void_p],
    "pdt_transpose16": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "pdt_ce_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int64, c_int, c_int, c_void_p],
    "pdt_ce_fwd_grad": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int64, c_int, c_int,
                        c_void_p],
    "pdt_ce_scale": [c_void_p, c_void_p, c_int64, c_int, c_int64, c_int, c_void_p],
    "pdt_ce_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int64, c_int64,
                   c_int, c_int, c_void_p],
    "pdt_flash_attn_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                           c_int, c_int, c_float, c_int, c_void_p],
    "pdt_flash_attn_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int,
                           c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "pdt_flash_attn_colsum_ws_floats": [c_int, c_int, c_int, c_int, c_int, c_int],
    "pdt_flash_attn_set_dkdv": [c_int],
    "pdt_flash_attn_set_dqp": [c_int],
    "pdt_flash_attn_set_variant": [c_int, c_int],
    "pdt_flash_attn_set_order": [c_int],
    "pdt_win_attn_grid": [c_int],
    "pdt_win_attn_mfma_ok": [c_int, c_int, c_int, c_int],
    "pdt_win_attn_mfma_grid": [c_int, c_int],
    "pdt_win_attn_mfma_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                              c_int, c_float, c_void_p, c_int, c_int, c_void_p],
    "pdt_win_bwd_prep": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         c_void_p],
    "pdt_rel_bias_gather": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "pdt_rel_bias_scatter": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p,
                             c_void_p],
    "pdt_win_attn_mfma_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p],
    "pdt_win_attn_mfma32_ok": [c_int, c_int, c_int],
    "pdt_win_attn_mfma32_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                c_int, c_float, c_void_p, c_int, c_int, c_void_p],
    "pdt_win_attn_mfma32_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p],
    "pdt_win_attn_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                         c_int, c_void_p],
    "pdt_win_attn_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p],
    "pdt_xgmi_alloc": [c_int64, c_int, c_void_p],
    "pdt_xgmi_free": [c_void_p],
    "pdt_xgmi_ipc_get": [c_void_p, c_void_p],
    "pdt_xgmi_ipc_handle_bytes": [],
    "pdt_xgmi_ipc_open": [c_void_p, c_void_p],
    "pdt_xgmi_ipc_close": [c_void_p],
    "pdt_xgmi_error": [c_void_p, c_void_p],
    "pdt_xgmi_collective": [c_int, c_void_p, c_void_p, c_int64, c_int64, c_int, c_float, c_void_p, c_int, c_int,
                            ctypes.c_uint, c_int64, ctypes.c_uint, c_void_p, c_void_p],
    "pdt_xgmi_host_flag_alloc": [c_void_p, c_void_p],
    "pdt_xgmi_host_flag_free": [c_void_p],
    "pdt_xgmi_wallclock_khz": [],
    "pdt_bn_ws_floats": [c_int],
    "pdt_bn_ok": [c_int],
    "pdt_maxpool_ok": [c_int, c_int, c_int, c_int],
    "pdt_bn_stats_finalize": [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_maxpool_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_void_p],
    "pdt_maxpool_bwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_void_p],
    "pdt_bn_stats": [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p],
    "pdt_bn_finalize": [c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_bn_eval_coef": [c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_bn_apply": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p],
    "pdt_bn_bwd_reduce": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_bn_bwd_apply": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p],
    "pdt_conv3x3_igemm_ok": [c_int, c_int, c_int, c_int, c_int],
    "pdt_conv3x3_igemm": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_conv3x3_igemm_act": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_void_p],
    "pdt_l1_partials": [c_int64],
    "pdt_l1_fwd_grad": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p],
    "pdt_narrow_gemm_f32_ok": [c_int64, c_int, c_int],
    "pdt_narrow_gemm_f32_partials": [c_int64],
    "pdt_narrow_gemm_f32": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p,
                            c_int, c_int, c_void_p, c_void_p],
    "pdt_narrow_wgrad_f32_ok": [c_int64, c_int, c_int],
    "pdt_narrow_wgrad_f32": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_void_p],
    "pdt_narrow_wgrad_ok": [c_int64, c_int, c_int],
    "pdt_narrow_wgrad_ws_floats": [c_int64, c_int, c_int],
    "pdt_narrow_wgrad": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_void_p, c_int, c_void_p],
    "pdt_narrow_gemm_ok": [c_int64, c_int, c_int],
    "pdt_narrow_gemm_partials": [c_int64, c_int, c_int],
    "pdt_narrow_gemm": [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p, c_int, c_void_p,
                        c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "pdt_window_perm": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_window_perm_f32": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "pdt_im2col3x3": [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int, c_int, c_int, c_int, c_int, c_void_p,
                      c_int, c_void_p],
    "pdt_pixel_shuffle_affine_fwd": [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int, c_int, c_int, c_int, c_int,
                                     c_float, c_void_p, c_void_p, c_int, c_void_p],
    "pdt_pixel_shuffle_affine_bwd": [c_void_p, c_int64, c_int64, c_int64, c_int64, c_int, c_int, c_int, c_int, c_int,
                                     c_float, c_void_p, c_int, c_void_p],
    "pdt_swin_mlp_ok": [c_int, c_int],
    "pdt_swin_mlp_ws_floats": [c_int],
    "pdt_swin_mlp_bwd_blocks": [c_int64],
    "pdt_swin_mlp_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                         c_void_p],
    "pdt_swin_mlp_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_int, c_void_p, c_int, c_int64, c_int, c_int, c_void_p],
    "pdt_gemm_ok": [c_int, c_int64, c_int64, c_int64, c_int64, c_int64, c_int],
    "pdt_gemm_bf16": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                      c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "pdt_gemm_stamps_bf16": [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                             c_void_p, c_void_p],
    "pdt_gemm_stamps_epi_bf16": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64,
                                 c_int64, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_gemm2_bf16": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64,
                       c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "pdt_syncbn_stats": [c_void_p, c_int64, c_int, c_int64, c_int, c_void_p, c_void_p, c_void_p],
    "pdt_syncbn_finalize": [c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "pdt_syncbn_elemt": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int64, c_int,
                         c_int, c_void_p],
    "pdt_syncbn_bwd_reduce": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int64, c_int, c_void_p, c_void_p,
                              c_void_p],
    "pdt_syncbn_bwd_elemt": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_int64, c_int, c_int64, c_int, c_int, c_void_p],
}

_RET64 = {"pdt_swin_mlp_ws_floats", "pdt_narrow_wgrad_ws_floats", "pdt_fp8_gelu_bwd_ws_floats", "pdt_flash_attn_colsum_ws_floats"}

F32, BF16, F16, F64 = 0, 1, 2, 3


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float16:
        return F16
    if dt == torch.float64:
        return F64
    raise TypeError(f"unsupported dtype for HIP kernel: {dt}")


def lib_path() -> str:
    return _LIB_PATH


def load():
    """Return the loaded kernel library (raises if it cannot be loaded)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            _load_error = FileNotFoundError(
                f"{_LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or python -m pytorch_distributedtraining_amd._build)")
            raise _load_error
        lib = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = args
            fn.restype = ctypes.c_int64 if name in _RET64 else c_int
        _lib = lib
        return _lib


def available() -> bool:
    """True when a GPU is present and the HIP kernel library loads."""
    if not torch.cuda.is_available():
        return False
    try:
        load()
        return True
    except Exception:  # pragma: no cover - reported by require()
        return False


def require():
    """The kernel library, or a loud error (used by every GPU code path)."""
    try:
        return load()
    except Exception as e:  # pragma: no cover
        raise RuntimeError(f"pytorch_distributedtraining_amd HIP kernels unavailable: {e}") from e


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def check(err: int, name: str) -> None:
    if err != 0:
        raise RuntimeError(f"HIP kernel {name} failed with hipError_t={err}")


def call(name: str, *args) -> None:
    lib = require()
    check(getattr(lib, name)(*args), name)
