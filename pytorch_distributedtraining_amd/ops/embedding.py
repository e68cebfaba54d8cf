"""Embedding with a graph-capturable HIP backward (``csrc/kernels/embedding.hip``).

Forward is torch's gather (F.embedding).  Under HIP-graph capture the backward replaces torch's dense
embedding backward, whose sort + device-wide unique/partition (rocprim) has data-dependent sizes above
3,072 indices and faulted when a DDP-wrapped GPT-2 124M step was replayed from a HIP graph, with a
fixed-shape fp32 atomic scatter-add followed by one cast to the weight dtype.  Eager steps keep torch's
sort-based backward: at LM shapes the atomic scatter is the slower of the two (1.3B flagship: +7.5 ms/step).  ``Embedding`` subclasses nn.Embedding (same parameters / keys).
Used for the GPT-2 token embedding (tied with the LM head) and Llama's token embedding.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

FORCE_SCATTER = False     # tests: run the HIP scatter backward outside graph capture too


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, idx):
        ctx.save_for_backward(idx)
        ctx.shape = weight.shape
        ctx.dtype = weight.dtype
        return F.embedding(idx, weight)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        v, d = ctx.shape
        if not (FORCE_SCATTER or torch.cuda.is_current_stream_capturing()):
            # eager: torch's sort-based backward is ~10x faster than fp32 atomics at LM shapes (the atomic
            # scatter cost the 1.3B flagship 7.5 ms/step: 67M atomics at ~11/cycle chip-wide)
            return torch.ops.aten.embedding_dense_backward(dy, idx, v, -1, False), None
        dy2 = dy.reshape(-1, d)
        if dy2.dtype not in (torch.float32, torch.bfloat16):
            dy2 = dy2.float()
        dy2 = dy2.contiguous()
        ids = idx.reshape(-1).to(torch.int64).contiguous()
        acc = torch.empty(v, d, dtype=torch.float32, device=dy.device)
        out = acc if ctx.dtype == torch.float32 else torch.empty(v, d, dtype=ctx.dtype, device=dy.device)
        _lib.call("pdt_embedding_bwd", ids.data_ptr(), dy2.data_ptr(), _lib.dtype_code(dy2.dtype), acc.data_ptr(),
                  out.data_ptr(), _lib.dtype_code(ctx.dtype), ids.numel(), d, v, _lib.stream_handle(dy.device))
        return out, None


def embedding(idx: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if weight.is_cuda and weight.requires_grad and torch.is_grad_enabled() and \
            weight.dtype in (torch.float32, torch.bfloat16):
        return _EmbeddingFn.apply(weight, idx)
    return F.embedding(idx, weight)


class Embedding(nn.Embedding):
    def forward(self, idx):
        if self.padding_idx is not None or self.max_norm is not None or self.scale_grad_by_freq or self.sparse:
            return super().forward(idx)
        return embedding(idx, self.weight)
