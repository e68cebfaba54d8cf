"""GPT-2 family (124M / 350M / 774M / 1.3B) built on the gfx950 kernels.

BASELINE.json configs 3 (GPT-2 124M DDP) and 4 (GPT-2 1.3B FSDP, the flagship bench).
MI355X-first choices:
  * attention = one fused qkv GEMM (hipBLASLt) -> ``flash_attn_qkvpacked`` (hand MFMA kernel) reading
    the [B, S, 3, H, D] projection in place and writing dq/dk/dv into one packed gradient;
  * MLP = GEMM without bias -> fused bias+GELU(tanh) kernel (saves the pre-activation once);
  * LayerNorm = wave-per-row HIP kernel (bf16 activations, fp32 statistics);
  * LM head tied to the token embedding, loss = fused softmax-CE with in-place backward;
  * vocab padded to a multiple of 128 (50257 -> 50304) so the head GEMM tiles cleanly;
  * dropout omitted (0.0), as in throughput benchmarks of this class.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops import bias_gelu, cross_entropy, flash_attn_qkvpacked
from ..ops.embedding import Embedding
from ..ops.fp8 import fp8_enabled, fp8_gelu_mlp, fp8_gelu_mlp_ok, fp8_recompute_safe
from ..ops.linear import Linear, gelu_mlp, gelu_mlp_ok, linear, linear_bias_gelu, linear_bias_gelu_ok, linear_residual
from ..ops.norms import LayerNorm


@dataclass
class GPT2Config:
    vocab_size: int = 50304
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    activation_checkpointing: bool = False
    # selective checkpointing: how many of the layers (the first ones) recompute their forward in backward;
    # None = all of them when activation_checkpointing is on.  With 288 GB of HBM most of the recompute can be
    # bought back (bench.py --act-ckpt-layers auto sizes it to the memory)
    checkpoint_layers: int | None = None

    @property
    def head_dim(self):
        return self.n_embd // self.n_head


GPT2_CONFIGS = {
    "gpt2-124m": dict(n_embd=768, n_layer=12, n_head=12),
    "gpt2-350m": dict(n_embd=1024, n_layer=24, n_head=16),
    "gpt2-774m": dict(n_embd=1280, n_layer=36, n_head=20),
    # GPT-2 "1.3B" (GPT-3 XL shape): L24, d2048; 16 heads x 128 keeps head_dim MFMA-friendly
    "gpt2-1.3b": dict(n_embd=2048, n_layer=24, n_head=16),
    "gpt2-tiny": dict(n_embd=128, n_layer=2, n_head=2, vocab_size=512, n_positions=256),
}


# attention c_proj bias folded into ln_2's fused residual-add kernel (its gradient from the norm backward's pass)
FOLD_PROJ_BIAS = os.environ.get("PDT_FOLD_PROJ_BIAS", "1") == "1"
# residual adds in the projection GEMMs (hipBLASLt's accumulate input reads the stream in the epilogue): the norms
# then read one stream and write one output instead of summing two (``ops.norms.norm_pass``).  Flagship shapes
# (profiles/r5/r5u_resid_gemm_ab.txt): attention c_proj 604 -> 641 us, MLP c_proj 2,156 -> 2,152 us, each norm
# 292 -> 178 us: 649.8 / 653.5 -> 646.9 / 649.0 ms per step.  PDT_RESID_GEMM=0 restores the norm-side adds.
RESID_GEMM = os.environ.get("PDT_RESID_GEMM", "1") == "1"


def _resid_mode(x, mlp) -> bool:
    """Projection GEMMs add the residual stream (RESID_GEMM): bf16 on the GPU, the fused MLP path, no fp8."""
    return (RESID_GEMM and FOLD_PROJ_BIAS and x.is_cuda and x.dtype == torch.bfloat16 and not fp8_enabled()
            and not torch.is_autocast_enabled("cuda")
            and gelu_mlp_ok(x, mlp.c_fc.weight, mlp.c_fc.bias, mlp.c_proj.weight, mlp.c_proj.bias))


def gpt2_config(name: str, **overrides) -> GPT2Config:
    kw = dict(GPT2_CONFIGS[name])
    kw.update(overrides)
    return GPT2Config(**kw)


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.n_head = cfg.n_head
        self.head_dim = cfg.head_dim
        self.c_attn = Linear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = Linear(cfg.n_embd, cfg.n_embd)

    def forward(self, x, fold_bias: bool = False, residual=None):
        """Attention branch output; with ``fold_bias`` the pair (c_proj(y) without its bias, the bias) for a
        consumer that adds the bias itself (the block's fused residual-add + LayerNorm, whose backward then
        returns the bias gradient from its own pass instead of a separate column sum over dY); with ``residual``
        the stream plus the branch, summed by the c_proj GEMM."""
        B, S, C = x.shape
        qkv = self.c_attn(x).view(B, S, 3, self.n_head, self.head_dim)
        # c_attn's bias gradient comes out of the attention backward kernels (per-workgroup column sums of the
        # dq / dk / dv rows they store), not from a separate pass over the [tokens, 3C] gradient
        y = flash_attn_qkvpacked(qkv, causal=True, bias_grad=self.c_attn.bias is not None).reshape(B, S, C)
        if residual is not None:
            return linear_residual(y, self.c_proj.weight, self.c_proj.bias, residual)
        if fold_bias:
            return self.c_proj.matmul(y), self.c_proj.bias
        return self.c_proj(y)


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = Linear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = Linear(4 * cfg.n_embd, cfg.n_embd)

    def forward(self, x, residual=None):
        if residual is not None:   # (the caller checked _resid_mode) + the stream, summed by the c_proj GEMM
            return gelu_mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias, residual)
        if fp8_enabled():
            m1, m2 = self.c_fc._fp8_meta(x), self.c_proj._fp8_meta(x)
            if m1 is not None and m2 is not None and fp8_gelu_mlp_ok(x, self.c_fc.weight, self.c_fc.bias,
                                                                    self.c_proj.weight, self.c_proj.bias):
                # fp8 GEMMs with bias + GELU fused into the casts (the bf16 hidden never reaches HBM)
                return fp8_gelu_mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias, m1, m2)
        if gelu_mlp_ok(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias):
            # c_fc + bias + GELU fused forward, c_proj dgrad + GELU backward + c_fc bias gradient fused backward
            return gelu_mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias)
        if linear_bias_gelu_ok(x, self.c_fc.weight, self.c_fc.bias):
            # bias + GELU in the hand GEMM's epilogue (ops.linear.linear_bias_gelu)
            return self.c_proj(linear_bias_gelu(x, self.c_fc.weight, self.c_fc.bias))
        h = self.c_fc.matmul(x)                      # GEMM without bias: the bias is folded into the GELU kernel
        h = bias_gelu(h, self.c_fc.bias, approximate="tanh")
        return self.c_proj(h)


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.mlp = MLP(cfg)

    def forward(self, x, pending=None, pending_colsum=False):
        """(x, pending) -> (x', mlp_out): the residual adds are fused into the following LayerNorm
        kernels (``pending`` is the previous block's branch output not yet added to the stream;
        ``pending_colsum``: it came from a biased Linear, whose bias gradient ln_1's backward sums).
        RESID_GEMM mode: (x, None) -> (x'', None), the branch outputs added to the stream by the projection GEMMs
        and the norms reading the summed stream (``pending`` None: x already holds the previous block's MLP)."""
        if pending is None:
            h, x = self.ln_1.forward_pass(x, r_colsum=pending_colsum)
        else:
            h, x = self.ln_1.forward_add(x, pending, r_colsum=pending_colsum and FOLD_PROJ_BIAS)
        if _resid_mode(h, self.mlp):
            x = self.attn(h, residual=x)
            y, x = self.ln_2.forward_pass(x, r_colsum=self.attn.c_proj.bias is not None)
            return self.mlp(y, residual=x), None
        if FOLD_PROJ_BIAS:
            a, a_bias = self.attn(h, fold_bias=True)   # c_proj's bias joins the residual sum in ln_2's kernel
            y, x = self.ln_2.forward_add(x, a, a_bias)
        else:
            y, x = self.ln_2.forward_add(x, self.attn(h))
        return x, self.mlp(y)


class GPT2LMHeadModel(nn.Module):
    """forward(input_ids, labels=None) -> loss (if labels) else logits."""

    block_class = GPT2Block

    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.config = cfg
        self.wte = Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        # which blocks' MLP c_proj carries a bias (read at build time: FSDP later swaps parameters in and out)
        self._mlp_proj_bias = [blk.mlp.c_proj.bias is not None for blk in self.h]
        self.reset_parameters()

    def reset_parameters(self):
        std = 0.02
        proj_std = 0.02 / math.sqrt(2 * self.config.n_layer)
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, proj_std)
            elif name.endswith(".weight") and p.dim() == 2:
                nn.init.normal_(p, 0.0, std)
            elif name.endswith(".bias"):
                nn.init.zeros_(p)
        for m in self.modules():
            if isinstance(m, LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def num_params(self, non_embedding=False):
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.wpe.weight.numel()
        return n

    def flops_per_token(self, seq_len: int, causal: bool = True) -> float:
        """Training FLOPs per token: 6N (N without the position table) + attention.  Attention is QK^T and PV,
        4 S d per token per layer forward, x3 for training = 12 L S d with every score computed; a causal mask
        makes half of them useful, so the default (``causal=True``) counts 6 L S d -- the work this model
        actually needs.  ``causal=False`` is the full-matrix convention some MFU figures use."""
        c = self.config
        n = self.num_params(non_embedding=True)
        return 6 * n + (6 if causal else 12) * c.n_layer * seq_len * c.n_embd

    def forward(self, input_ids, labels=None):
        B, S = input_ids.shape
        x = self.wte(input_ids)
        # positions are 0..S-1: the first S rows of the table, no gather (its backward was a sort-based
        # embedding_dense_backward over B*S indices; now a slice copy of S rows)
        pending = self.wpe.weight[:S].unsqueeze(0).expand(B, S, -1)
        n_ckpt = self.config.checkpoint_layers if self.config.checkpoint_layers is not None else len(self.h)
        for i, blk in enumerate(self.h):
            # block i > 0 receives the previous MLP's c_proj output (biased Linear): ln_1 sums its gradient
            colsum = i > 0 and self._mlp_proj_bias[i - 1] and not fp8_enabled()
            if self.config.activation_checkpointing and self.training and i < n_ckpt:
                x, pending = torch.utils.checkpoint.checkpoint(fp8_recompute_safe(blk), x, pending, colsum,
                                                               use_reentrant=False)
            else:
                x, pending = blk(x, pending, colsum)
        last = self._mlp_proj_bias[-1] and not fp8_enabled() and FOLD_PROJ_BIAS
        if pending is None:       # RESID_GEMM: the last MLP's c_proj already added its output to the stream
            x, _ = self.ln_f.forward_pass(x, r_colsum=last)
        else:
            x, _ = self.ln_f.forward_add(x, pending, r_colsum=last)
        logits = linear(x, self.wte.weight)     # tied head (framework linear: transposed-layout dgrad)
        if labels is None:
            return logits
        # training: the gradient is written over the (dead) logits in the forward's single read; eval keeps them
        return cross_entropy(logits, labels, inplace_backward=True, grad_in_forward=self.training)


def build_gpt2(name: str = "gpt2-124m", **overrides) -> GPT2LMHeadModel:
    return GPT2LMHeadModel(gpt2_config(name, **overrides))
