"""Llama-3 family (BASELINE.json config 5: Llama-3 8B FSDP full-shard + fused AdamW + activation
checkpointing).  Architecture from the public Llama-3 description (RMSNorm pre-norm, RoPE theta 5e5,
GQA 32q/8kv heads of 128, SwiGLU FFN 14336, vocab 128256), random init.

MI355X-first layout: one fused q|k|v projection (``attention.wqkv``) and one fused gate|up projection
(``feed_forward.w13``) so each block issues 4 large GEMMs instead of 7; RMSNorm / RoPE / SwiGLU /
GQA flash attention / cross-entropy run on the HIP kernels.  ``convert_meta_state_dict`` maps Meta-style
checkpoints (wq/wk/wv, w1/w3) onto the fused layout and ``export_meta_state_dict`` maps back (bitwise: the fused
weights are row concatenations), so a checkpoint saved here loads into a standard Meta-layout Llama
(``Trainer(portable_checkpoint=True)`` writes that layout into the envelope).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import cross_entropy, rope_tables, swiglu
from ..ops.attention import flash_attn_gqa_packed
from ..ops.rope import apply_rope_qk_
from ..ops.embedding import Embedding
from ..ops.fp8 import fp8_enabled, fp8_recompute_safe
from ..ops.linear import Linear, linear_residual
from ..ops.norms import RMSNorm, rms_norm
from ..utils import recompute
from . import gpt2 as _gpt2


@dataclass
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    vocab_size: int = 128256
    ffn_dim: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192
    activation_checkpointing: bool = False
    # how many of the layers (the first ones) are checkpointed; None = all of them when activation_checkpointing is
    # on.  With 288 GB of HBM most of the recompute can be bought back (bench.py --act-ckpt-layers auto sizes it)
    checkpoint_layers: int | None = None
    # "full": a checkpointed layer re-runs its whole forward in backward (torch.utils.checkpoint); "selective": it
    # keeps its GEMM outputs (qkv, gate/up) and residual stream and recomputes only the norms, the attention
    # forward and SwiGLU when backward needs their outputs (utils.recompute) -- no GEMM runs twice
    checkpoint_policy: str = "full"

    @property
    def head_dim(self):
        return self.dim // self.n_heads


LLAMA_CONFIGS = {
    "llama3-8b": dict(),
    "llama3-1b": dict(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192),
    "llama3-tiny": dict(dim=256, n_layers=2, n_heads=2, n_kv_heads=1, ffn_dim=512, vocab_size=1024, max_seq_len=512),
}


def llama_config(name="llama3-8b", **overrides):
    kw = dict(LLAMA_CONFIGS[name])
    kw.update(overrides)
    return LlamaConfig(**kw)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.h, self.hkv, self.d = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        self.wqkv = Linear(cfg.dim, (self.h + 2 * self.hkv) * self.d, bias=False)
        self.wo = Linear(self.h * self.d, cfg.dim, bias=False)

    def forward(self, x, cos, sin, residual=None):
        B, S, _ = x.shape
        qkv = apply_rope_qk_(self.wqkv(x), self.h, self.hkv, self.d, cos, sin)
        qkv = qkv.view(B, S, self.h + 2 * self.hkv, self.d)
        # RoPE rotates the q and k heads of the packed projection in place and the packed GQA flash attention
        # reads q / k / v as head ranges of it (and writes ONE packed gradient): no separate rotated q / k
        # tensors and no gradient scatter into the packed layout
        o = flash_attn_gqa_packed(qkv, self.h, self.hkv, causal=True)
        o2 = o.reshape(B, S, self.h * self.d)
        r = getattr(o, "_pdt_recipe", None)          # selective recompute: wo's saved input is the same forward
        if r is not None:
            recompute.tag(o2, r[0], r[1], view=lambda t: t.reshape(B, S, self.h * self.d))
        if residual is not None:   # + the residual stream, added by the wo GEMM (ops.linear.linear_residual)
            return linear_residual(o2, self.wo.weight, None, residual)
        return self.wo(o2)


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.w13 = Linear(cfg.dim, 2 * cfg.ffn_dim, bias=False)
        self.w2 = Linear(cfg.ffn_dim, cfg.dim, bias=False)

    def forward(self, x, residual=None):
        g = self.w13(x)
        a = swiglu(g)
        recompute.tag(a, recompute.Recipe(lambda: swiglu(g)))   # (only inside selective_recompute)
        if residual is not None:
            return linear_residual(a, self.w2.weight, None, residual)
        return self.w2(a)


class LlamaBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attention_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x, cos, sin, pending=None):
        """(x, pending) -> (x', ffn_out); residual adds fused into the next RMSNorm kernel.  Inside
        ``utils.recompute.selective_recompute()`` the norm outputs are saved as recipes over the residual stream.
        RESID_GEMM mode: (x, None) -> (x'', None), wo and w2 add their outputs to the stream in the GEMM and the
        norms pass the summed stream through (``ops.norms.norm_pass``)."""
        if _resid_mode(x):
            h, x = self.attention_norm.forward_pass(x) if pending is None else \
                self.attention_norm.forward_add(x, pending)
            _tag_norm(h, x, self.attention_norm)
            x = self.attention(h, cos, sin, residual=x)
            y, x = self.ffn_norm.forward_pass(x)
            _tag_norm(y, x, self.ffn_norm)
            return self.feed_forward(y, residual=x), None
        if pending is None:
            h = self.attention_norm(x)
        else:
            h, x = self.attention_norm.forward_add(x, pending)
        _tag_norm(h, x, self.attention_norm)
        y, x = self.ffn_norm.forward_add(x, self.attention(h, cos, sin))
        _tag_norm(y, x, self.ffn_norm)
        return x, self.feed_forward(y)


def _resid_mode(x) -> bool:
    """wo / w2 add the residual stream in their GEMMs (PDT_RESID_GEMM, models.gpt2): bf16 on the GPU, no fp8."""
    return (_gpt2.RESID_GEMM and x.is_cuda and x.dtype == torch.bfloat16 and not fp8_enabled()
            and not torch.is_autocast_enabled("cuda"))


def _tag_norm(out, s, norm):
    """norm(s) is exactly ``out`` (the fused add-norm normalises the rounded sum it stores): saved as that recipe."""
    if recompute.active():
        w, eps = norm.weight, norm.eps
        recompute.tag(out, recompute.Recipe(lambda: rms_norm(s, w, eps)))


class Llama(nn.Module):
    block_class = LlamaBlock

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        self.tok_embeddings = Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList([LlamaBlock(cfg) for _ in range(cfg.n_layers)])
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.output = Linear(cfg.dim, cfg.vocab_size, bias=False)
        cos, sin = rope_tables(cfg.head_dim, cfg.max_seq_len, cfg.rope_theta)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)
        self.reset_parameters()

    def reset_parameters(self):
        std = 0.02
        out_std = 0.02 / math.sqrt(2 * self.config.n_layers)
        for n, p in self.named_parameters():
            if p.dim() == 2:
                nn.init.normal_(p, 0.0, out_std if (n.endswith("wo.weight") or n.endswith("w2.weight")) else std)
            else:
                nn.init.ones_(p)

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def flops_per_token(self, seq_len, causal: bool = True):
        """6N (N without the embedding table) + causal attention 6 L S d (12 L S d with ``causal=False``): see
        ``GPT2.flops_per_token``."""
        c = self.config
        n = self.num_params() - self.tok_embeddings.weight.numel()
        return 6 * n + (6 if causal else 12) * c.n_layers * seq_len * c.dim

    def to_portable_state_dict(self, sd: dict) -> dict:
        """This module's (fused) state dict -> the Meta layout (``export_meta_state_dict``)."""
        return export_meta_state_dict(sd, self.config)

    def from_portable_state_dict(self, sd: dict) -> dict:
        """A Meta-layout state dict -> this module's fused layout; a fused one passes through."""
        return convert_meta_state_dict(sd, self.config) if any(".attention.wq." in k for k in sd) else sd

    def forward(self, tokens, labels=None):
        S = tokens.shape[1]
        x = self.tok_embeddings(tokens)
        cos, sin = self.rope_cos[:S], self.rope_sin[:S]
        pending = None
        n_ckpt = self.config.checkpoint_layers if self.config.checkpoint_layers is not None else len(self.layers)
        selective = self.config.checkpoint_policy == "selective"
        for i, layer in enumerate(self.layers):
            ckpt = self.config.activation_checkpointing and self.training and i < n_ckpt
            if ckpt and selective:
                with recompute.selective_recompute():
                    x, pending = layer(x, cos, sin, pending)
            elif ckpt:
                x, pending = torch.utils.checkpoint.checkpoint(fp8_recompute_safe(layer), x, cos, sin, pending,
                                                               use_reentrant=False)
            else:
                x, pending = layer(x, cos, sin, pending)
        h = self.norm(x) if pending is None else self.norm.forward_add(x, pending)[0]
        logits = self.output(h)
        if labels is None:
            return logits
        # training: the gradient is written over the (dead) logits in the forward's single read; eval keeps them
        return cross_entropy(logits, labels, inplace_backward=True, grad_in_forward=self.training)


def build_llama(name="llama3-8b", **overrides) -> Llama:
    return Llama(llama_config(name, **overrides))


def convert_meta_state_dict(sd: dict, cfg: LlamaConfig) -> dict:
    """Meta-format Llama checkpoint (tok_embeddings, layers.i.attention.{wq,wk,wv,wo},
    feed_forward.{w1,w2,w3}, {attention,ffn}_norm, norm, output) -> this module's fused layout."""
    out = {}
    for k, v in sd.items():
        if ".attention.wq." in k:
            base = k.replace(".attention.wq.", ".attention.wqkv.")
            out[base] = torch.cat([v, sd[k.replace(".wq.", ".wk.")], sd[k.replace(".wq.", ".wv.")]], 0)
        elif ".attention.wk." in k or ".attention.wv." in k or ".feed_forward.w3." in k:
            continue
        elif ".feed_forward.w1." in k:
            out[k.replace(".w1.", ".w13.")] = torch.cat([v, sd[k.replace(".w1.", ".w3.")]], 0)
        else:
            out[k] = v
    return out


def export_meta_state_dict(sd: dict, cfg: LlamaConfig) -> dict:
    """Inverse of ``convert_meta_state_dict``: attention.wqkv -> wq | wk | wv (rows H*d | Hkv*d | Hkv*d) and
    feed_forward.w13 -> w1 | w3 (rows ffn_dim each), every other key unchanged; views are cloned so the result
    owns its storage."""
    nq, nkv = cfg.n_heads * cfg.head_dim, cfg.n_kv_heads * cfg.head_dim
    out = {}
    for k, v in sd.items():
        if ".attention.wqkv." in k:
            q, kk, vv = torch.split(v, [nq, nkv, nkv], 0)
            for name, t in ((".wq.", q), (".wk.", kk), (".wv.", vv)):
                out[k.replace(".wqkv.", name)] = t.clone()
        elif ".feed_forward.w13." in k:
            w1, w3 = torch.split(v, [cfg.ffn_dim, cfg.ffn_dim], 0)
            out[k.replace(".w13.", ".w1.")] = w1.clone()
            w2k = k.replace(".w13.", ".w2.")
            if w2k in sd:
                out[w2k] = sd[w2k]
            out[k.replace(".w13.", ".w3.")] = w3.clone()
        elif ".feed_forward.w2." in k and k.replace(".w2.", ".w13.") in sd:
            continue                          # emitted next to w1 / w3 above
        else:
            out[k] = v
    return out
