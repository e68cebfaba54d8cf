"""SwinIR (image super-resolution Swin Transformer) -- the model the reference trains in Stoke-DDP.py:206-208:
    SwinIR(upscale=2, in_chans=3, img_size=64, window_size=8, img_range=1., depths=[6]*4, embed_dim=60,
           num_heads=[6]*4, mlp_ratio=2, upsampler='pixelshuffledirect', resi_connection='1conv')
(SwinIR-S x2, 910,152 parameters per SURVEY.md §2.D).  Re-implemented from the published architecture
(Liang et al., ICCV-W 2021) with the upstream parameter names (conv_first, patch_embed.norm,
layers.{i}.residual_group.blocks.{j}.{norm1,attn.qkv,attn.proj,attn.relative_position_bias_table,
norm2,mlp.fc1,mlp.fc2}, layers.{i}.conv, norm, conv_after_body, upsample.0), so upstream checkpoints
keyed 'params' load with strict=True (Stoke-DDP.py:209-213).

MI355X notes (on GPU): LayerNorms run on the narrow-row HIP kernel (C = 60); window attention (64 tokens /
window, head_dim 10) on the fused MFMA kernels of ops/window_attention.py (relative-position bias + shift
mask applied in-register, never materialised); the 3x3 convolutions on im2col + hipBLASLt
(ops/conv.py; MIOpen has no bf16 implicit-GEMM solver for these channel counts); Linear weight gradients on
the row-split batched GEMM (ops/linear.py); the MLP's bias + erf-GELU fused.  ``to_stock_torch`` swaps
every one of them back to the stock torch module (the baseline of scripts/bench_torch_baseline.py).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activations import bias_gelu
from ..ops.conv import Conv2d3x3, pixel_shuffle_affine
from ..ops.linear import Linear, linear, linear_from_head_major, linear_head_major, linear_residual
from ..ops.swin_mlp import fused_mlp, fused_mlp_ok
from ..ops.norms import LayerNorm, add_layer_norm_from_windows, layer_norm_to_windows, window_norm_ok
from ..ops.window_attention import (fused_window_ok, head_major_ok, window_attention, window_attention_table,
                                    window_partition_shifted, window_reverse_shifted_add)

# PDT_SWINIR_FUSED_TAIL=0: stock PixelShuffle + de-normalisation (A/B of the fused HIP tail)
_FUSED_TAIL = os.environ.get("PDT_SWINIR_FUSED_TAIL", "1") == "1"
# PDT_SWIN_WINDOW_NORMS=0: separate roll / partition / reverse(+residual) passes instead of the window-mapped norms
WINDOW_NORMS = os.environ.get("PDT_SWIN_WINDOW_NORMS", "1") == "1"
# PDT_SWIN_REL_TABLE_KERNELS=0: relative-position bias gathered / scattered by torch ops (A/B)
REL_TABLE_KERNELS = os.environ.get("PDT_SWIN_REL_TABLE_KERNELS", "1") == "1"
# PDT_SWIN_HEAD_MAJOR_PROJ=0: the window attention writes its output token-major for the output projection (A/B)
HEAD_MAJOR_PROJ = os.environ.get("PDT_SWIN_HEAD_MAJOR_PROJ", "1") == "1"
# PDT_SWIN_MLP_RESIDUAL_GEMM=0: the unfused (fp32) MLP adds its residual in a separate pass (A/B)
MLP_RESIDUAL_GEMM = os.environ.get("PDT_SWIN_MLP_RESIDUAL_GEMM", "1") == "1"


def window_partition(x, ws):
    B, H, W, C = x.shape
    x = x.view(B, H // ws, ws, W // ws, ws, C)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)


def window_reverse(w, ws, H, W):
    B = w.shape[0] // ((H // ws) * (W // ws))
    x = w.view(B, H // ws, W // ws, ws, ws, -1)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, -1)


class _RelBiasGather(torch.autograd.Function):
    """table[idx] whose backward is one atomic index_add_ into the (225 x heads) table instead of the
    sort-based index backward (5-6 small kernels per block per micro-step on the GPU)."""

    @staticmethod
    def forward(ctx, table, idx):
        ctx.save_for_backward(idx)
        ctx.rows = table.shape[0]
        return table.index_select(0, idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        if torch.are_deterministic_algorithms_enabled():
            gt = torch.zeros((ctx.rows, g.shape[1]), dtype=g.dtype, device=g.device)
            return gt.index_put_((idx,), g, accumulate=True), None
        return torch.zeros((ctx.rows, g.shape[1]), dtype=g.dtype, device=g.device).index_add_(0, idx, g), None


class WindowAttention(nn.Module):
    def __init__(self, dim, window_size, num_heads, qkv_bias=True):
        super().__init__()
        self.dim, self.ws, self.num_heads = dim, window_size, num_heads
        self.scale = (dim // num_heads) ** -0.5
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * window_size - 1) ** 2, num_heads))
        coords = torch.stack(torch.meshgrid(torch.arange(window_size), torch.arange(window_size), indexing="ij"))
        cf = coords.flatten(1)
        rel = (cf[:, :, None] - cf[:, None, :]).permute(1, 2, 0).contiguous()
        rel[:, :, 0] += window_size - 1
        rel[:, :, 1] += window_size - 1
        rel[:, :, 0] *= 2 * window_size - 1
        self.register_buffer("relative_position_index", rel.sum(-1), persistent=True)
        self.qkv = Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = Linear(dim, dim)
        self.native = True    # False: stock torch path (SDPA + materialised bias), see to_stock_torch()
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)

    def forward(self, x, mask=None):
        Bw, N, C = x.shape
        h = self.num_heads
        if x.is_cuda and self.native:
            # fused HIP window attention: reads the qkv projection in place, never materialises the
            # [Bw, h, N, N] bias+mask or the scores (ops/window_attention.py)
            # the projection writes q / k / v head-major where the narrow GEMM computes it (ops.linear)
            hm = head_major_ok(x, N, h, C // h)
            qkv = linear_head_major(self.qkv, x, N, C // h) if hm else self.qkv(x)
            # bf16: the attention writes its output head-major and the projection reads it so (and its backward
            # hands dO back head-major) -- ops.linear.linear_from_head_major
            o_hm = HEAD_MAJOR_PROJ and hm and Bw * N >= 16384 and (
                torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype) == torch.bfloat16
            if REL_TABLE_KERNELS:
                # the table gather and its gradient scatter fused into two small kernels (ops.window_attention)
                out = window_attention_table(qkv, self.relative_position_bias_table, self.relative_position_index,
                                             mask, h, self.scale, out_head_major=o_hm)
            else:
                bias = _RelBiasGather.apply(self.relative_position_bias_table, self.relative_position_index.view(-1))
                out = window_attention(qkv, bias.view(N, N, h).permute(2, 0, 1), mask, h, self.scale,
                                       out_head_major=o_hm)
            return linear_from_head_major(self.proj, out)
        qkv = self.qkv(x).reshape(Bw, N, 3, h, C // h).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        bias = self.relative_position_bias_table[self.relative_position_index.view(-1)].view(N, N, h)
        bias = bias.permute(2, 0, 1).unsqueeze(0)                  # 1, h, N, N
        if mask is not None:
            nw = mask.shape[0]
            bias = (bias.unsqueeze(0) + mask.view(1, nw, 1, N, N)).expand(Bw // nw, nw, h, N, N).reshape(Bw, h, N, N)
        out = F.scaled_dot_product_attention(q, k, v, attn_mask=bias.to(q.dtype), scale=self.scale)
        return self.proj(out.transpose(1, 2).reshape(Bw, N, C))


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = Linear(hidden, dim)
        self.native = True

    def forward(self, x, residual=None):
        """MLP(x), plus ``residual`` when given (fused into the kernel's epilogue on the fused path)."""
        if x.is_cuda and self.native:
            if fused_mlp_ok(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias) and (
                    residual is None or (residual.dtype == torch.bfloat16 and residual.shape == x.shape)):
                # C = 60 -> 120 -> 60: whole MLP in one MFMA kernel per direction (hidden kept on chip)
                return fused_mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, residual)
            # GEMM without bias -> fused bias + erf-GELU kernel (backward also reduces the bias gradient); the
            # residual added in fc2's GEMM store
            h = linear(x, self.fc1.weight)
            a = bias_gelu(h, self.fc1.bias, approximate="none")
            if MLP_RESIDUAL_GEMM and residual is not None and residual.dtype == a.dtype == self.fc2.weight.dtype \
                    and not torch.is_autocast_enabled("cuda"):
                return linear_residual(a, self.fc2.weight, self.fc2.bias, residual)
            y = self.fc2(a)
        else:
            y = self.fc2(self.act(self.fc1(x)))
        return y if residual is None else residual + y


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim, input_resolution, num_heads, window_size=8, shift_size=0, mlp_ratio=2.0):
        super().__init__()
        self.dim, self.input_resolution, self.num_heads = dim, input_resolution, num_heads
        self.window_size, self.shift_size = window_size, shift_size
        if min(input_resolution) <= window_size:
            self.shift_size, self.window_size = 0, min(input_resolution)
        self.norm1 = LayerNorm(dim)
        self.attn = WindowAttention(dim, self.window_size, num_heads)
        self.norm2 = LayerNorm(dim)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))
        self.register_buffer("attn_mask", self._mask(input_resolution) if self.shift_size > 0 else None,
                             persistent=False)

    def _mask(self, res):
        H, W = res
        ws, ss = self.window_size, self.shift_size
        img = torch.zeros(1, H, W, 1)
        cnt = 0
        for hs in (slice(0, -ws), slice(-ws, -ss), slice(-ss, None)):
            for wsl in (slice(0, -ws), slice(-ws, -ss), slice(-ss, None)):
                img[:, hs, wsl, :] = cnt
                cnt += 1
        mw = window_partition(img, ws).squeeze(-1)
        m = mw.unsqueeze(1) - mw.unsqueeze(2)
        return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)

    def _mask_for(self, H, W, device):
        """Shifted-window mask for an H x W input, built once per resolution / device and kept (no host-built
        mask + H2D copy per forward; required for HIP-graph capture of the step)."""
        if (H, W) == tuple(self.input_resolution) and self.attn_mask.device == device:
            return self.attn_mask
        cache = self.__dict__.setdefault("_mask_cache", {})
        m = cache.get((H, W, device))
        if m is None:
            m = cache[(H, W, device)] = self._mask((H, W)).to(device)
        return m

    def forward(self, x, x_size):
        H, W = x_size
        B, L, C = x.shape
        if self.attn.native and fused_window_ok(x, H, W, self.window_size, self.shift_size) and (
                x.dtype == torch.bfloat16 or not torch.is_autocast_enabled()):
            # roll + partition and reverse + roll + residual add as one permutation pass each (bf16, or fp32 --
            # the reference's own precision -- when no autocast region would mix the two)
            if self.shift_size > 0:
                mask = self._mask_for(H, W, x.device)
            else:
                mask = None
            ws, ss = self.window_size, self.shift_size
            if WINDOW_NORMS and window_norm_ok(x, H, W, ws, ss) and self.norm1.weight.dtype == self.norm2.weight.dtype:
                # the roll / partition / reverse permutations ride inside the two LayerNorms (ops.norms WinMap):
                # norm1 writes window order, norm2 reads the attention output from window order
                # (xs: x passed through norm1, so the residual's gradient is added inside norm1's backward pass)
                win, xs = layer_norm_to_windows(x, self.norm1.weight, self.norm1.bias, self.norm1.eps, H, W, ws, ss)
                a = self.attn(win, mask=mask).to(x.dtype)
                y, s = add_layer_norm_from_windows(xs, a, self.norm2.weight, self.norm2.bias, self.norm2.eps, H, W,
                                                   ws, ss)
                return self.mlp(y, residual=s)
            h = self.norm1(x).to(x.dtype)
            win = window_partition_shifted(h, H, W, ws, ss)
            a = self.attn(win, mask=mask).to(x.dtype)
            x = window_reverse_shifted_add(a, x, H, W, ws, ss)
            return self.mlp(self.norm2(x), residual=x)
        sc = x
        x = self.norm1(x).view(B, H, W, C)
        if self.shift_size > 0:
            x = torch.roll(x, shifts=(-self.shift_size, -self.shift_size), dims=(1, 2))
        if self.shift_size > 0:
            mask = self._mask_for(H, W, x.device)
        else:
            mask = None
        a = self.attn(window_partition(x, self.window_size), mask=mask)
        x = window_reverse(a, self.window_size, H, W)
        if self.shift_size > 0:
            x = torch.roll(x, shifts=(self.shift_size, self.shift_size), dims=(1, 2))
        x = sc + x.reshape(B, L, C)
        return x + self.mlp(self.norm2(x))


class BasicLayer(nn.Module):
    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio):
        super().__init__()
        self.blocks = nn.ModuleList([
            SwinTransformerBlock(dim, input_resolution, num_heads, window_size,
                                 0 if i % 2 == 0 else window_size // 2, mlp_ratio) for i in range(depth)])

    def forward(self, x, x_size):
        for b in self.blocks:
            x = b(x, x_size)
        return x


class RSTB(nn.Module):
    """Residual Swin Transformer Block ('1conv' residual connection)."""

    def __init__(self, dim, input_resolution, depth, num_heads, window_size, mlp_ratio):
        super().__init__()
        self.residual_group = BasicLayer(dim, input_resolution, depth, num_heads, window_size, mlp_ratio)
        self.conv = Conv2d3x3(dim, dim)

    def forward(self, x, x_size):
        B, L, C = x.shape
        y = self.residual_group(x, x_size)
        y = y.transpose(1, 2).reshape(B, C, *x_size)
        return self.conv(y).flatten(2).transpose(1, 2) + x


class PatchEmbed(nn.Module):
    def __init__(self, embed_dim, norm=True):
        super().__init__()
        self.norm = LayerNorm(embed_dim) if norm else None

    def forward(self, x):
        x = x.flatten(2).transpose(1, 2)
        return self.norm(x) if self.norm is not None else x


class SwinIR(nn.Module):
    def __init__(self, img_size=64, in_chans=3, embed_dim=60, depths=(6, 6, 6, 6), num_heads=(6, 6, 6, 6),
                 window_size=8, mlp_ratio=2.0, upscale=2, img_range=1.0, upsampler="pixelshuffledirect",
                 resi_connection="1conv", **_ignored):
        super().__init__()
        if upsampler != "pixelshuffledirect" or resi_connection != "1conv":
            raise NotImplementedError("this build implements the lightweight SwinIR-S path used by the reference "
                                      "(upsampler='pixelshuffledirect', resi_connection='1conv')")
        self.img_range, self.upscale, self.window_size = img_range, upscale, window_size
        self.register_buffer("mean", torch.tensor([0.4488, 0.4371, 0.4040]).view(1, 3, 1, 1) if in_chans == 3
                             else torch.zeros(1, 1, 1, 1), persistent=False)
        self.conv_first = Conv2d3x3(in_chans, embed_dim)
        self.patch_embed = PatchEmbed(embed_dim, norm=True)
        res = (img_size, img_size)
        self.layers = nn.ModuleList([RSTB(embed_dim, res, d, h, window_size, mlp_ratio)
                                     for d, h in zip(depths, num_heads)])
        self.norm = LayerNorm(embed_dim)
        self.conv_after_body = Conv2d3x3(embed_dim, embed_dim)
        self.upsample = nn.Sequential(Conv2d3x3(embed_dim, upscale ** 2 * in_chans), nn.PixelShuffle(upscale))
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)

    def _pad(self, x):
        _, _, h, w = x.shape
        ph = (self.window_size - h % self.window_size) % self.window_size
        pw = (self.window_size - w % self.window_size) % self.window_size
        return F.pad(x, (0, pw, 0, ph), "reflect") if (ph or pw) else x

    def forward_features(self, x):
        x_size = (x.shape[2], x.shape[3])
        t = self.patch_embed(x)
        for layer in self.layers:
            t = layer(t, x_size)
        t = self.norm(t)
        B, L, C = t.shape
        return t.transpose(1, 2).reshape(B, C, *x_size)

    def forward(self, x):
        H, W = x.shape[2:]
        x = self._pad(x)
        mean = self.mean.to(x.dtype)
        x = (x - mean) * self.img_range
        x = self.conv_first(x)
        x = self.conv_after_body(self.forward_features(x)) + x
        if x.is_cuda and _FUSED_TAIL and isinstance(self.upsample[0], Conv2d3x3):
            # conv -> PixelShuffle -> x / img_range + mean as conv + ONE fused HIP pass
            y = self.upsample[0](x)
            x = pixel_shuffle_affine(y, self.upscale, 1.0 / self.img_range, mean)
            dt = torch.promote_types(y.dtype, mean.dtype)    # the unfused tail's type promotion
            x = x if x.dtype == dt else x.to(dt)
        else:
            x = self.upsample(x)
            x = x / self.img_range + mean
        return x[:, :, : H * self.upscale, : W * self.upscale]


def to_stock_torch(model: nn.Module) -> nn.Module:
    """Swap the HIP-kernel layers for stock torch ones (nn.LayerNorm, SDPA window attention) in place --
    same parameters and state_dict keys; used by the stock PyTorch-ROCm baseline benchmark."""
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, LayerNorm):
                ln = nn.LayerNorm(child.normalized_shape, eps=child.eps).to(child.weight.device)
                ln.load_state_dict(child.state_dict())
                setattr(mod, cname, ln)
            elif isinstance(child, Linear):
                li = nn.Linear(child.in_features, child.out_features, bias=child.bias is not None)
                li = li.to(child.weight.device)
                li.load_state_dict(child.state_dict())
                setattr(mod, cname, li)
            elif isinstance(child, Conv2d3x3):
                cv = nn.Conv2d(child.in_channels, child.out_channels, 3, 1, 1).to(child.weight.device)
                cv.load_state_dict(child.state_dict())
                setattr(mod, cname, cv)
        if isinstance(mod, (WindowAttention, Mlp)):
            mod.native = False
    return model


def swinir_s_x2(**kw):
    """The reference's exact configuration (Stoke-DDP.py:206-208)."""
    cfg = dict(upscale=2, in_chans=3, img_size=64, window_size=8, img_range=1.0, depths=[6, 6, 6, 6], embed_dim=60,
               num_heads=[6, 6, 6, 6], mlp_ratio=2, upsampler="pixelshuffledirect", resi_connection="1conv")
    cfg.update(kw)
    return SwinIR(**cfg)
