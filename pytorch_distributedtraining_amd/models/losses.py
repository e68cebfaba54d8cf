"""Losses used by the reference workloads.

* ``feat_loss`` / ``PerceptualLoss`` -- the perceptual (feature-space) loss of Stoke-DDP.py:35,224
  (module ``PyTorchPercept``, absent from the reference, SURVEY.md F4: callable (outputs, targets) ->
  scalar).  A frozen VGG-16-style feature extractor compares relu1_2 / relu2_2 / relu3_3 activations
  (L1) plus a pixel L1 term.  No pretrained ImageNet weights are fetchable here: the extractor is
  random-init unless ``load_feature_weights()`` is given a local state dict ("parity unpinned").
* ``mse_loss`` -- nn.MSELoss() of Fairscale-DDP.py:76.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.conv import conv3x3_relu
from ..ops.pool import MaxPool2d

# PDT_PERCEPT_OWN_CONVS=0: every feature conv on torch / MIOpen (A/B).  Default: in bf16 the <= 64-channel convs
# (RGB -> 64, 64 -> 64) run ops.conv's kernels -- the RGB conv's data gradient (64 -> 3 channels) was one 0.78 ms CK
# kernel per micro-step, the implicit-GEMM conv takes it at any output width up to 64 (SwinIR feat 561 -> 574
# samples/s); fp32 stays on MIOpen (im2col + fp32 GEMM measured 4 % slower there)
_OWN_CONVS = os.environ.get("PDT_PERCEPT_OWN_CONVS", "1") == "1"


class _NarrowConvReLU(nn.Conv2d):
    """relu(nn.Conv2d(c, v, 3, padding=1)(x)) (same parameters / state_dict; the ReLU slot after it in ``features``
    is an Identity): in bf16 ops.conv.conv3x3_relu -- the ReLU in the implicit-GEMM conv's store."""

    def forward(self, x):
        dt = torch.get_autocast_dtype("cuda") if (x.is_cuda and torch.is_autocast_enabled("cuda")) else x.dtype
        if x.is_cuda and dt == torch.bfloat16:
            return conv3x3_relu(x, self.weight, self.bias)
        return F.relu(super().forward(x))

_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256]
_TAPS = {3: "relu1_2", 8: "relu2_2", 15: "relu3_3"}


class PerceptualLoss(nn.Module):
    def __init__(self, weights=(1.0, 1.0, 1.0), pixel_weight: float = 1.0, seed: int = 0):
        super().__init__()
        layers, c = [], 3
        for v in _CFG:
            if v == "M":
                # channels-last bf16: ops.pool's kernels (one slot byte per output, gather backward); else torch
                layers.append(MaxPool2d(2) if _OWN_CONVS else nn.MaxPool2d(2))
            else:
                if _OWN_CONVS and c <= 64 and v <= 64:
                    layers += [_NarrowConvReLU(c, v, 3, padding=1), nn.Identity()]
                else:
                    layers += [nn.Conv2d(c, v, 3, padding=1), nn.ReLU(inplace=False)]
                c = v
        self.features = nn.Sequential(*layers)
        g = torch.Generator().manual_seed(seed)
        for m in self.features:
            if isinstance(m, nn.Conv2d):
                with torch.no_grad():
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / (m.in_channels * 9)) ** 0.5)
                    m.bias.zero_()
        for p in self.parameters():
            p.requires_grad_(False)
        self.register_buffer("mean", torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1), persistent=False)
        self.register_buffer("std", torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1), persistent=False)
        self.weights, self.pixel_weight = weights, pixel_weight

    def load_feature_weights(self, sd):
        self.features.load_state_dict(sd, strict=False)

    def _taps(self, x):
        out = []
        x = (x - self.mean.to(x.dtype)) / self.std.to(x.dtype)
        for i, m in enumerate(self.features):
            x = m(x)
            if i in _TAPS:
                out.append(x)
        return out

    def forward(self, outputs, targets):
        self.features.eval()
        targets = targets.detach()
        if outputs.dim() == 4 and targets.shape == outputs.shape and targets.stride() != outputs.stride() and \
                outputs.is_contiguous(memory_format=torch.channels_last):
            # a channels-last model output (the NHWC conv path): run the target branch in the same layout, so the
            # feature maps pair up element for element (fused L1) and both branches take the same conv kernels
            targets = targets.contiguous(memory_format=torch.channels_last)
        fo, ft = self._taps(outputs), self._taps(targets)
        # fused L1 (ops.l1): mean |a - b| and its gradient in one read, in the maps' own dtype (autocast would run
        # F.l1_loss as fp32 copies + four elementwise passes over each 18 x 64 x 256 x 256 map)
        loss = self.pixel_weight * _l1(outputs, targets.detach())
        for w, a, b in zip(self.weights, fo, ft):
            loss = loss + w * _l1(a, b)
        return loss


def _l1(a, b):
    if a.is_cuda:
        from ..ops.l1 import l1_loss
        b = b.to(a.dtype) if b.dtype != a.dtype else b
        if b.stride() != a.stride():
            cl = a.dim() == 4 and a.is_contiguous(memory_format=torch.channels_last)
            b = b.contiguous(memory_format=torch.channels_last) if cl else b.contiguous()
        return l1_loss(a, b)
    return F.l1_loss(a, b)


_feat = None


def feat_loss(outputs, targets):
    """Module-level perceptual loss callable, as imported by the reference (``from PyTorchPercept import feat_loss``)."""
    global _feat
    if _feat is None or next(_feat.buffers()).device != outputs.device:
        _feat = PerceptualLoss().to(outputs.device)
    return _feat(outputs, targets)


mse_loss = nn.MSELoss()
