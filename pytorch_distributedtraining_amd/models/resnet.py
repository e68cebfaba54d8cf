"""ResNet-18/34/50/101/152 (BASELINE.json configs 1-2: ResNet-18 DDP gloo plumbing, ResNet-50 DDP bf16).

Parameter / buffer names match torchvision's ResNet (conv1, bn1, layer{1-4}.{i}.conv{1,2,3}, bn*,
downsample.{0,1}, fc) so torchvision checkpoints load with ``strict=True``.  Convolutions run on
MIOpen (framework layer); use ``channels_last`` + bf16 autocast on MI355X.  With ``fused_bn=True`` (default)
every BatchNorm is an ``ops.batchnorm.BatchNormAct2d`` (an nn.BatchNorm2d subclass) that fuses the
following ReLU and, at the end of a block, the residual add into one channels-last HIP pass
(``relu(bn3(conv3(h)) + identity)``), and the stem's max pool keeps a 1-byte window slot instead of an int64
argmax (``ops.pool``); ``fused_bn=False`` builds the plain nn.BatchNorm2d / nn.ReLU model
(the stock-torch baseline).  ``parallel.syncbn.convert_sync_batchnorm`` makes either cross-rank.
Written from the published architecture (He et al. 2015), random init.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops.batchnorm import BatchNormAct2d
from ..ops.conv import Conv2d1x1
from ..ops.pool import MaxPool2d


def _bn(c, act, fused):
    return BatchNormAct2d(c, act=act) if fused else nn.BatchNorm2d(c)


def conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin, cout, stride=1, fused=False):
    """Stride-1 1x1 convs of the fused model go through ops.conv.Conv2d1x1 (MIOpen or GEMM per shape and
    direction, measured); same parameters / state_dict as nn.Conv2d."""
    if fused and stride == 1:
        return Conv2d1x1(cin, cout)
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


# the downsample blocks fork x too (PDT_RESNET_FORK_DS=1: their downsample conv's data gradient joins conv1's dgrad
# GEMM as its C operand) -- measured 0.6-1 % SLOWER than autograd's separate add over those 4 block inputs
# (9,217 / 9,169 vs 9,252 / 9,276 samples/s, profiles/r5/r5_resnet_fork_ds_ab.txt), so off by default
FORK_DOWNSAMPLE = os.environ.get("PDT_RESNET_FORK_DS", "0") == "1"


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None, fused=True):
        super().__init__()
        self.fused = fused
        self.conv1 = conv3x3(cin, planes, stride)
        self.bn1 = _bn(planes, "relu", fused)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = _bn(planes, "relu", fused)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        if self.fused:
            return self.bn2(self.conv2(self.bn1(self.conv1(x))), residual=idt)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None, fused=True):
        super().__init__()
        self.fused = fused
        self.conv1 = conv1x1(cin, planes, fused=fused)
        self.bn1 = _bn(planes, "relu", fused)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = _bn(planes, "relu", fused)
        self.conv3 = conv1x1(planes, planes * 4, fused=fused)
        self.bn3 = _bn(planes * 4, "relu", fused)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        if self.fused and hasattr(self.conv1, "forward_fork") and (self.downsample is None or FORK_DOWNSAMPLE):
            # conv1 and the identity (or the downsample branch) share x: their two input gradients are summed
            # inside conv1's dgrad GEMM instead of by a separate add over the block input's gradient
            h, xa = self.conv1.forward_fork(x)
            idt = xa if self.downsample is None else self.downsample(xa)
            return self.bn3(self.conv3(self.bn2(self.conv2(self.bn1(h)))), residual=idt)
        idt = x if self.downsample is None else self.downsample(x)
        if self.fused:
            out = self.bn2(self.conv2(self.bn1(self.conv1(x))))
            return self.bn3(self.conv3(out), residual=idt)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, zero_init_residual=True, fused_bn=True):
        super().__init__()
        self.fused = fused_bn
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(64, "relu", fused_bn)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool2d(3, stride=2, padding=1) if fused_bn else nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make(self, block, planes, n, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride, fused=self.fused),
                                 _bn(planes * block.expansion, None, self.fused))
        layers = [block(self.inplanes, planes, stride, down, fused=self.fused)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, fused=self.fused) for _ in range(1, n)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.bn1(self.conv1(x))
        x = self.maxpool(x if self.fused else self.relu(x))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
