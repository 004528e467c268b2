"""ResNet family (ResNet-18/34/50/101/152), written for MI355X training.

The reference has no model code of its own: its benchmarks pull ResNet-50 from
``tf.keras.applications`` (``benchmarks/system/benchmark_kungfu.py:96``) or
torchvision (``benchmarks/system/benchmark_kungfu_torch.py:64``).  torchvision is
not installed in this image, so the architecture is defined here (ResNet v1.5:
stride on the 3x3 convolution of each bottleneck, the torchvision layout, 25.56 M
parameters for ResNet-50 — the same count as the reference's gradient table in
``srcs/python/kungfu/tensorflow/v1/benchmarks/model_sizes.py:7-25``).

MI355X-specific choices:
* ``channels_last`` (NHWC) memory format end to end, so MIOpen picks its NHWC
  implicit-GEMM (MFMA) convolution solvers and batch-norm stays contiguous in C.
* Optional fused BN(+residual)+ReLU epilogue from :mod:`kungfu_amd.ops.fused_bn`
  (HIP kernel), selected with ``fused_bn=True``; in training each bottleneck then runs
  as one autograd node on the MFMA convolution kernels (:mod:`kungfu_amd.ops.fused_block`).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Type, Union

import torch
import torch.nn as nn

from ..ops import stem as stem_ops


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _norm_factory(fused: bool) -> Callable[[int, bool], nn.Module]:
    if fused:
        from kungfu_amd.ops.fused_bn import BatchNormAct2d

        return lambda c, relu: BatchNormAct2d(c, relu=relu)

    return lambda c, relu: _BNReLU(c, relu)


class _BNReLU(nn.BatchNorm2d):
    """Plain PyTorch BN(+ReLU) with the same state_dict keys as the fused module."""

    def __init__(self, c: int, relu: bool):
        super().__init__(c)
        self.relu = relu

    def forward(self, x):
        y = super().forward(x)
        return torch.relu_(y) if self.relu else y


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None, norm=None):
        super().__init__()
        self.conv1 = conv3x3(cin, planes, stride)
        self.bn1 = norm(planes, True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm(planes, False)
        self.downsample = downsample
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        return self.relu(out + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None, norm=None,
                 fused_tail: bool = False):
        super().__init__()
        width = planes
        self.conv1 = conv1x1(cin, width)
        self.bn1 = norm(width, True)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = norm(width, True)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.downsample = downsample
        self.fused_tail = fused_tail
        if fused_tail:
            # BN3 + residual add + ReLU in one HIP kernel (forward and backward).
            from kungfu_amd.ops.fused_bn import BatchNormAddAct2d

            self.bn3 = BatchNormAddAct2d(planes * self.expansion)
        else:
            self.bn3 = norm(planes * self.expansion, False)
            self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        if self.fused_tail:
            # training: the whole block as one node on the MFMA conv + fused BN kernels
            # (conv epilogue BN statistics, in-place residual gradient; ops/fused_block.py)
            from kungfu_amd.ops import fused_block

            if fused_block.eligible(self, x):
                return fused_block.bottleneck_forward(self, x)
        idt = x if self.downsample is None else self.downsample(x)
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        out = self.conv3(out)
        if self.fused_tail:
            return self.bn3(out, idt)
        return self.relu(self.bn3(out) + idt)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: List[int],
                 num_classes: int = 1000, fused_bn: bool = False,
                 zero_init_residual: bool = False):
        super().__init__()
        norm = _norm_factory(fused_bn)
        self._norm = norm
        self._fused = fused_bn
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = norm(64, True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d,)):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    w = m.bn3.weight if hasattr(m.bn3, "weight") else m.bn3[0].weight
                    nn.init.zeros_(w)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                conv1x1(self.inplanes, planes * block.expansion, stride),
                self._norm(planes * block.expansion, False),
            )
        kw = {}
        if block is Bottleneck:
            kw["fused_tail"] = self._fused
        layers = [block(self.inplanes, planes, stride, downsample, norm=self._norm, **kw)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, norm=self._norm, **kw))
        return nn.Sequential(*layers)

    def forward(self, x):
        if self._fused and stem_ops.eligible(self.conv1, x):
            # MFMA stem conv with the BN batch statistics in its epilogue (ops/stem.py),
            # then BN+ReLU+MaxPool(3,2,1) in one HIP pass without a statistics pass
            from ..ops.fused_block import _sums
            from ..parallel.mixed import shadow

            sums = _sums(self.bn1, x.device) if self.training else None
            if self.training and stem_ops.block_eligible(x, self.bn1):
                # conv + BN + ReLU + MaxPool as one node: the weight gradient forms dx while staging
                x = stem_ops.stem_block(x, shadow(self.conv1.weight), self.bn1, sums)
            else:
                x = self.bn1.forward_pool(stem_ops.stem_conv(x, shadow(self.conv1.weight), sums), sums=sums)
        elif self._fused:
            x = self.bn1.forward_pool(self.conv1(x))  # BN+ReLU+MaxPool(3,2,1) in one HIP pass
        else:
            x = self.maxpool(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self._fused:
            from ..ops.pool import global_avg_pool

            return self.fc(global_avg_pool(x))  # HIP kernels (torch's backward: ~100 us at batch 256)
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


def resnet18(**kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def resnet152(**kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
