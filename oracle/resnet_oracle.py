"""ORACLE / TEST INFRASTRUCTURE ONLY — never imported by the product path.

CPU restatement of the torchvision ResNet-50/101 body that the reference's
`Backbone` instantiates (`src/trackformer/models/backbone.py:102-104`,
`getattr(torchvision.models, name)(replace_stride_with_dilation=..., norm_layer=FrozenBatchNorm2d)`).

torchvision is a third-party dependency absent from this image and from
/root/reference (docs/INSTALL.md:12 names "torchvision 0.6"; requirements.txt pins
nothing).  This file restates its published ResNet v1.5 definition:
  * stem: 7x7/2 conv (pad 3, no bias) -> norm -> ReLU -> 3x3/2 max-pool (pad 1)
  * Bottleneck(expansion 4): 1x1 -> norm -> ReLU -> 3x3 (stride here, v1.5) -> norm -> ReLU
    -> 1x1 -> norm, + identity / downsample(1x1 stride conv + norm), ReLU
  * layers [3,4,6,3] (R-50) / [3,4,23,3] (R-101), widths 64/128/256/512.
Module attribute names match torchvision so state_dict keys equal the reference's
(`backbone.0.body.layer1.0.conv1.weight`, ...).  Backbone parity vs torchvision
itself is therefore UNPINNED (no torchvision to compare against); conv arithmetic
is torch.nn.functional on CPU.

`FrozenBatchNorm2d` restates backbone.py:22-58 (eps 1e-5 inside the rsqrt).
`IntermediateLayerGetter` restates torchvision.models._utils semantics (run the
children in order, collect the named ones, stop after the last requested).
"""
from collections import OrderedDict

import torch
from torch import nn


class FrozenBatchNorm2d(nn.Module):
    """backbone.py:22-58: y = x * (w * rsqrt(rv + 1e-5)) + (b - rm * scale)."""

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict,
                              missing_keys, unexpected_keys, error_msgs):
        state_dict.pop(prefix + 'num_batches_tracked', None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict,
                                      missing_keys, unexpected_keys, error_msgs)

    def forward(self, x):
        w = self.weight.reshape(1, -1, 1, 1)
        b = self.bias.reshape(1, -1, 1, 1)
        rv = self.running_var.reshape(1, -1, 1, 1)
        rm = self.running_mean.reshape(1, -1, 1, 1)
        scale = w * (rv + 1e-5).rsqrt()
        bias = b - rm * scale
        return x * scale + bias


def _conv3x3(cin, cout, stride=1, dilation=1):
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=dilation, dilation=dilation, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, dilation=1, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.conv1 = _conv1x1(inplanes, planes)
        self.bn1 = norm_layer(planes)
        self.conv2 = _conv3x3(planes, planes, stride, dilation)
        self.bn2 = norm_layer(planes)
        self.conv3 = _conv1x1(planes, planes * 4)
        self.bn3 = norm_layer(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)


class ResNet(nn.Module):
    def __init__(self, layers, replace_stride_with_dilation=None, norm_layer=None):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self._norm_layer = norm_layer
        self.inplanes = 64
        self.dilation = 1
        if replace_stride_with_dilation is None:
            replace_stride_with_dilation = [False, False, False]
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], 2, replace_stride_with_dilation[0])
        self.layer3 = self._make_layer(256, layers[2], 2, replace_stride_with_dilation[1])
        self.layer4 = self._make_layer(512, layers[3], 2, replace_stride_with_dilation[2])
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, 1000)

    def _make_layer(self, planes, blocks, stride=1, dilate=False):
        norm_layer = self._norm_layer
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(_conv1x1(self.inplanes, planes * 4, stride), norm_layer(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample, previous_dilation, norm_layer)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes, dilation=self.dilation, norm_layer=norm_layer))
        return nn.Sequential(*layers)


def resnet50(pretrained=False, **kw):
    # pretrained weights are a remote fetch (backbone.py:104) -- unavailable offline; ignored.
    return ResNet([3, 4, 6, 3], **kw)


def resnet101(pretrained=False, **kw):
    return ResNet([3, 4, 23, 3], **kw)


class IntermediateLayerGetter(nn.ModuleDict):
    """torchvision.models._utils.IntermediateLayerGetter semantics."""

    def __init__(self, model, return_layers):
        wanted = dict(return_layers)
        layers = OrderedDict()
        remaining = set(wanted)
        for name, module in model.named_children():
            layers[name] = module
            remaining.discard(name)
            if not remaining:
                break
        super().__init__(layers)
        self.return_layers = wanted

    def forward(self, x):
        out = OrderedDict()
        for name, module in self.items():
            x = module(x)
            if name in self.return_layers:
                out[self.return_layers[name]] = x
        return out
