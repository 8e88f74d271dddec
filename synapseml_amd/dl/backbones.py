"""Vision backbones for DeepVisionClassifier (reference: deep-learning/.../dl/
LitDeepVisionModel.py, which pulls torchvision's pretrained zoo).

torchvision is not part of this stack and nothing can be downloaded, so the
ResNet family (ResNet-18/34/50/101/152, ResNeXt-50 32x4d, Wide-ResNet-50-2)
is defined here, random-initialised, or loaded from a local state dict /
safetensors file (``weights=path``). Layout is channels_last-friendly: every
conv is followed by BN+ReLU so MIOpen's fused NHWC kernels apply.
``head_and_trainable`` reproduces the reference's fine-tuning policy: freeze
the backbone, replace the classifier, and unfreeze the last
``additional_layers_to_train`` (0-3) stages."""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, c, stride=1, down=None, groups=1, width=64):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(c)
        self.conv2 = nn.Conv2d(c, c, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(c)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, c, stride=1, down=None, groups=1, width=64):
        super().__init__()
        w = int(c * (width / 64.0)) * groups
        self.conv1 = nn.Conv2d(cin, w, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(w)
        self.conv2 = nn.Conv2d(w, w, 3, stride, 1, groups=groups, bias=False)
        self.bn2 = nn.BatchNorm2d(w)
        self.conv3 = nn.Conv2d(w, c * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(c * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, block, layers: List[int], num_classes: int = 1000, groups: int = 1, width: int = 64,
                 base: int = 64):
        super().__init__()
        self.cin = base
        self.groups, self.width = groups, width
        self.conv1 = nn.Conv2d(3, base, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(base)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, base, layers[0], 1)
        self.layer2 = self._make(block, base * 2, layers[1], 2)
        self.layer3 = self._make(block, base * 4, layers[2], 2)
        self.layer4 = self._make(block, base * 8, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(base * 8 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make(self, block, c, n, stride):
        down = None
        if stride != 1 or self.cin != c * block.expansion:
            down = nn.Sequential(nn.Conv2d(self.cin, c * block.expansion, 1, stride, bias=False),
                                 nn.BatchNorm2d(c * block.expansion))
        layers = [block(self.cin, c, stride, down, self.groups, self.width)]
        self.cin = c * block.expansion
        layers += [block(self.cin, c, 1, None, self.groups, self.width) for _ in range(1, n)]
        return nn.Sequential(*layers)

    def features(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(self.avgpool(x), 1)

    def forward(self, x):
        return self.fc(self.features(x))


_ZOO = {
    "resnet18": (BasicBlock, [2, 2, 2, 2], {}),
    "resnet34": (BasicBlock, [3, 4, 6, 3], {}),
    "resnet50": (Bottleneck, [3, 4, 6, 3], {}),
    "resnet101": (Bottleneck, [3, 4, 23, 3], {}),
    "resnet152": (Bottleneck, [3, 8, 36, 3], {}),
    "resnext50_32x4d": (Bottleneck, [3, 4, 6, 3], {"groups": 32, "width": 4}),
    "resnext101_32x8d": (Bottleneck, [3, 4, 23, 3], {"groups": 32, "width": 8}),
    "wide_resnet50_2": (Bottleneck, [3, 4, 6, 3], {"width": 128}),
    # small variant for tests / CPU smoke runs
    "resnet_tiny": (BasicBlock, [1, 1, 1, 1], {"base": 8}),
}


def available() -> List[str]:
    return sorted(_ZOO)


def build(name: str, num_classes: int = 1000, weights: Optional[str] = None) -> ResNet:
    if name not in _ZOO:
        raise ValueError(f"No model: {name} found (available: {', '.join(available())})")
    block, layers, kw = _ZOO[name]
    m = ResNet(block, layers, 1000, **kw)
    if weights:
        if weights.endswith(".safetensors"):
            from safetensors.torch import load_file

            sd = load_file(weights)
        else:
            sd = torch.load(weights, map_location="cpu", weights_only=True)
        m.load_state_dict(sd, strict=False)
    m.fc = nn.Linear(m.fc.in_features, num_classes)
    return m


def head_and_trainable(model: ResNet, additional_layers_to_train: int) -> None:
    if not 0 <= additional_layers_to_train <= 3:
        raise ValueError(f"additional_layers_to_train has to between 0 and 3: {additional_layers_to_train} found")
    for p in model.parameters():
        p.requires_grad = False
    for p in model.fc.parameters():
        p.requires_grad = True
    for stage in [model.layer4, model.layer3, model.layer2][:additional_layers_to_train]:
        for p in stage.parameters():
            p.requires_grad = True


__all__ = ["ResNet", "build", "available", "head_and_trainable"]
