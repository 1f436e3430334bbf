"""CIFAR-style ResNets with the reference's state_dict layout (src/models/resnet.py:122,130).

Only the parameter/buffer layout matters to the aggregation path; tests check it against the
reference's own layouts (tests/golden/layouts.json).
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F


def _conv_bn(cin: int, cout: int, k: int, stride: int):
    pad = k // 2
    return nn.Conv2d(cin, cout, kernel_size=k, stride=stride, padding=pad, bias=False), nn.BatchNorm2d(cout)


class _Shortcut(nn.Sequential):
    def __init__(self, cin: int, cout: int, stride: int):
        if stride == 1 and cin == cout:
            super().__init__()
        else:
            conv, bn = _conv_bn(cin, cout, 1, stride)
            super().__init__(conv, bn)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes: int, planes: int, stride: int = 1):
        super().__init__()
        self.conv1, self.bn1 = _conv_bn(in_planes, planes, 3, stride)
        self.conv2, self.bn2 = _conv_bn(planes, planes, 3, 1)
        self.shortcut = _Shortcut(in_planes, planes, stride)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + self.shortcut(x))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_planes: int, planes: int, stride: int = 1):
        super().__init__()
        self.conv1, self.bn1 = _conv_bn(in_planes, planes, 1, 1)
        self.conv2, self.bn2 = _conv_bn(planes, planes, 3, stride)
        self.conv3, self.bn3 = _conv_bn(planes, planes * 4, 1, 1)
        self.shortcut = _Shortcut(in_planes, planes * 4, stride)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return F.relu(y + self.shortcut(x))


class ResNet(nn.Module):
    def __init__(self, block, num_blocks, num_classes: int = 10):
        super().__init__()
        self.conv1, self.bn1 = _conv_bn(3, 64, 3, 1)
        width = 64
        stages = []
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), num_blocks)):
            layers = []
            for j in range(n):
                stride = 2 if (i > 0 and j == 0) else 1
                layers.append(block(width, planes, stride))
                width = planes * block.expansion
            stages.append(nn.Sequential(*layers))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.linear = nn.Linear(512 * block.expansion, num_classes)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.layer4(self.layer3(self.layer2(self.layer1(y))))
        y = F.avg_pool2d(y, 4).flatten(1)
        return self.linear(y)


def ResNet18():
    return ResNet(BasicBlock, [2, 2, 2, 2])


def ResNet50():
    return ResNet(Bottleneck, [3, 4, 6, 3])
