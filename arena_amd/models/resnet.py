"""ResNet v1.5 (bottleneck) in plain ``torch.nn`` -- the Horovod image's benchmark model family.

The reference's allreduce demo runs the Horovod TF image's ``hvd-distribute.sh``
(charts/tf-horovod/README.md:66-69, SURVEY §2.11 "Horovod TF image"). That image's benchmark is
the tf_cnn_benchmarks ResNet family on synthetic ImageNet-shaped data. The script is not in the
reference repo, so the exact model flags are unpinned. The architecture here is the standard
one: a 7x7 stem, 4 stages of bottleneck blocks with the stride on the 3x3 conv (v1.5), global
average pooling, and a 1000-way FC. ``width``/``depth`` knobs give tiny variants for CPU tests.

MI355X layout: the model is meant to run with ``memory_format=torch.channels_last`` under bf16
autocast, so the MIOpen convolutions take their NHWC MFMA paths. Parameters stay fp32 (master
weights) for the data-parallel buckets and the optimizer.
"""
from __future__ import annotations

from typing import List

import torch
from torch import nn

DEPTHS = {"resnet50": [3, 4, 6, 3], "resnet101": [3, 4, 23, 3],
          "resnet152": [3, 8, 36, 3], "resnet_tiny": [1, 1, 1, 1]}


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, mid: int, stride: int):
        super().__init__()
        cout = mid * self.expansion
        self.conv1 = nn.Conv2d(cin, mid, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(mid)
        self.conv2 = nn.Conv2d(mid, mid, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(mid)
        self.conv3 = nn.Conv2d(mid, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        nn.init.zeros_(self.bn3.weight)  # zero-init the residual branch's last BN (goyal et al.)
        self.relu = nn.ReLU(inplace=True)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False),
                                      nn.BatchNorm2d(cout))

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


class ResNet(nn.Module):
    def __init__(self, depths: List[int], num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False),
                                  nn.BatchNorm2d(width), nn.ReLU(inplace=True),
                                  nn.MaxPool2d(3, stride=2, padding=1))
        layers = []
        cin = width
        for i, n in enumerate(depths):
            mid = width * (2 ** i)
            for j in range(n):
                layers.append(Bottleneck(cin, mid, stride=2 if (j == 0 and i > 0) else 1))
                cin = mid * Bottleneck.expansion
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(x, 1), 1))


def resnet(name: str = "resnet50", num_classes: int = 1000, width: int = 64) -> ResNet:
    depths = DEPTHS.get(name)
    if depths is None:
        raise ValueError(f"unknown model {name!r}; choose one of "
                         f"{sorted(DEPTHS)}")
    return ResNet(depths, num_classes=num_classes, width=width)
