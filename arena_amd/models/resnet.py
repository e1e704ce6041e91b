"""ResNet v1.5 (bottleneck) in plain ``torch.nn`` -- the Horovod image's benchmark model family.

The reference's allreduce demo runs the Horovod TF image's ``hvd-distribute.sh``
(charts/tf-horovod/README.md:66-69, SURVEY §2.11 "Horovod TF image"). That image's benchmark is
the tf_cnn_benchmarks ResNet family on synthetic ImageNet-shaped data. The script is not in the
reference repo, so the exact model flags are unpinned. The architecture here is the standard
one: a 7x7 stem, 4 stages of bottleneck blocks with the stride on the 3x3 conv (v1.5), global
average pooling, and a 1000-way FC. ``width``/``depth`` knobs give tiny variants for CPU tests.

MI355X layout: the model is meant to run with ``memory_format=torch.channels_last`` under bf16
autocast. Every convolution runs on the hand-written MFMA implicit-GEMM kernels
(``csrc/ops/conv_kernels.hip``, tile autotuned per shape and direction): ``Conv2dNHWC`` for the
bottleneck convs (stride-2 backward-data as phase convolutions), ``StemConv2d`` for the 7x7/2 stem
in space-to-depth form. Each BatchNorm, with its ReLU and residual add, is one fused HIP kernel
pair per direction (``arena_amd.ops.batchnorm``); its forward statistics come from the producing
conv's epilogue.
Parameters stay fp32 (master weights) for the data-parallel buckets and the optimizer.
"""
from __future__ import annotations

import os
from typing import List

import torch
from torch import nn

from ..ops.batchnorm import BatchNormAct2d, ResidualMask, bn_relu_maxpool
from ..ops.conv import BNGradLink, Conv2dNHWC, GradJoin, StemConv2d, WeightFlipper
from ..ops.pool import MaxPool2dNHWC, global_avg_pool

# Downsample blocks build their shortcut after the main path (see Bottleneck.forward; A/B switch,
# ARENA_DOWN_LAST=0 builds it first).
_DOWN_LAST = os.environ.get("ARENA_DOWN_LAST", "1") == "1"


def set_downsample_last(on: bool) -> None:
    global _DOWN_LAST
    _DOWN_LAST = bool(on)


DEPTHS = {"resnet50": [3, 4, 6, 3], "resnet101": [3, 4, 23, 3],
          "resnet152": [3, 8, 36, 3], "resnet_tiny": [1, 1, 1, 1]}


class Bottleneck(nn.Module):
    """conv1x1-BN-ReLU, conv3x3(stride)-BN-ReLU, conv1x1-BN, + shortcut, ReLU. Every BN is a
    ``BatchNormAct2d``, so the last one also takes the residual add and the final ReLU
    (one fused kernel pair instead of BN + add + ReLU)."""
    expansion = 4

    def __init__(self, cin: int, mid: int, stride: int):
        super().__init__()
        cout = mid * self.expansion
        self.conv1 = Conv2dNHWC(cin, mid, 1, bias=False)
        self.bn1 = BatchNormAct2d(mid, act="relu")
        self.conv2 = Conv2dNHWC(mid, mid, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormAct2d(mid, act="relu")
        self.conv3 = Conv2dNHWC(mid, cout, 1, bias=False)
        self.bn3 = BatchNormAct2d(cout, act="relu")
        nn.init.zeros_(self.bn3.weight)  # zero-init the residual branch's last BN (goyal et al.)
        self.down_conv = self.down_bn = None
        if stride != 1 or cin != cout:
            self.down_conv = Conv2dNHWC(cin, cout, 1, stride=stride, bias=False)
            self.down_bn = BatchNormAct2d(cout, act="none")

    def forward(self, x, link: BNGradLink | None = None, link_out: BNGradLink | None = None):
        """``link``: x is the output of the previous block's last BN, which filled this link;
        ``link_out``: handed to this block's last BN for the next block."""
        # forward_stats: when a conv runs on the MFMA kernel, its epilogue also produces the
        # BatchNorm statistics partials of its output, and the BN skips its statistics pass.
        # join: x feeds conv1 and the shortcut; its two gradients are summed inside the second
        # backward (conv1's backward-data epilogue) instead of by a separate add pass.
        # links: each BN's output feeds a conv whose backward-data epilogue computes that BN's
        # backward partial sums (the BN skips its reduction pass); for the block input, the conv
        # that completes the join does it.
        train = torch.is_grad_enabled() and x.requires_grad
        join = GradJoin() if train else None
        lk1, lk2 = (BNGradLink(), BNGradLink()) if train else (None, None)
        idt = x
        # downsample block: bn3's residual gradient reaches down_bn as (dy, bn3's ReLU mask)
        rmask = ResidualMask() if (train and self.down_conv is not None) else None

        def shortcut():
            y_, st_ = self.down_conv.forward_stats(x, join=join, bn_link=link)
            return self.down_bn(y_, stats=st_, res_in=rmask)

        if self.down_conv is not None and not _DOWN_LAST:
            idt = shortcut()
        y, st = self.conv1.forward_stats(x, join=join, bn_link=link)
        a = self.bn1(y, stats=st, link=lk1)
        y, st = self.conv2.forward_stats(a, bn_link=lk1)
        a = self.bn2(y, stats=st, link=lk2)
        y, st = self.conv3.forward_stats(a, bn_link=lk2)
        if self.down_conv is not None and _DOWN_LAST:
            # created after the main path, the shortcut's backward runs first (autograd takes
            # the ready node with the highest sequence number): its strided dgrad parks at the
            # join and conv1's stride-1 dgrad completes it -- so conv1's epilogue can take the
            # previous BN's backward sums (BNGradLink), which a strided dgrad cannot
            idt = shortcut()
        return self.bn3(y, residual=idt, stats=st, join=join if self.down_conv is None else None,
                        link=link_out, res_out=rmask)


class ResNet(nn.Module):
    def __init__(self, depths: List[int], num_classes: int = 1000, width: int = 64):
        super().__init__()
        self.stem = nn.Sequential(StemConv2d(3, width, 7, stride=2, padding=3, bias=False),
                                  BatchNormAct2d(width, act="relu"),
                                  MaxPool2dNHWC(3, stride=2, padding=1))
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
        # every stride-1 conv weight flipped for its backward-data pass in one launch per step
        self._flipper = WeightFlipper(list(self.layers.modules()))

    def forward(self, x):
        with self._flipper.scope():
            y, st = self.stem[0].forward_stats(x)    # epilogue BN statistics, as in the blocks
            # BN + ReLU + max pool as one pass each way when the statistics come summed
            x = bn_relu_maxpool(self.stem[1], self.stem[2], y, st)
            link = None
            for blk in self.layers:
                out_link = BNGradLink() if torch.is_grad_enabled() else None
                x = blk(x, link=link, link_out=out_link)
                link = out_link
        return self.fc(global_avg_pool(x))


def resnet(name: str = "resnet50", num_classes: int = 1000, width: int = 64) -> ResNet:
    depths = DEPTHS.get(name)
    if depths is None:
        raise ValueError(f"unknown model {name!r}; choose one of "
                         f"{sorted(DEPTHS)}")
    return ResNet(depths, num_classes=num_classes, width=width)
