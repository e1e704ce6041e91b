#!/usr/bin/env python3
"""Fused-BN kernel sweep on the ResNet-50 (batch 128, bf16, NHWC) layer shapes.

Times the training forward (stats + finalize + apply) and backward (reduce + finalize + dx) of
every distinct (M, C) BN shape of ResNet-50, for several reduction geometries (max partial blocks,
minimum row rounds per thread; csrc/ops/bn_kernels.hip::reduce_blocks), and prints one JSON line
per geometry with per-shape microseconds, the total weighted by how often ResNet-50 uses each
shape, and the effective HBM bandwidth of the whole set.

    python tools/bn_bench.py --geoms 512:8,1024:8,2048:8,2048:4
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (rows M at batch 128, channels C, uses per step, relu, residual)
SHAPES = [
    (128 * 112 * 112, 64, 1, True, False),    # stem
    (128 * 56 * 56, 64, 6, True, False),      # layer1 conv1/conv2
    (128 * 56 * 56, 256, 4, False, False),    # layer1 conv3 (1 with residual below) + downsample
    (128 * 56 * 56, 128, 1, True, False),     # layer2 block0 conv1 at input resolution
    (128 * 28 * 28, 128, 7, True, False),
    (128 * 28 * 28, 512, 5, True, True),
    (128 * 28 * 28, 256, 1, True, False),     # layer3 block0 conv1
    (128 * 14 * 14, 256, 11, True, False),
    (128 * 14 * 14, 1024, 7, True, True),
    (128 * 14 * 14, 512, 1, True, False),     # layer4 block0 conv1
    (128 * 7 * 7, 512, 5, True, False),
    (128 * 7 * 7, 2048, 4, True, True),
]


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--geoms", default="512:8,1024:8,2048:8,1024:4,2048:4")
    args = ap.parse_args()
    from arena_amd.ops import _ext
    ext = _ext.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    data = []
    for M, C, uses, relu, res in SHAPES:
        def t4():
            return torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16).view(
                M, 1, 1, C).permute(0, 3, 1, 2)  # NCHW view of NHWC memory: channels_last
        x, dy = t4(), t4()
        r = t4() if res else None
        w = torch.rand(C, device=dev, generator=g) + 0.5
        bias = torch.randn(C, device=dev, generator=g)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        data.append((M, C, uses, relu, res, x, dy, r, w, bias, rm, rv))
    for spec in args.geoms.split(","):
        mb, mr = (int(v) for v in spec.split(":"))
        ext.bn_set_reduce_geometry(mb, mr)
        rows, tot_us, tot_bytes = [], 0.0, 0.0
        for M, C, uses, relu, res, x, dy, r, w, bias, rm, rv in data:
            y, mean, invstd, mask, _ = ext.bn_fwd(x, r, w, bias, rm, rv, True, 0.1, 1e-5, relu, None,
                                               None, 0)
            f = timed(lambda: ext.bn_fwd(x, r, w, bias, rm, rv, True, 0.1, 1e-5, relu, None, None, 0))
            bk = timed(lambda: ext.bn_bwd(dy, mask if relu else None, x, mean, invstd, w, relu, res, True))
            e = M * C * 2
            # fwd: read x twice (+ res), write y; bwd: read dy, x (+ y) twice, write dx (+ dres)
            nbytes = e * ((3 + res) + (2 * (2 + relu) + 1 + res))
            rows.append({"M": M, "C": C, "fwd_us": round(f, 1), "bwd_us": round(bk, 1)})
            tot_us += uses * (f + bk)
            tot_bytes += uses * nbytes
        print(json.dumps({"max_blocks": mb, "min_rounds": mr, "resnet50_bn_us_per_step":
                          round(tot_us, 1), "eff_TBs": round(tot_bytes / tot_us / 1e6, 2),
                          "shapes": rows}), flush=True)
    ext.bn_set_reduce_geometry(512, 8)


if __name__ == "__main__":
    main()
