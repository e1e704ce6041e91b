#!/usr/bin/env python3
"""Timing of the MIOpen-free paths that replace MIOpen in the ResNet-50 step: stride-2 backward
data (phase decomposition into stride-1 convs) and the space-to-depth 7x7/2 stem (forward +
weight gradient), each against MIOpen at the same shapes. One JSON line per layer.

    python tools/conv_s2_bench.py --batch 128 > gpurun_out/conv_s2.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import _ext, conv  # noqa: E402
from tools.conv_roofline import resnet50_convs, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    ext = _ext.load()
    tot = {"miopen": 0.0, "ours": 0.0}
    for (n, h, w, cin, cout, k, st), cnt in resnet50_convs(args.batch):
        if st != 2 or cin % 64:
            continue
        pad = k // 2
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wb = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, wb, stride=st, padding=pad)
        dy = torch.randn_like(y)
        res = {"layer": f"dgrad {k}x{k}/{st} {cin}->{cout} @{h}x{w}", "count": cnt}
        t_mi = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, wb, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
            [True, False, False]), args.reps)
        res["miopen_us"] = round(t_mi, 1)
        best = None
        for v in conv.variants_for(cin):
            t = timeit(lambda: conv.conv2d_bwd_data_strided(dy, wb, (h, w), st, pad, v),
                       args.reps)
            res[f"ours_v{v}_us"] = round(t, 1)
            best = t if best is None else min(best, t)
        res["speedup"] = round(t_mi / best, 3)
        tot["miopen"] += t_mi * cnt
        tot["ours"] += best * cnt
        print(json.dumps(res), flush=True)
    # ---- stem ----
    n = args.batch
    x = torch.randn(n, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    m = conv.StemConv2d(3, 64, 7, stride=2, padding=3, bias=False).to(dev).to(
        memory_format=torch.channels_last)
    wb = m.weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = {"layer": "stem 7x7/2 3->64 @224x224", "count": 1}
    res["miopen_fwd_us"] = round(timeit(lambda: F.conv2d(x, wb, stride=2, padding=3), args.reps), 1)
    z = ext.s2d_stem(x)
    w16 = conv.stem_weight(wb)
    res["ours_s2d_us"] = round(timeit(lambda: ext.s2d_stem(x), args.reps), 1)
    res["ours_weight_prep_us"] = round(timeit(lambda: conv.stem_weight(wb), args.reps), 1)
    for v in [v for v in conv.variants_for(64) if conv.TILES[v][1] == 64]:
        res[f"ours_fwd_v{v}_us"] = round(timeit(lambda: ext.conv_fwd_ex(
            z, w16, 1, 2, 2, 112, 112, v, True, None, None, [], True), args.reps), 1)
    y = F.conv2d(x, wb, stride=2, padding=3)
    dy = torch.randn_like(y)
    res["miopen_wgrad_us"] = round(timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False]),
        args.reps), 1)
    for v in (3, 7):
        for sp in (0, 64, 128, 256):
            res[f"ours_wgrad_v{v}_s{sp}_us"] = round(timeit(lambda: ext.conv_wgrad_ex(
                z, dy, 4, 4, 1, 2, 2, v, sp, False, 1.0, True), args.reps), 1)
    print(json.dumps(res), flush=True)
    print(json.dumps({"dgrad_s2_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
