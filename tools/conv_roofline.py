#!/usr/bin/env python3
"""Per-layer roofline of the ResNet-50 convolutions (NHWC bf16) on one MI355X.

For every distinct conv of ResNet-50 v1.5 at a given batch, times forward, backward-data and
backward-weight (MIOpen via torch, ``cudnn.benchmark`` on) and, for 1x1 stride-1 convs, the same
three GEMMs through ``torch.matmul`` (hipBLASLt). Prints one JSON line per layer with achieved
TFLOP/s and the effective bandwidth over the minimum bytes (inputs read once, output written
once), weighted by how often the layer occurs in the network, so the table says which layers
are compute- or memory-bound and where the step's conv time goes.

    python tools/conv_roofline.py --batch 128 > gpurun_out/conv_roofline.jsonl
"""
from __future__ import annotations

import argparse
import json
import sys
from collections import Counter

import torch
import torch.nn.functional as F


def resnet50_convs(batch: int):
    """(n, h, w, cin, cout, k, stride) -> occurrences, in network order."""
    convs = Counter()
    order = []

    def add(key):
        if key not in convs:
            order.append(key)
        convs[key] += 1

    add((batch, 224, 224, 3, 64, 7, 2))
    h = 56
    cin = 64
    for i, nblk in enumerate([3, 4, 6, 3]):
        mid = 64 * 2 ** i
        for j in range(nblk):
            stride = 2 if (j == 0 and i > 0) else 1
            add((batch, h, h, cin, mid, 1, 1))
            add((batch, h, h, mid, mid, 3, stride))
            ho = h // stride
            add((batch, ho, ho, mid, mid * 4, 1, 1))
            if j == 0:
                add((batch, h, h, cin, mid * 4, 1, stride))
            cin = mid * 4
            h = ho
    return [(k, convs[k]) for k in order]


def timeit(fn, reps):
    """Median GPU time (us) of fn(): ``reps`` graph replays of 4 captured calls each (no host
    launch cost, which a library like MIOpen would otherwise add to every eager call)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(4):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / 4)
    ts.sort()
    del g
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--matmul", type=int, default=1)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    tot = Counter()
    for (n, h, w, cin, cout, k, st), cnt in resnet50_convs(args.batch):
        pad = k // 2
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last) * 0.05
        y = F.conv2d(x, wt, stride=st, padding=pad)
        dy = torch.randn_like(y)
        ho, wo = y.shape[2], y.shape[3]
        flop = 2.0 * n * ho * wo * cout * cin * k * k
        bx, bw, by = x.numel() * 2, wt.numel() * 2, y.numel() * 2
        res = {"layer": f"{k}x{k}/{st} {cin}->{cout} @{h}x{w}", "count": cnt,
               "gflop": round(flop / 1e9, 2)}
        ops = {
            "fwd": (lambda: F.conv2d(x, wt, stride=st, padding=pad), bx + bw + by),
            "bwd_data": (lambda: torch.ops.aten.convolution_backward(
                dy, x, wt, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                [True, False, False]), by + bw + bx),
            "bwd_weight": (lambda: torch.ops.aten.convolution_backward(
                dy, x, wt, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                [False, True, False]), by + bx + bw),
        }
        if args.matmul and k == 1 and st == 1:
            a = x.permute(0, 2, 3, 1).reshape(-1, cin)          # view (NHWC)
            w2 = wt.reshape(cout, cin)
            g = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            ops["mm_fwd"] = (lambda: a @ w2.t(), bx + bw + by)
            ops["mm_bwd_data"] = (lambda: g @ w2, by + bw + bx)
            ops["mm_bwd_weight"] = (lambda: g.t() @ a, by + bx + bw)
        for name, (fn, nbytes) in ops.items():
            us = timeit(fn, args.reps)
            res[name + "_us"] = round(us, 1)
            res[name + "_tflops"] = round(flop / us / 1e6, 1)
            res[name + "_tbps"] = round(nbytes / us / 1e6, 2)
            tot[name] += us * cnt
        print(json.dumps(res), flush=True)
        del x, wt, y, dy
    print(json.dumps({"total_us_per_step": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
