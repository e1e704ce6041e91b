#!/usr/bin/env python3
"""Numerics + timing of the MFMA implicit-GEMM conv kernel vs MIOpen on the ResNet-50 layers.

For every ResNet-50 conv with C % 64 == 0 (all but the stem), at the given batch: checks the
kernel against an fp32 F.conv2d of the same bf16 inputs (every tile variant), then times
forward (and, for stride-1 convs, backward-data through the flipped weight) against MIOpen
(torch, cudnn.benchmark). One JSON line per layer; a summary line weighted by layer count.

    python tools/conv_bench.py --batch 128 > gpurun_out/conv_bench.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from collections import Counter

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import conv  # noqa: E402
from tools.conv_roofline import resnet50_convs, timeit  # noqa: E402


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--check-batch", type=int, default=8, help="batch of the numerics check")
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    tot = Counter()
    bad = 0
    for (n, h, w, cin, cout, k, st), cnt in resnet50_convs(args.batch):
        if cin % 64:
            continue
        pad = k // 2
        g = torch.Generator(device=dev).manual_seed(cin * 7 + cout + k)
        # ---- numerics on a small batch, every variant ----
        xs = torch.randn(args.check_batch, cin, h, w, device=dev, generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device=dev, generator=g) * 0.05).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ref = F.conv2d(xs.float(), wt.float(), stride=st, padding=pad)
        errs = {}
        for v in conv.variants_for(cout):
            y = conv.conv2d_fwd(xs, wt, st, pad, v)
            errs[f"fwd_v{v}"] = rel_err(y, ref)
        if st == 1:
            dys = torch.randn_like(ref).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            dref = torch.ops.aten.convolution_backward(
                dys.float(), xs.float(), wt.float(), None, [1, 1], [pad, pad], [1, 1], False,
                [0, 0], 1, [True, False, False])[0]
            for v in conv.variants_for(cin):
                dx = conv.conv2d_bwd_data(dys, wt, pad, v)
                errs[f"bwd_v{v}"] = rel_err(dx, dref)
        dys = torch.randn_like(ref).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wref = torch.ops.aten.convolution_backward(
            dys.float(), xs.float(), wt.float(), None, [st, st], [pad, pad], [1, 1], False,
            [0, 0], 1, [False, True, False])[1]
        for v in conv.wgrad_variants_for(cin, cout):
            dw = conv.conv2d_wgrad(xs, dys, (k, k), st, pad, v, out_dtype=torch.float32)
            errs[f"wgrad_v{v}"] = rel_err(dw, wref)
        worst = max(errs.values())
        ok = worst < 2e-2
        bad += not ok
        # ---- timing at the full batch ----
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wb = (torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, wb, stride=st, padding=pad)
        m = y.shape[0] * y.shape[2] * y.shape[3]
        flop = 2.0 * m * cout * cin * k * k
        res = {"layer": f"{k}x{k}/{st} {cin}->{cout} @{h}x{w}", "count": cnt, "ok": ok,
               "max_rel_err": round(worst, 5)}
        t_mi = timeit(lambda: F.conv2d(x, wb, stride=st, padding=pad), args.reps)
        res["miopen_fwd_us"] = round(t_mi, 1)
        best = None
        for v in conv.variants_for(cout):
            t = timeit(lambda: conv.conv2d_fwd(x, wb, st, pad, v), args.reps)
            res[f"ours_fwd_v{v}_us"] = round(t, 1)
            best = t if best is None else min(best, t)
        res["ours_fwd_best_tflops"] = round(flop / best / 1e6, 1)
        res["fwd_speedup"] = round(t_mi / best, 3)
        tot["miopen_fwd"] += t_mi * cnt
        tot["ours_fwd"] += min(best, t_mi) * cnt
        if st == 1:
            dy = torch.randn_like(y)
            t_mi = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, x, wb, None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1,
                [True, False, False]), args.reps)
            res["miopen_bwd_data_us"] = round(t_mi, 1)
            best = None
            for v in conv.variants_for(cin):
                t = timeit(lambda: conv.conv2d_bwd_data(dy, wb, pad, v), args.reps)
                res[f"ours_bwd_v{v}_us"] = round(t, 1)
                best = t if best is None else min(best, t)
            res["bwd_data_speedup"] = round(t_mi / best, 3)
            tot["miopen_bwd_data"] += t_mi * cnt
            tot["ours_bwd_data"] += min(best, t_mi) * cnt
        dy = torch.randn_like(y)
        t_mi = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, wb, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
            [False, True, False]), args.reps)
        res["miopen_wgrad_us"] = round(t_mi, 1)
        best = None
        for v in conv.wgrad_variants_for(cin, cout):
            bm, bn = conv.WGRAD_TILES[v]
            tiles = (cout // bm) * (k * k * cin // bn)
            auto = max(1, (1024 + tiles // 2) // tiles)
            for sp in sorted({max(1, auto // 2), auto, auto * 2}):
                t = timeit(lambda: conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, splits=sp),
                           args.reps)
                res[f"ours_wgrad_v{v}_s{sp}_us"] = round(t, 1)
                best = t if best is None else min(best, t)
        res["wgrad_speedup"] = round(t_mi / best, 3)
        tot["miopen_wgrad"] += t_mi * cnt
        tot["ours_wgrad"] += min(best, t_mi) * cnt
        print(json.dumps(res), flush=True)
    print(json.dumps({"total_us_per_step": {k: round(v, 1) for k, v in tot.items()},
                      "numerics_failures": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
