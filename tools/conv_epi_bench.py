#!/usr/bin/env python3
"""Cost of the BatchNorm-statistics epilogue (EPI 1) of the conv kernel, per ResNet-50 layer.

For every conv with C % 64 == 0 and every tile variant: graph-replayed GPU time of the plain
forward and of the forward that also writes the per-tile BN partials. One JSON line per layer.

    python tools/conv_epi_bench.py --batch 128 > gpurun_out/conv_epi.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import conv  # noqa: E402
from tools.conv_roofline import resnet50_convs, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--variants", default="", help="comma list (default: every variant)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    want = [int(v) for v in args.variants.split(",")] if args.variants else None
    tot_plain = tot_stats = 0.0
    for (n, h, w, cin, cout, k, st), cnt in resnet50_convs(args.batch):
        if cin % 64:
            continue
        pad = k // 2
        x = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        row = {"layer": f"{k}x{k}/{st} {cin}->{cout} @{h}x{w}", "count": cnt}
        bp = bs = None
        for v in conv.variants_for(cout):
            if want is not None and v not in want:
                continue
            tp = timeit(lambda: conv.conv2d_fwd(x, wt, st, pad, v), args.reps)
            ts = timeit(lambda: conv.conv2d_fwd(x, wt, st, pad, v, with_stats=True), args.reps)
            row[f"v{v}_plain_us"] = round(tp, 1)
            row[f"v{v}_stats_us"] = round(ts, 1)
            bp = tp if bp is None else min(bp, tp)
            bs = ts if bs is None else min(bs, ts)
        row["best_plain_us"], row["best_stats_us"] = round(bp, 1), round(bs, 1)
        tot_plain += bp * cnt
        tot_stats += bs * cnt
        print(json.dumps(row), flush=True)
        del x, wt
        torch.cuda.empty_cache()
    print(json.dumps({"summary": True, "step_fwd_plain_us": round(tot_plain, 1),
                      "step_fwd_stats_us": round(tot_stats, 1)}), flush=True)


if __name__ == "__main__":
    main()
