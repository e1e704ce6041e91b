#!/usr/bin/env python3
"""Run chosen conv kernel variants on chosen ResNet-50 layers, one after another, for a profiler.

Each (layer, direction, variant) arm is warmed up, then run ``--reps`` times eagerly, so a
``rocprofv3 --kernel-trace [--pmc ...]`` run attributes times and counters per kernel dispatch;
``--arms-out`` records the arm order (the dispatch sequence) for tools/pmc_summary.py. No
autotuning, no MIOpen.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc -o run -- \\
        python3 tools/conv_layer_pmc.py --layers 14:256:256:3:1 --variants 0,8,4096,4098
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import conv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--layers", default="14:256:256:3:1",
                    help="comma list of hw:cin:cout:k:stride")
    ap.add_argument("--variants", default="0,4096",
                    help="forward/dgrad tile variants (v1 codes, 4096 + i for v2)")
    ap.add_argument("--wgrad", default="", help="weight-gradient variants (v1 0..7, v2 8..11)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--arms-out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda")
    arms = []
    for spec in args.layers.split(","):
        hw, cin, cout, k, st = (int(v) for v in spec.split(":"))
        pad = k // 2
        g = torch.Generator(device=dev).manual_seed(hw + cin + cout)
        x = torch.randn(args.batch, cin, hw, hw, device=dev, generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device=dev, generator=g) * 0.05).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ho, wo = conv.out_hw(hw, hw, k, k, st, pad)
        dy = torch.randn(args.batch, cout, ho, wo, device=dev, generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        for v in (int(s) for s in args.variants.split(",") if s):
            if cout % conv.TILES[v][1]:
                continue
            try:   # shape-restricted forms (halo: 3x3 / stride 1 / pad 1)
                conv.conv2d_fwd(x, w, st, pad, v)
            except RuntimeError:
                continue
            for _ in range(2):
                conv.conv2d_fwd(x, w, st, pad, v)
            torch.cuda.synchronize()
            for _ in range(args.reps):
                conv.conv2d_fwd(x, w, st, pad, v)
            torch.cuda.synchronize()
            arms.append({"layer": spec, "dir": "fwd", "variant": v, "reps": args.reps})
            if st == 1 and cin % conv.TILES[v][1] == 0:
                wf = conv.flip_weight(w)
                for _ in range(2):
                    conv.conv2d_bwd_data(dy, w, pad, v, wflip=wf)
                torch.cuda.synchronize()
                for _ in range(args.reps):
                    conv.conv2d_bwd_data(dy, w, pad, v, wflip=wf)
                torch.cuda.synchronize()
                arms.append({"layer": spec, "dir": "bwd", "variant": v, "reps": args.reps})
        for v in (int(s) for s in args.wgrad.split(",") if s):
            if v not in conv.wgrad_variants_for(cin, cout):
                continue
            for _ in range(2):
                conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, 0)
            torch.cuda.synchronize()
            for _ in range(args.reps):
                conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, 0)
            torch.cuda.synchronize()
            arms.append({"layer": spec, "dir": "wgrad", "variant": v, "reps": args.reps})
    if args.arms_out:
        with open(args.arms_out, "w") as f:
            for a in arms:
                f.write(json.dumps(a) + "\n")
    print(json.dumps({"arms": len(arms)}))


if __name__ == "__main__":
    main()
