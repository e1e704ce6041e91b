#!/usr/bin/env python3
"""Where the 3x3 halo conv kernel's time goes: per ResNet-50 3x3 layer (batch 128), each halo
variant timed with parts of its K loop switched off (ConvArgs::dbg, timing only -- the outputs
are garbage with any bit set):

    0  the kernel as it runs          1  no weight loads after chunk 0's prologue
    2  no window loads after chunk 0  4  no barriers in the tap loop     8  no MFMAs

and combinations. One JSON line per (layer, variant, flags): us, TFLOP/s.

    python tools/halo_ablation.py > gpurun_out/halo_ablation.jsonl
    FLAGS=0 python tools/halo_ablation.py     # the variants as they run, no ablation
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import _ext, conv  # noqa: E402

LAYERS = [(64, 56), (128, 28), (256, 14), (512, 7)]
FLAGS = [int(f) for f in os.environ.get("FLAGS", "0,1,2,3,4,8,12,15").split(",")]


def main():
    n = int(os.environ.get("BATCH", "128"))
    ext = _ext.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    for c, hw in LAYERS:
        x = torch.randn(n, c, hw, hw, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda", generator=g) * 0.05).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        flop = 2.0 * n * hw * hw * c * c * 9
        for v in conv.halo_variants_for(c, (3, 3), 1, 1, hw, c):
            for stats in (False, True):
                for f in FLAGS:
                    ext.conv_set_dbg(f)
                    try:
                        us = conv._time(lambda: conv.conv2d_fwd(x, w, 1, 1, v, with_stats=stats,
                                                                final=stats), reps=8, iters=5)
                    finally:
                        ext.conv_set_dbg(0)
                    print(json.dumps({"layer": f"3x3 {c}@{hw}", "variant": v, "stats": stats,
                                      "flags": f, "us": round(us, 2),
                                      "tflops": round(flop / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
