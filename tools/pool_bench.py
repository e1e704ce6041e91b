#!/usr/bin/env python3
"""ResNet-50 stem max pool (batch 128, 64 x 112 x 112, bf16 NHWC, 3x3 / 2 / pad 1): the fused HIP
kernels vs PyTorch's max_pool2d, forward and backward, microseconds per call (best of 3 x 20)."""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    return round(best, 1)


def main():
    from arena_amd.ops import _ext
    ext = _ext.load()
    x = torch.randn(128, 64, 112, 112, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y, pos = ext.maxpool_fwd(x, 3, 2, 1)
    dy = torch.randn_like(y)
    xr = x.detach().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    out = {
        "shape": "128x64x112x112 bf16 NHWC, k3 s2 p1",
        "arena_fwd_us": timed(lambda: ext.maxpool_fwd(x, 3, 2, 1)),
        "arena_bwd_us": timed(lambda: ext.maxpool_bwd(dy, pos, 112, 112, 3, 2, 1)),
        "torch_fwd_us": timed(lambda: F.max_pool2d(x, 3, 2, 1)),
        "torch_fwd_bwd_us": timed(lambda: torch.autograd.grad(F.max_pool2d(xr, 3, 2, 1), xr, dy)),
    }
    out["torch_bwd_us_approx"] = round(out["torch_fwd_bwd_us"] - out["torch_fwd_us"], 1)
    # bytes: fwd reads x once (window overlap served by cache), writes y + pos; bwd reads dy + pos
    # (~once), writes dx
    ex, ey = x.numel(), y.numel()
    out["arena_fwd_TBs"] = round((2 * ex + 3 * ey) / out["arena_fwd_us"] / 1e6, 2)
    out["arena_bwd_TBs"] = round((2 * ex + 3 * ey) / out["arena_bwd_us"] / 1e6, 2)
    print(json.dumps(out), flush=True)
    del yr


if __name__ == "__main__":
    main()
