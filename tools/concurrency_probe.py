#!/usr/bin/env python3
"""Would running a layer's backward-data and weight-gradient kernels at the same time pay?

For the latency-bound 14x14 / 7x7 ResNet-50 layers (batch 128) each direction alone leaves most
of the MFMA pipe idle. This probe times, per layer, captured in hipGraphs of ``reps`` repetitions:
dgrad alone, wgrad alone (split-K + its reduction), both in sequence on one stream, and both on
two streams (fork / join inside the graph). One JSON line per layer.

    python tools/concurrency_probe.py > gpurun_out/concurrency_probe.jsonl
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import conv  # noqa: E402

# (cin, cout, k, hw, dgrad variant, (wgrad variant, splits)) -- the tuner's picks in
# profiles/r6_conv_budget_per_layer_floors.md
LAYERS = [
    (256, 1024, 1, 14, 4098, (4, 32)),
    (1024, 256, 1, 14, 4107, (4, 32)),
    (256, 256, 3, 14, 4108, (4, 29)),
    (512, 2048, 1, 7, 4103, (4, 8)),
    (2048, 512, 1, 7, 4106, (4, 8)),
    (512, 512, 3, 7, 4110, (12, 4)),
]


def timed(fn, reps=8, iters=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / (reps * iters)


def main():
    n = int(os.environ.get("BATCH", "128"))
    gen = torch.Generator(device="cuda").manual_seed(0)
    side = torch.cuda.Stream()
    for cin, cout, k, hw, vd, (vw, sp) in LAYERS:
        cl = torch.channels_last
        x = torch.randn(n, cin, hw, hw, device="cuda", generator=gen).to(torch.bfloat16).contiguous(
            memory_format=cl)
        dy = torch.randn(n, cout, hw, hw, device="cuda", generator=gen).to(
            torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, k, k, device="cuda", generator=gen) * 0.05).to(
            torch.bfloat16).contiguous(memory_format=cl)
        wf = conv.flip_weight(w)
        pad = (k - 1) // 2

        def dgrad():
            conv.conv2d_bwd_data(dy, w, pad, vd, wflip=wf)

        def wgrad():
            conv.conv2d_wgrad(x, dy, (k, k), 1, pad, vw, sp)

        def seq():
            dgrad()
            wgrad()

        def par():
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                wgrad()
            dgrad()
            main.wait_stream(side)

        r = {"layer": f"{k}x{k} {cin}->{cout} @{hw}", "dgrad_us": round(timed(dgrad), 1),
             "wgrad_us": round(timed(wgrad), 1), "seq_us": round(timed(seq), 1),
             "two_streams_us": round(timed(par), 1)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
