#!/usr/bin/env python3
"""Per-layer conv times of the ResNet-50 training step as the autotuner measured them.

Builds the cnn_bench model, runs two eager training steps (which tune every conv shape), then
prints one JSON line per distinct conv shape: the chosen forward / backward-data / weight-gradient
variant, its time, the layer count, and a roofline floor (FLOPs at 1.3 PFLOP/s vs minimum bytes at
5 TB/s), plus a summary line. Tells which layers hold the conv share of the step.

    python tools/conv_plan_dump.py > gpurun_out/conv_plan.jsonl
"""
from __future__ import annotations

import json
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.examples import cnn_bench  # noqa: E402
from arena_amd.ops import conv  # noqa: E402


def main():
    batch = int(os.environ.get("BATCH", "128"))
    args = cnn_bench.parse(["--model", "resnet50", "--batch_size", str(batch), "--dtype", "bf16"])
    dev = torch.device("cuda")
    model, opt, x, y = cnn_bench.build(args, dev, 1)
    for _ in range(2):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
    torch.cuda.synchronize()
    counts = Counter()
    for m in model.modules():
        if isinstance(m, conv.Conv2dNHWC):
            counts[(m.in_channels, m.out_channels, m.kernel_size[0], m.stride[0])] += 1
    tot = Counter()
    for key, plan in conv._PLANS.items():
        xs, ws, stride, pad = key[0], key[1], key[2], key[3]
        n, c, h, w = xs
        co, _, r, s = ws
        ho, wo = conv.out_hw(h, w, r, s, stride, pad)
        cnt = counts.get((c, co, r, stride), 1)
        flop = 2.0 * n * ho * wo * co * c * r * s
        row = {"layer": f"{r}x{s}/{stride} {c}->{co} @{h}x{w}", "count": cnt,
               "gflop": round(flop / 1e9, 2)}
        byts = {"fwd": 2 * (n * h * w * c + n * ho * wo * co),
                "bwd": 2 * (n * h * w * c + n * ho * wo * co),
                "wgrad": 2 * (n * h * w * c + n * ho * wo * co)}
        for kind in ("fwd", "bwd", "wgrad"):
            choice = getattr(plan, kind)
            t = plan.times.get(f"{kind}:{choice}")
            floor = max(flop / 1.3e15, byts[kind] / 5e12) * 1e6
            row[kind] = {"choice": str(choice), "us": t, "floor_us": round(floor, 1)}
            if t is not None:
                tot[kind] += t * cnt
                tot[kind + "_floor"] += floor * cnt
        row["all"] = plan.times
        print(json.dumps(row), flush=True)
    print(json.dumps({"summary_us_per_step": {k: round(v, 1) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
