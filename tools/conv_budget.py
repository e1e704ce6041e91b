#!/usr/bin/env python3
"""Per-class convolution budget of the ResNet-50 bs128 training step.

Builds the cnn_bench model, runs eager training steps (which tune every conv shape), then sums
the tuned per-layer kernel times of the directions the step actually runs -- forward with its
BatchNorm-statistics epilogue, backward-data (the BN-linked form where the layer's input is a
BatchNorm output and its dgrad is stride 1; plain otherwise), weight gradient incl. its split
reduction -- weighted by the layer counts, into classes:

    1x1 s1, 3x3 s1, 3x3 s2, 1x1 s2, stem  x  fwd / dgrad / wgrad

Each class row: us per step, TFLOP/s, % of the 2.5 PFLOP/s dense bf16 peak, and x its byte floor
(minimum bytes -- inputs read once, output written once -- at the 4.75 TB/s device-copy rate
measured on this box in round 5). Prints a markdown table, then one JSON line per layer.

    python tools/conv_budget.py > gpurun_out/conv_budget.md
"""
from __future__ import annotations

import json
import os
import sys
from collections import Counter, defaultdict

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.examples import cnn_bench  # noqa: E402
from arena_amd.ops import conv  # noqa: E402

PEAK = 2.5e15
HBM = 4.75e12


def main():
    batch = int(os.environ.get("BATCH", "128"))
    args = cnn_bench.parse(["--model", "resnet50", "--batch_size", str(batch), "--dtype", "bf16"])
    dev = torch.device("cuda")
    model, opt, x, y = cnn_bench.build(args, dev, 1)
    for _ in range(2):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
    torch.cuda.synchronize()
    counts = Counter()
    # layers whose input is NOT a BatchNorm output: the first block's conv1 and shortcut (they
    # read the max pool's output), so their dgrad runs unlinked
    unlinked = Counter()
    for name, m in model.named_modules():
        if isinstance(m, conv.Conv2dNHWC) and not isinstance(m, conv.StemConv2d):
            key = (m.in_channels, m.out_channels, m.kernel_size[0], m.stride[0])
            counts[key] += 1
            if name.startswith("layers.0.") and (name.endswith("conv1") or "down" in name):
                unlinked[key] += 1
    cls = defaultdict(lambda: {"us": 0.0, "flop": 0.0, "bytes": 0.0})
    rows = []
    for key, plan in conv._PLANS.items():
        xs, ws, stride, pad = key[0], key[1], key[2], key[3]
        n, c, h, w = xs
        co, _, r, s = ws
        ho, wo = conv.out_hw(h, w, r, s, stride, pad)
        k = (c, co, r, stride)
        cnt = counts.get(k, 0)
        if cnt == 0:
            continue
        flop = 2.0 * n * ho * wo * co * c * r * s
        io = 2.0 * (n * h * w * c + n * ho * wo * co)
        name = f"{r}x{s} s{stride}"
        row = {"layer": f"{r}x{s}/{stride} {c}->{co} @{h}x{w}", "count": cnt,
               "gflop": round(flop / 1e9, 2)}
        for kind in ("fwd", "bwd", "wgrad"):
            choice = getattr(plan, kind)
            t = plan.times.get(f"{kind}:{choice}")
            parts = [(t, cnt)]
            if kind == "bwd" and stride == 1:
                tb = plan.times.get(f"bwdbn:{plan.bwd_bn}")
                if tb is not None:
                    parts = [(tb, cnt - unlinked[k]), (t, unlinked[k])]
                    row["bwd_linked_us"] = tb
                    row["bwd_linked_choice"] = str(plan.bwd_bn)
                    # floor of the linked form: dy in, dx out, the BN input x and its ReLU bits in
                    lb = (2.0 * n * ho * wo * co + 2.0 * n * h * w * c * 2 + n * h * w * c / 8)
                    row["bwd_linked_x_floor"] = round(tb / (lb / HBM * 1e6), 2)
            if t is None:
                continue
            row[kind] = {"choice": str(choice), "us": t,
                         "x_floor": round(t / ((io + (2.0 * co * c * r * s if kind != "wgrad" else 0))
                                              / HBM * 1e6), 2)}
            # the linked dgrad also reads the BN input (bf16) and its ReLU bits
            extra = (2.0 * n * h * w * c + n * h * w * c / 8) if kind == "bwd" else 0.0
            for tt, nn in parts:
                if tt is None or nn <= 0:
                    continue
                d = cls[(name, kind)]
                d["us"] += tt * nn
                d["flop"] += flop * nn
                d["bytes"] += (io + (extra if tt is not t else 0.0)) * nn
        rows.append(row)
    stem = conv._STEM_PLANS
    print("| class | direction | us / step | TFLOP/s | % of 2.5 PF | x byte floor |")
    print("|---|---|---|---|---|---|")
    tot = 0.0
    order = ["1x1 s1", "3x3 s1", "3x3 s2", "1x1 s2"]
    for name in order:
        for kind in ("fwd", "bwd", "wgrad"):
            d = cls.get((name, kind))
            if not d:
                continue
            tot += d["us"]
            tf = d["flop"] / (d["us"] * 1e-6) / 1e12
            floor = d["bytes"] / HBM * 1e6
            print(f"| {name} | {'dgrad' if kind == 'bwd' else kind} | {d['us']:.0f} | {tf:.0f} | "
                  f"{100 * tf * 1e12 / PEAK:.0f} % | {d['us'] / floor:.2f} |")
    print(f"| all (excl. stem) | | {tot:.0f} | | | |")
    print()
    print(json.dumps({"stem_plans": {str(k): v for k, v in stem.items()}}))
    for row in rows:
        print(json.dumps(row))


if __name__ == "__main__":
    main()
