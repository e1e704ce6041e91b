#!/usr/bin/env python3
"""Which framework ops launch the small "glue" kernels of a ResNet training step (copies, fills,
adds, flips)? Runs eager steps under torch.profiler and prints, per aten op that launched GPU
work outside the arena/MIOpen kernels, its device time per step and the Python frames above it.

    python tools/cnn_glue_prof.py [--model resnet50] [--batch 128] > gpurun_out/glue.txt
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

GLUE = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::flip",
        "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy", "aten::zeros",
        "aten::mul", "aten::mul_", "aten::sum", "aten::cat")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    from arena_amd.examples import cnn_bench
    from arena_amd.parallel import hvd
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = True
    hvd.init("gloo")
    args = cnn_bench.parse(["--model", a.model, "--batch_size", str(a.batch)])
    model, opt, x, y = cnn_bench.build(args, dev, 1)
    for _ in range(3):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for _ in range(a.steps):
            cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
        torch.cuda.synchronize()
    rows = []
    for ev in prof.key_averages(group_by_stack_n=6):
        if ev.key not in GLUE:
            continue
        dev_us = getattr(ev, "self_device_time_total", 0) or getattr(ev, "device_time_total", 0)
        if dev_us <= 0:
            continue
        rows.append((dev_us / a.steps, ev.count / a.steps, ev.key, ev.stack))
    rows.sort(key=lambda r: -r[0])
    tot = collections.Counter()
    for us, n, key, stack in rows:
        tot[key] += us
        frames = [f for f in stack if "arena_amd" in f or "torch/autograd" in f][:4]
        print(f"{us:8.1f} us/step {n:5.1f}/step  {key}")
        for f in frames:
            print(f"            {f}")
    print("--- per op ---")
    for k, v in tot.most_common():
        print(f"{v:8.1f} us/step  {k}")
    print("--- device kernels (per step) ---")
    kern = collections.Counter()
    cnt = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA:
            kern[ev.name[:90]] += ev.device_time_total / a.steps if hasattr(ev, "device_time_total") else 0
            cnt[ev.name[:90]] += 1 / a.steps
    for k, v in kern.most_common(40):
        print(f"{v:8.1f} us {cnt[k]:5.1f}x  {k}")
    hvd.shutdown()


if __name__ == "__main__":
    main()
