#!/usr/bin/env python3
"""Time-to-accuracy of the MNIST demo workload on one GPU (BASELINE.md north-star rows 1-2).

The reference's only published numbers are the demo job's test accuracies (0.9649 at step 990,
docs/userguide/1-tfjob-standalone.md:178-186): TF `mnist_with_summaries` evaluates the test set
every 10 steps. This script does the same loop -- 10 training steps, then a full 10k test-set
evaluation -- and reports the accuracy at step 990, the first step reaching 97 %, and the wall
time to get there (training + evaluations, synchronised), for the fused HIP trainer and for the
eager PyTorch version of the same model.

    python tools/tta.py [--impl fused|torch|both] [--max_steps 1000] [--target 0.97]

Data: synthetic MNIST-shaped digits (arena_amd.data.mnist), no download on the GPU box.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(impl: str, max_steps: int, target: float, every: int) -> dict:
    from arena_amd.data.mnist import load_mnist
    from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig
    from arena_amd.models.torch_mlp import EagerMLPTrainer
    data = load_mnist()
    cfg = MLPConfig()
    if impl == "fused":
        tr = FusedMLPTrainer(cfg, data.train_images, data.train_labels, device="cuda")
        tr.enable_graphs(every)
    else:
        tr = EagerMLPTrainer(cfg, data.train_images, data.train_labels, device="cuda")
    tx, ty = data.test_images.cuda(), data.test_labels.cuda()
    tr.evaluate(tx, ty)          # warm the eval path (kernel load), not timed
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hit_step = hit_s = None
    acc_at = {}
    step = 0
    while step < max_steps:
        _, acc = tr.evaluate(tx, ty)            # host sync: accuracy is read back
        acc_at[step] = acc
        if hit_step is None and acc >= target:
            hit_step, hit_s = step, time.perf_counter() - t0
        tr.train_steps(every)
        step += every
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    _, final = tr.evaluate(tx, ty)
    return {"impl": impl, "eval_every": every, "steps": max_steps,
            "acc_at_990": round(acc_at.get(990, float("nan")), 4),
            "final_acc": round(final, 4), "target": target, "steps_to_target": hit_step,
            "seconds_to_target": None if hit_s is None else round(hit_s, 4),
            "seconds_total": round(total, 4), "data": data.source}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", choices=["fused", "torch", "both"], default="both")
    ap.add_argument("--max_steps", type=int, default=1000)
    ap.add_argument("--target", type=float, default=0.97)
    ap.add_argument("--eval_every", type=int, default=10)
    a = ap.parse_args()
    impls = ["fused", "torch"] if a.impl == "both" else [a.impl]
    for impl in impls:
        print(json.dumps(run(impl, a.max_steps, a.target, a.eval_every)), flush=True)


if __name__ == "__main__":
    main()
