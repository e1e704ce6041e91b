#!/usr/bin/env python3
"""Graph-launch schedule sweep for the 20-step MNIST window (bench.py --steps 20 --warmup 5).

hipGraph replays are submitted node by node by the host, so the first kernel of a long graph
starts only after its packets are written, while a short graph pays the fixed per-launch cost per
few steps. This times 20 training steps run as different sequences of graph replays (dynamic
step parity, so any sequence is valid) and prints samples/s per schedule (median of reps).

    python tools/mlp_sched_sweep.py
"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from arena_amd.data.mnist import load_mnist  # noqa: E402
from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig  # noqa: E402


def main():
    data = load_mnist()
    tr = FusedMLPTrainer(MLPConfig(), data.train_images, data.train_labels, device="cuda")
    tr.enable_graphs(5)             # allocations, warm code objects
    scheds = [[5, 5, 5, 5], [4, 4, 4, 4, 4], [2, 6, 6, 6], [2, 9, 9], [1, 19], [3, 17],
              [5, 15], [2, 18], [4, 8, 8], [10, 10], [20], [2, 2, 2, 2, 2, 2, 2, 2, 2, 2],
              [1, 4, 5, 5, 5], [2, 3, 5, 5, 5]]
    sizes = sorted({k for s in scheds for k in s})
    graphs = {}
    for k in sizes:
        tr._graph_parity0 = 0
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(k):
                tr._launch_step(parity=-1)
        g.replay()              # upload
        torch.cuda.synchronize()
        graphs[k] = g
    out = []
    for rep in range(7):
        for sch in scheds:
            for _ in range(5):
                tr._launch_step(parity=-1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in sch:
                graphs[k].replay()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            out.append((tuple(sch), 2000 / dt))
    for sch in scheds:
        v = [x for s, x in out if s == tuple(sch)]
        print(json.dumps({"schedule": sch, "samples_per_s_median": round(statistics.median(v)),
                          "max": round(max(v))}), flush=True)


if __name__ == "__main__":
    main()
