#!/usr/bin/env python3
"""Minimal check: does a captured torch-only hipGraph still compute the same result after many
eager kernel launches between its replays? (Isolates a runtime-level problem from our kernels.)

    python scripts/graph_kernarg_check.py [--nodes 200] [--eager 2400]
"""
from __future__ import annotations

import argparse

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=200)
    ap.add_argument("--eager", type=int, default=2400)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(1 << 16, device=dev)
    bufs = [torch.empty_like(x) for _ in range(4)]

    def body():
        t = x
        for i in range(a.nodes):   # distinct scalars: every node has its own kernel arguments
            t = torch.add(t, float(i % 7) * 1e-3, out=bufs[i % 4] if t is not bufs[i % 4] else
                          bufs[(i + 1) % 4])
        return t

    ref = body().clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        out = body()
    g.replay()
    torch.cuda.synchronize()
    print(f"replay before eager: max err {float((out - ref).abs().max()):.3e}", flush=True)
    t = torch.randn(1 << 20, device=dev)
    for _ in range(a.eager):
        t = t * 1.0001 + 0.5
    torch.cuda.synchronize()
    for k in range(3):
        g.replay()
        torch.cuda.synchronize()
        print(f"replay {k} after {a.eager} eager iterations: max err "
              f"{float((out - ref).abs().max()):.3e}", flush=True)


if __name__ == "__main__":
    main()
