#!/usr/bin/env python3
"""Are results of a captured hipGraph correct when every kernel reads data the previous kernel
wrote from OTHER workgroups (hence other XCDs, whose L2 is separate on MI355X)? An elementwise
chain never does (workgroup i reads what workgroup i wrote); a permuted gather always does.

Each replay: y = x[perm] + 1 ; x = y[inv] (so x grows by exactly 1 per replay, elementwise).
With eager traffic between replays (to churn the caches) the result must stay exact.

    python scripts/graph_xcd_check.py [--n 16777216] [--replays 50] [--eager 200]
"""
from __future__ import annotations

import argparse

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 24)
    ap.add_argument("--chain", type=int, default=20, help="gather pairs per replay")
    ap.add_argument("--replays", type=int, default=50)
    ap.add_argument("--eager", type=int, default=200, help="eager kernels between replays")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g0 = torch.Generator(device=dev).manual_seed(0)
    perm = torch.randperm(a.n, device=dev, generator=g0)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(a.n, device=dev)
    x0 = torch.randn(a.n, device=dev, generator=g0).round()
    x = x0.clone()
    y = torch.empty_like(x)

    def body():
        for _ in range(a.chain):
            torch.index_select(x, 0, perm, out=y)
            y.add_(1.0)
            torch.index_select(y, 0, inv, out=x)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    x.copy_(x0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    x.copy_(x0)
    junk = torch.randn(1 << 22, device=dev)
    bad = 0
    for r in range(1, a.replays + 1):
        g.replay()
        for _ in range(a.eager):
            junk = junk * 1.0001 + 0.5
        torch.cuda.synchronize()
        err = float((x - (x0 + r * a.chain)).abs().max())
        if err != 0.0:
            bad += 1
            print(f"replay {r}: max err {err}", flush=True)
    print(f"{bad} of {a.replays} replays wrong", flush=True)


if __name__ == "__main__":
    main()
