#!/usr/bin/env python3
"""How much do the BatchNorm-sum epilogues pay for same-address fp64 atomics?

For the ResNet-50 bs128 layers, times the chosen-style conv variants in three forms: no BN sums,
per-tile partials (plain stores, no atomics), and the acc form (fp64 atomics into the replicated
set, abi.h ARENA_ACC_REP). Forward: statistics of y; backward-data: the linked BN-backward sums.
acc - partials bounds what more replicas (less contention) could recover per layer.

    python tools/acc_contention_probe.py > gpurun_out/acc_probe.jsonl
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import conv  # noqa: E402
from arena_amd.ops.batchnorm import acc_rep  # noqa: E402

# (N, Cin, H, W, Cout, k, count per step)
LAYERS = [(128, 64, 56, 56, 256, 1, 4), (128, 256, 56, 56, 64, 1, 2), (128, 64, 56, 56, 64, 3, 3),
          (128, 64, 56, 56, 64, 1, 1), (128, 256, 56, 56, 128, 1, 1),
          (128, 128, 28, 28, 512, 1, 4), (128, 512, 28, 28, 128, 1, 3),
          (128, 128, 28, 28, 128, 3, 3), (128, 256, 14, 14, 1024, 1, 6),
          (128, 1024, 14, 14, 256, 1, 5), (128, 256, 14, 14, 256, 3, 5),
          (128, 512, 7, 7, 2048, 1, 3), (128, 2048, 7, 7, 512, 1, 2), (128, 512, 7, 7, 512, 3, 2)]


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    ext = conv._ext.load()
    for n, ci, h, w_, co, k, cnt in LAYERS:
        pad = k // 2
        x = torch.randn(n, ci, h, w_, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = (torch.randn(co, ci, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(n, co, h, w_, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        m = n * h * w_
        rec = {"layer": f"{ci}->{co} k{k} @{h}", "count": cnt}
        for direction, c, kc in (("fwd", co, ci), ("bwd", ci, co)):
            cands = conv.v2_variants_for(c) + conv.halo_variants_for(c, (k, k), 1, pad, w_, kc)
            best = {}
            for v in cands:
                try:
                    if direction == "fwd":
                        plain = conv._time(lambda: conv.conv2d_fwd(x, wt, 1, pad, v))
                        acc = torch.zeros(acc_rep() * 2 * c, dtype=torch.float64, device=dev)
                        ext.bn_acc_scratch(True)
                        try:
                            part = conv._time(lambda: conv.conv2d_fwd(x, wt, 1, pad, v,
                                                                      with_stats=True))
                            fin = conv._time(lambda: conv.conv2d_fwd(x, wt, 1, pad, v,
                                                                     with_stats=True, final=True))
                        finally:
                            ext.bn_acc_scratch(False)
                    else:
                        bnx = torch.randn_like(x)
                        bmask = torch.randint(0, 256, (m * ci // 8,), device=dev,
                                              dtype=torch.uint8)
                        bmean = torch.zeros(ci, device=dev)
                        acc = torch.zeros(acc_rep() * 2 * ci, dtype=torch.float64, device=dev)
                        plain = conv._time(lambda: conv.conv2d_bwd_data(dy, wt, pad, v))
                        part = conv._time(lambda: conv.conv2d_bwd_data(
                            dy, wt, pad, v, bn=(bnx, bmask, bmean)))
                        fin = conv._time(lambda: conv.conv2d_bwd_data(
                            dy, wt, pad, v, bn=(bnx, bmask, bmean), bn_acc=acc))
                except RuntimeError as e:   # shape not taken by this variant
                    print(f"skip {rec['layer']} {direction} {v}: {e}", file=sys.stderr)
                    continue
                best[v] = (round(plain, 1), round(part, 1), round(fin, 1))
            if best:
                v = min(best, key=lambda q: best[q][2])
                rec[direction] = {"variant": v, "plain_part_acc_us": best[v],
                                  "best_part_us": min(b[1] for b in best.values())}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
