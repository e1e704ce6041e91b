#!/usr/bin/env python3
"""Effective HBM bandwidth of the BN streaming passes as the training step runs them.

Per ResNet-50 (batch 128, bf16, NHWC) BN shape: the apply pass with its statistics already summed
(the conv-epilogue acc form: no reduction, no finalize) and the backward dx pass fed ready sums
(the linked dgrad's), timed in hipGraphs, bytes counted as the kernels move them. A torch copy of
the largest tensor is the reference rate; ``x_floor`` is each pass's time over its bytes at the
4.75 TB/s floor rate (below 1: the MALL serves part of the bytes).

    python tools/bn_pass_bw.py --configs slice:4096,flat:4096 > gpurun_out/bn_pass_bw.jsonl

Each config is <grid>:<dx max blocks>: grid ``slice`` (256-channel slices for C > 256, the
default) or ``flat``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import _ext  # noqa: E402
from arena_amd.ops.batchnorm import acc_rep  # noqa: E402
from arena_amd.ops.conv import _time  # noqa: E402

# the byte floor's rate: the 4.75 TB/s of a large device copy (read + write) on this box, round 5
FLOOR_BPS = 4.75e12

# (rows M at batch 128, channels C, uses per step, relu, residual)
SHAPES = [
    (128 * 56 * 56, 64, 6, True, False),
    (128 * 56 * 56, 256, 3, True, True),
    (128 * 56 * 56, 128, 1, True, False),
    (128 * 28 * 28, 128, 7, True, False),
    (128 * 28 * 28, 512, 4, True, True),
    (128 * 28 * 28, 256, 1, True, False),
    (128 * 14 * 14, 256, 11, True, False),
    (128 * 14 * 14, 1024, 6, True, True),
    (128 * 14 * 14, 512, 1, True, False),
    (128 * 7 * 7, 512, 5, True, False),
    (128 * 7 * 7, 2048, 3, True, True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="slice:1024")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ext = _ext.load()
    for cfg in a.configs.split(","):
        grid, _, dxb = cfg.partition(":")
        ext.bn_set_slice(1 if grid == "slice" else 0)
        ext.bn_set_dx_max_blocks(int(dxb or 1024))
        print(json.dumps({"config": cfg}), flush=True)
        run(ext, dev)
    ext.bn_set_slice(1)
    ext.bn_set_dx_max_blocks(1024)


def run(ext, dev):
    big = torch.empty(128 * 56 * 56 * 256 * 2, dtype=torch.bfloat16, device=dev)
    big2 = torch.empty_like(big)
    t = _time(lambda: big2.copy_(big))
    print(json.dumps({"copy_MB": round(big.numel() * 2 / 1e6), "us": round(t, 1),
                      "TBps": round(2 * big.numel() * 2 / t / 1e6, 2)}), flush=True)
    del big, big2
    tot = {"apply": [0.0, 0.0], "dx": [0.0, 0.0]}
    for m, c, uses, relu, res in SHAPES:
        n = 128
        hw = m // n
        h = int(round(hw ** 0.5))
        x = torch.randn(n, c, h, h, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        dy = torch.randn_like(x)
        g = torch.ones(c, device=dev)
        b = torch.zeros(c, device=dev)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        fin = torch.zeros(acc_rep() * 2 * c, dtype=torch.float64, device=dev)
        fin.view(-1, 2, c)[0, 1].fill_(float(m))       # unit variance
        out = ext.bn_fwd(x, r, g, b, rm, rv, True, 0.1, 1e-5, relu, None, None, 0, stats_fin=fin)
        mean, invstd, mask = out[1], out[2], out[3]
        ta = _time(lambda: ext.bn_fwd(x, r, g, b, rm, rv, True, 0.1, 1e-5, relu, None, None, 0,
                                      stats_fin=fin))
        acc = torch.zeros(acc_rep() * 2 * c, dtype=torch.float64, device=dev)
        td = _time(lambda: ext.bn_bwd(dy, mask, x, mean, invstd, g, relu, res, True, acc_b=acc,
                                      acc_ready=True))
        e = m * c * 2
        bits = m * c // 8 if relu else 0
        ba = e * (2 + (1 if res else 0)) + bits
        bd = e * (3 + (1 if res else 0)) + bits
        rec = {"M": m, "C": c, "uses": uses, "res": res,
               "apply_us": round(ta, 1), "apply_TBps": round(ba / ta / 1e6, 2),
               "apply_x_floor": round(ta / (ba / FLOOR_BPS * 1e6), 2),
               "dx_us": round(td, 1), "dx_TBps": round(bd / td / 1e6, 2),
               "dx_x_floor": round(td / (bd / FLOOR_BPS * 1e6), 2)}
        tot["apply"][0] += uses * ta
        tot["apply"][1] += uses * ba
        tot["dx"][0] += uses * td
        tot["dx"][1] += uses * bd
        print(json.dumps(rec), flush=True)
    print(json.dumps({k: {"us_per_step": round(v[0], 1), "TBps": round(v[1] / v[0] / 1e6, 2),
                          "x_floor": round(v[0] / (v[1] / FLOOR_BPS * 1e6), 2)}
                      for k, v in tot.items()}), flush=True)


if __name__ == "__main__":
    main()
