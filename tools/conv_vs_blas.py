#!/usr/bin/env python3
"""Library yardstick for the 1x1 stride-1 convolutions of ResNet-50.

A 1x1 stride-1 NHWC convolution IS a GEMM: forward Y[M, Cout] = X[M, Cin] · Wᵀ, backward-data
dX[M, Cin] = dY[M, Cout] · W, backward-weight dW[Cout, Cin] = dYᵀ · X, with M = N·H·W pixels.
For every such layer at the given batch this times, on the same box and the same tensors:

* **ours**: the conv kernels at the plan's autotuned choice (``conv.plan_for``), timed plain and
  in the form the training step runs them (forward with BatchNorm statistics in the epilogue;
  weight gradient including its split-K slab reduction);
* **blas**: the identical GEMM through ``torch.matmul``, with hipBLASLt and with rocBLAS as the
  preferred library (the faster of the two is the yardstick), same bf16 inputs and outputs. The
  weight gradient dYᵀ·X is a small [Cout, Cin] output over a huge M reduction, which a plain
  ``g.t() @ a`` hands the library as ONE GEMM with no split-K (679 us for a 64x64 dW at 56x56:
  not a yardstick). It is timed as a split-K batched GEMM instead: g and a reshaped to [S, M/S, C],
  ``torch.bmm`` over the S slices, then an fp32 sum over S -- the best S of 4..512 (the plain
  form stays in the record as ``blas_plain_us``);
* **floor**: the layer's minimum bytes (inputs read once, output written once) over the copy
  bandwidth measured here with a large device-to-device copy (``--copy-mb``), and its FLOPs over
  2.5 PFLOP/s dense bf16 -- the larger of the two.

One JSON line per layer and direction, then a summary. Timing: graph replays of 4 captured calls,
median of ``--reps`` (``tools/conv_roofline.timeit``).

    python tools/conv_vs_blas.py --batch 128 > gpurun_out/conv_vs_blas.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.ops import conv  # noqa: E402
from tools.conv_roofline import resnet50_convs, timeit  # noqa: E402

PEAK_BF16 = 2.5e15


def copy_bandwidth(mb: int, reps: int) -> float:
    """Device copy bandwidth in bytes/s, counting read + write bytes."""
    a = torch.empty(mb << 18, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    us = timeit(lambda: b.copy_(a), reps)
    return 2 * a.numel() * 4 / (us * 1e-6)


def blas_time(fn, reps: int):
    """(best us, library) of fn over hipBLASLt and rocBLAS."""
    out = {}
    for lib in ("cublaslt", "cublas"):      # torch's names: hipBLASLt / rocBLAS on ROCm
        try:
            torch.backends.cuda.preferred_blas_library(lib)
            out[{"cublaslt": "hipblaslt", "cublas": "rocblas"}[lib]] = timeit(fn, reps)
        except Exception as e:  # noqa: BLE001
            print(f"# {lib}: {e!r}", file=sys.stderr)
    torch.backends.cuda.preferred_blas_library("cublaslt")
    lib = min(out, key=out.get)
    return out[lib], lib, out


def splitk_wgrad(g: torch.Tensor, a: torch.Tensor, reps: int):
    """(best us, library, S) of dW = g^T a as S batched slice GEMMs + an fp32 sum over S."""
    m = g.shape[0]
    best = None
    for s_ in (4, 8, 16, 32, 64, 128, 256, 512):
        if m % s_:
            continue
        gs = g.reshape(s_, m // s_, g.shape[1])
        as_ = a.reshape(s_, m // s_, a.shape[1])

        def fn(gs=gs, as_=as_):
            return torch.bmm(gs.transpose(1, 2), as_).sum(0, dtype=torch.float32)
        t, lib, _ = blas_time(fn, reps)
        if best is None or t < best[0]:
            best = (t, lib, s_)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--copy-mb", type=int, default=1024)
    args = ap.parse_args()
    dev = torch.device("cuda")
    bw = copy_bandwidth(args.copy_mb, args.reps)
    print(json.dumps({"copy_bandwidth_tbps": round(bw / 1e12, 2)}), flush=True)
    conv.set_mode("auto")
    totals = {"ours": 0.0, "ours_step": 0.0, "blas": 0.0, "floor": 0.0}
    worst = []
    for (n, h, w, cin, cout, k, st), cnt in resnet50_convs(args.batch):
        if k != 1 or st != 1:
            continue
        m = n * h * w
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(n, cout, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        plan = conv.plan_for(x, wt, 1, 0)
        a = x.permute(0, 2, 3, 1).reshape(m, cin)            # NHWC views: no copies
        g = dy.permute(0, 2, 3, 1).reshape(m, cout)
        w2 = wt.reshape(cout, cin)
        flop = 2.0 * m * cin * cout
        layer = f"1x1 {cin}->{cout} @{h}x{w}"
        bx, bw_, by = m * cin * 2, cin * cout * 2, m * cout * 2
        dirs = {
            "fwd": (lambda: conv.conv2d_fwd(x, wt, 1, 0, plan.fwd),
                    lambda: conv.conv2d_fwd(x, wt, 1, 0, plan.fwd, with_stats=True,
                                            final=conv._use_acc(m, plan.fwd, cout)),
                    lambda: a @ w2.t(), bx + bw_ + by),
            "dgrad": (lambda: conv.conv2d_bwd_data(dy, wt, 0, plan.bwd),
                      None, lambda: g @ w2, by + bw_ + bx),
            "wgrad": (lambda: conv.conv2d_wgrad(x, dy, (1, 1), 1, 0, plan.wgrad[0],
                                                plan.wgrad[1]),
                      None, lambda: g.t() @ a, by + bx + bw_),
        }
        for d, (ours, ours_step, blas, nbytes) in dirs.items():
            t_ours = timeit(ours, args.reps)
            t_step = timeit(ours_step, args.reps) if ours_step is not None else t_ours
            t_blas, lib, libs = blas_time(blas, args.reps)
            extra = {}
            if d == "wgrad":
                extra["blas_plain_us"] = round(t_blas, 1)
                t_blas, lib, s_ = splitk_wgrad(g, a, args.reps)
                extra["blas_splitk_S"] = s_
            floor = max(nbytes / bw * 1e6, flop / PEAK_BF16 * 1e6)
            rec = {"layer": layer, "dir": d, "count": cnt, "gflop": round(flop / 1e9, 2),
                   "mb": round(nbytes / 2**20, 1),
                   "variant": str(plan.fwd if d == "fwd" else plan.bwd if d == "dgrad"
                                  else plan.wgrad),
                   "ours_us": round(t_ours, 1), "ours_step_form_us": round(t_step, 1),
                   "blas_us": round(t_blas, 1), "blas_lib": lib,
                   "blas_all_us": {k_: round(v, 1) for k_, v in libs.items()},
                   "floor_us": round(floor, 1),
                   "ours_vs_blas": round(t_ours / t_blas, 3),
                   "ours_vs_floor": round(t_ours / floor, 2),
                   "ours_tbps": round(nbytes / t_ours / 1e6, 2), **extra}
            print(json.dumps(rec), flush=True)
            totals["ours"] += t_ours * cnt
            totals["ours_step"] += t_step * cnt
            totals["blas"] += t_blas * cnt
            totals["floor"] += floor * cnt
            worst.append((t_ours / t_blas, layer, d))
        del x, wt, dy
    worst.sort(reverse=True)
    print(json.dumps({"summary_us_per_step_1x1_s1": {k_: round(v, 1) for k_, v in totals.items()},
                      "worst_vs_blas": [[round(r, 3), l_, d] for r, l_, d in worst[:6]]}),
          flush=True)
    conv.set_mode(None)


if __name__ == "__main__":
    sys.exit(main())
