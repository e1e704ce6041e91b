#!/usr/bin/env python3
"""Steady-state kernel breakdown from a rocprofv3 kernel trace: drops everything up to the last
MIOpen find-mode ("naive_conv") kernel, then groups kernels by category.

    python tools/steady_kernels.py gpurun_out/cnn/prof/r50_kernel_trace.csv [--top 40] [--csv out]
"""
import argparse
import collections
import csv


def category(n: str) -> str:
    if n.startswith("(anonymous namespace)::bn_") or "bn_stats" in n or "bn_apply" in n or "bn_bwd" in n:
        return "arena fused BN (HIP)"
    if "BatchNorm" in n:
        return "batchnorm (MIOpen)"
    if "wrw" in n or "bwd_weight" in n or "conv_wgrad" in n:
        return "conv wgrad"
    if "igemm_bwd" in n or "bwd_data" in n:
        return "conv dgrad"
    if "conv_fwd" in n or "igemm_fwd" in n or "conv2_kernel" in n:
        return "conv fwd / dgrad (implicit GEMM)"
    if "conv_phase_weights" in n or "flip_weight" in n:
        return "conv weight transforms"
    if "Cijk" in n or "gemm" in n.lower():
        return "gemm"
    if "elementwise" in n or "Functor" in n:
        return "elementwise (torch)"
    if "fill" in n.lower():
        return "fill"
    if "pool" in n:
        return "pool"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--csv", default="")
    ap.add_argument("--last-ms", type=float, default=0.0,
                    help="keep only kernels that start in the last N ms of the trace (graph "
                         "replays at the end of a run) instead of cutting at MIOpen's find")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    naive = [int(r["End_Timestamp"]) for r in rows if "naive" in r["Kernel_Name"]]
    t_cut = max(naive) if naive else 0
    if a.last_ms > 0:
        t_end = max(int(r["End_Timestamp"]) for r in rows)
        t_cut = t_end - int(a.last_ms * 1e6)
    ss = [r for r in rows if int(r["Start_Timestamp"]) > t_cut]
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])  # noqa: E731
    busy = sum(dur(r) for r in ss)
    span = max(int(r["End_Timestamp"]) for r in ss) - int(ss[0]["Start_Timestamp"])
    cats = collections.defaultdict(lambda: [0, 0])
    kern = collections.defaultdict(lambda: [0, 0])
    for r in ss:
        for d, k in ((cats, category(r["Kernel_Name"])), (kern, r["Kernel_Name"][:110])):
            d[k][0] += 1
            d[k][1] += dur(r)
    print(f"steady-state kernels: {len(ss)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms")
    for k, (c, t) in sorted(cats.items(), key=lambda x: -x[1][1]):
        print(f"{100 * t / busy:6.2f}%  {t / 1e6:9.2f} ms  {c:6d}  {k}")
    out = []
    for k, (c, t) in sorted(kern.items(), key=lambda x: -x[1][1])[:a.top]:
        out.append((100 * t / busy, t / 1e6, c, k))
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("pct,total_ms,calls,kernel\n")
            for p, t, c, k in out:
                f.write(f"{p:.2f},{t:.2f},{c},\"{k}\"\n")


if __name__ == "__main__":
    main()
