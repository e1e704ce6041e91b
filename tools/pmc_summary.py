#!/usr/bin/env python3
"""Aggregate a rocprofv3 ``--pmc ... --kernel-trace --output-format csv`` run per kernel.

Reads ``*_counter_collection.csv`` (one row per dispatch and counter) and ``*_kernel_trace.csv``
(one row per dispatch) from a directory and prints, per kernel name (truncated), the dispatch
count, total time, and each counter summed over dispatches, plus derived ratios when the
counters are present:
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs... reported raw per wave-cycle)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue_stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  l2_hit      = TCC_HIT / (TCC_HIT + TCC_MISS), lds_conf = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS

    python tools/pmc_summary.py gpurun_out/r3_pmc1 --top 25 > summary.txt
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--width", type=int, default=90)
    ap.add_argument("--last-frac", type=float, default=1.0,
                    help="only the dispatches in the last fraction of the run (by dispatch id): "
                         "drops autotuning and warmup from a steady-state summary")
    a = ap.parse_args()
    cc = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    counters = defaultdict(lambda: defaultdict(float))
    names = set()

    def cut_of(files):
        ids = []
        for f in files:
            with open(f, newline="") as fh:
                ids += [int(r["Dispatch_Id"]) for r in csv.DictReader(fh) if r.get("Dispatch_Id")]
        if not ids or a.last_frac >= 1.0:
            return -1
        ids = sorted(set(ids))
        return ids[int(len(ids) * (1.0 - a.last_frac))]

    cut_c, cut_k = cut_of(cc), cut_of(kt)
    for f in cc:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if cut_c >= 0 and int(row.get("Dispatch_Id") or 0) < cut_c:
                    continue
                k = row.get("Kernel_Name", "?")[: a.width]
                counters[k][row["Counter_Name"]] += float(row["Counter_Value"])
                names.add(row["Counter_Name"])
    time_ns = defaultdict(float)
    calls = defaultdict(int)
    for f in kt:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if cut_k >= 0 and int(row.get("Dispatch_Id") or 0) < cut_k:
                    continue
                k = row.get("Kernel_Name", "?")[: a.width]
                time_ns[k] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                calls[k] += 1
    keys = sorted(set(counters) | set(time_ns), key=lambda k: -time_ns.get(k, 0.0))[: a.top]
    names = sorted(names)
    print("kernel\tcalls\ttotal_us\t" + "\t".join(names) +
          "\twait_frac\tissue_stall\tmfma_per_wavecyc\tl2_hit\tlds_conf_per_inst")
    for k in keys:
        c = counters.get(k, {})
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        der = [
            c.get("SQ_WAIT_ANY", 0.0) / wc if wc else float("nan"),
            c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else float("nan"),
            c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (4 * wc) if wc else float("nan"),
        ]
        h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        der.append(h / (h + m) if (h + m) else float("nan"))
        li = c.get("SQ_INSTS_LDS", 0.0)
        der.append(c.get("SQ_LDS_BANK_CONFLICT", 0.0) / li if li else float("nan"))
        print(f"{k}\t{calls.get(k, 0)}\t{time_ns.get(k, 0.0) / 1e3:.1f}\t" +
              "\t".join(f"{c.get(n, 0.0):.4g}" for n in names) + "\t" +
              "\t".join(f"{v:.3f}" for v in der))


if __name__ == "__main__":
    main()
