#!/usr/bin/env python3
"""Per-arm kernel times of a tools/conv_layer_pmc.py run under ``rocprofv3 --kernel-trace``.

conv_layer_pmc.py runs its (layer, direction, variant) arms one after another: a forward arm is
one probe call, 2 warmups and ``reps`` timed calls, a backward-data arm 2 + ``reps`` calls, one
conv kernel dispatch each. This walks the trace's conv dispatches in order, assigns them to the
arms, and prints the median of each arm's timed dispatches (weight-gradient arms are skipped:
their split-K reduction launches make the count variable, so runs with --wgrad are refused).

    python tools/arm_times.py gpurun_out/run_kernel_trace.csv gpurun_out/ws2_arms.jsonl
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys


def is_conv(name: str) -> bool:
    return ("conv2_kernel" in name or "conv_fwd_kernel" in name) and "flip" not in name


def main():
    trace, arms_path = sys.argv[1], sys.argv[2]
    arms = [json.loads(line) for line in open(arms_path)]
    if any(a["dir"] == "wgrad" for a in arms):
        raise SystemExit("arm_times: weight-gradient arms are not supported")
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    convs = [r for r in rows if is_conv(r["Kernel_Name"])]
    i = 0
    out = []
    for a in arms:
        n = (3 if a["dir"] == "fwd" else 2) + a["reps"]
        chunk = convs[i:i + n]
        i += n
        ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in chunk[-a["reps"]:]]
        rec = dict(a, us=round(statistics.median(ts), 1),
                   kernel=re.sub(r"\(anonymous namespace\)::", "",
                                 chunk[-1]["Kernel_Name"]).split("(")[0].replace("void ", ""))
        out.append(rec)
        print(json.dumps(rec))
    if i != len(convs):
        print(f"# warning: {len(convs) - i} conv dispatches not assigned to arms", file=sys.stderr)


if __name__ == "__main__":
    main()
