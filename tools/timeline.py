#!/usr/bin/env python3
"""Phase timeline of the two training-step kernels (needs the instrumented build):

    rm -rf build/hip_objs && ARENA_TIMELINE=1 python setup.py build_ext --inplace
    python tools/timeline.py

Replays the captured step graph, then reads the per-block s_memrealtime stamps (100 MHz, 10 ns)
of the LAST step's forward (kid 0) and weight-gradient (kid 1) kernels. Reports, per phase, the
median / max over blocks of the time since the kernel's first block started, the block-start
skew, and the fwd-end -> wgrad-start gap (the kernel boundary).
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = {
    0: ["entry", "gather(prow ready)", "mfma done", "lds reduce", "H stored", "atomics issued",
        "drained"],
    1: ["entry", "step ready", "staged (loads+LDS)", "softmax", "dZ image", "mfma done",
        "adam stores issued", "drained"],
}


EXTRA = {1: {8: "x_issued", 9: "head_loads_issued", 10: "logits_issued"}}


def analyse(tl, kid, nblocks):
    t = tl[kid, :nblocks].double() * 10.0 / 1000.0  # ticks (10 ns) -> us
    nph = len(PHASES[kid])
    t = t[:, :nph]
    valid = (t[:, 0] > 0)
    t = t[valid]
    t0 = t[:, 0].min()
    rel = t - t0
    out = {"blocks": int(valid.sum()), "entry_skew_us": round(float(rel[:, 0].max()), 3),
           "span_us": round(float(rel[:, nph - 1].max()), 3), "phases": {}}
    extra = tl[kid, :nblocks].double()[valid] * 10.0 / 1000.0 - t0
    for j, name in EXTRA.get(kid, {}).items():   # auxiliary stamps: median time since start
        col = extra[:, j]
        if bool((col > -t0 / 2).all()):
            out[f"at_{name}_us"] = round(float(col.median()), 3)
    for i in range(1, nph):
        d = rel[:, i] - rel[:, i - 1]
        out["phases"][PHASES[kid][i]] = {"med_delta_us": round(float(d.median()), 3),
                                         "max_delta_us": round(float(d.max()), 3),
                                         "max_since_start_us": round(float(rel[:, i].max()), 3)}
    return out, float(t0), float(t[:, nph - 1].max())


def main():
    from arena_amd.data.mnist import load_mnist
    from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig
    from arena_amd.ops import _ext
    ext = _ext.load()
    if not hasattr(ext, "timeline_read"):
        raise SystemExit("extension built without ARENA_TIMELINE=1")
    data = load_mnist()
    tr = FusedMLPTrainer(MLPConfig(), data.train_images, data.train_labels, device="cuda")
    tr.enable_graphs(60)
    tr.train_steps(600)
    torch.cuda.synchronize()
    ext.timeline_read(True)
    tr.train_steps(60)
    torch.cuda.synchronize()
    tl = ext.timeline_read(False)
    fwd, f0, f1 = analyse(tl, 0, 32 * 7)
    wg, w0, w1 = analyse(tl, 1, 424)
    res = {"fwd": fwd, "wgrad": wg, "fwd_end_to_wgrad_start_us": round(w0 - f1, 3),
           "step_span_us": round(w1 - f0, 3)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
