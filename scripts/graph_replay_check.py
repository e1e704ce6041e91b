#!/usr/bin/env python3
"""Does a captured ResNet training step keep training when replayed, before and after a second
model's step is captured in the same process? Prints the loss per replay and the parameter /
BatchNorm-statistics movement, so a replay that silently stops updating shows up.

    python scripts/graph_replay_check.py [--model resnet50] [--batch 32]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--replays", type=int, default=6)
    ap.add_argument("--modes", default="auto,auto", help="conv mode per variant (as cnn_ab)")
    ap.add_argument("--ab", action="store_true",
                    help="cnn_ab's exact sequence: both captured first, then interleaved chunks "
                         "of back-to-back replays")
    ap.add_argument("--sync_each", action="store_true", help="(--ab) sync after every replay")
    ap.add_argument("--reset_mode", action="store_true",
                    help="(--ab) conv.set_mode(None) after the captures, as cnn_ab does")
    a = ap.parse_args()
    from arena_amd.ops import conv
    from arena_amd.examples import cnn_bench
    from arena_amd.parallel import hvd
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = True
    hvd.init("gloo")
    args = cnn_bench.parse(["--model", a.model, "--batch_size", str(a.batch)])

    def make(mode):
        conv.set_mode(mode)
        model, opt, x, y = cnn_bench.build(args, dev, 1)
        for _ in range(4):
            cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
        torch.cuda.synchronize()
        g, loss = cnn_bench.capture_step(model, opt, x, y, torch.bfloat16)
        return dict(model=model, opt=opt, x=x, y=y, g=g, loss=loss)

    def replay(v, tag):
        m = v["model"]
        w0 = m.fc.weight.detach().float().clone()
        rm0 = m.stem[1].running_mean.clone()
        losses = []
        for _ in range(a.replays):
            v["g"].replay()
            torch.cuda.synchronize()
            losses.append(round(float(v["loss"]), 4))
        dw = float((m.fc.weight.detach().float() - w0).abs().max())
        drm = float((m.stem[1].running_mean - rm0).abs().max())
        print(f"{tag}: losses {losses} |dW_fc| {dw:.3e} |d running_mean| {drm:.3e}", flush=True)

    m1, m2 = a.modes.split(",")
    if a.ab:
        vs = []
        for m in (m1, m2):
            v = make(m)
            v["g"].replay()
            torch.cuda.synchronize()
            vs.append(v)
        if a.reset_mode:
            conv.set_mode(None)
        for r in range(4):
            line = []
            for i, v in enumerate(vs):
                torch.cuda.synchronize()
                for _ in range(10):
                    v["g"].replay()
                    if a.sync_each:
                        torch.cuda.synchronize()
                torch.cuda.synchronize()
                line.append(f"v{i + 1} {float(v['loss']):.4f}")
            print(f"round {r}: " + "  ".join(line), flush=True)
        hvd.shutdown()
        return
    v1 = make(m1)
    replay(v1, "v1 alone")
    v2 = make(m2)
    replay(v1, "v1 after v2 captured")
    replay(v2, "v2")
    replay(v1, "v1 after v2 replayed")
    hvd.shutdown()


if __name__ == "__main__":
    main()
