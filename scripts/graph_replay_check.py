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
    ap.add_argument("--no_benchmark", action="store_true", help="cudnn.benchmark off (no MIOpen find)")
    ap.add_argument("--warm_replays", type=int, default=1,
                    help="(--ab) replays of each graph right after its capture")
    ap.add_argument("--reset_mode", action="store_true",
                    help="(--ab) conv.set_mode(None) after the captures, as cnn_ab does")
    a = ap.parse_args()
    from arena_amd.ops import conv
    from arena_amd.examples import cnn_bench
    from arena_amd.parallel import hvd
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = not a.no_benchmark
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
    def nonfinite(v):
        """(#params with non-finite weights, #with non-finite grads, #non-finite BN running
        stats) of a model."""
        nw = ng = nb = 0
        for p in v["model"].parameters():
            nw += int(not bool(torch.isfinite(p.detach().float()).all()))
            ng += int(p.grad is not None and not bool(torch.isfinite(p.grad.float()).all()))
        for b in v["model"].buffers():
            if b.is_floating_point():
                nb += int(not bool(torch.isfinite(b).all()))
        return nw, ng, nb

    if a.ab:
        vs = []
        for m in (m1, m2):
            v = make(m)
            print(f"{m}: after capture nonfinite {nonfinite(v)}", flush=True)
            for _ in range(a.warm_replays):
                v["g"].replay()
                torch.cuda.synchronize()
                print(f"{m}: after replay nonfinite {nonfinite(v)} loss {float(v['loss']):.4f}",
                      flush=True)
            if vs:
                print(f"v1 after v2 built: nonfinite {nonfinite(vs[0])}", flush=True)
            vs.append(v)
        for k in range(3):
            vs[0]["g"].replay()
            torch.cuda.synchronize()
            print(f"v1 replay {k}: nonfinite {nonfinite(vs[0])} loss {float(vs[0]['loss']):.4f}",
                  flush=True)
        if a.reset_mode:
            conv.set_mode(None)
        for r in range(4):
            line = []
            for i, v in enumerate(vs):
                w0 = v["model"].fc.weight.detach().float().clone()
                c0 = v["model"].layers[0].conv1.weight.detach().float().clone()
                torch.cuda.synchronize()
                for _ in range(10):
                    v["g"].replay()
                    if a.sync_each:
                        torch.cuda.synchronize()
                torch.cuda.synchronize()
                dfc = float((v["model"].fc.weight.detach().float() - w0).abs().max())
                dc1 = float((v["model"].layers[0].conv1.weight.detach().float() - c0).abs().max())
                line.append(f"v{i + 1} {float(v['loss']):.4f} dfc {dfc:.2e} dconv {dc1:.2e}")
            print(f"round {r}: " + "  ".join(line), flush=True)
        # where are the non-finite values? (weights, fp32 masters, momentum, gradients)
        for i, v in enumerate(vs):
            bad = []
            for n, p in v["model"].named_parameters():
                nf = int((~torch.isfinite(p.detach().float())).sum())
                ng = int((~torch.isfinite(p.grad.float())).sum()) if p.grad is not None else -1
                if nf or ng > 0:
                    bad.append(f"{n}: w {nf}/{p.numel()} g {ng}")
            for o in getattr(v["opt"], "opts", [v["opt"]]):
                if hasattr(o, "master"):
                    for j, (pp, off) in enumerate(zip(o.params, o.offsets)):
                        m = o.master[off:off + pp.numel()]
                        mo = o.mom[off:off + pp.numel()]
                        nm, nmo = int((~torch.isfinite(m)).sum()), int((~torch.isfinite(mo)).sum())
                        if nm or nmo:
                            bad.append(f"master[{j}] shape {tuple(pp.shape)}: {nm} mom {nmo}")
            print(f"v{i + 1} non-finite: {bad[:12]} ({len(bad)} entries)", flush=True)
        # one eager step on each: does the model itself still train outside its graph?
        for i, v in enumerate(vs):
            l0 = float(cnn_bench.train_step(v["model"], v["opt"], v["x"], v["y"], torch.bfloat16))
            l1 = float(cnn_bench.train_step(v["model"], v["opt"], v["x"], v["y"], torch.bfloat16))
            print(f"v{i + 1} eager steps: {l0:.4f} -> {l1:.4f}", flush=True)
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
