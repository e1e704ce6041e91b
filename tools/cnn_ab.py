#!/usr/bin/env python3
"""In-process A/B of ResNet training-step variants on one GPU (interleaved graph replays).

Builds one model + optimizer + synthetic batch per variant (same seed), warms each up eagerly
(conv autotuning happens there), captures each whole step as a hipGraph, then alternates
``--chunk`` timed replays of each variant for ``--rounds`` rounds, so clock/thermal drift hits
every variant alike (cdna_hip_programming.md §5.4 rule 24). Variants are conv modes
(ARENA_CONV values), optionally suffixed ``:async`` (weight gradients on a side stream) and/or
``:link`` / ``:nolink`` (BN-backward partials in the dgrad epilogues; on by default) and/or
``:laccP<n>`` (their fp64-sum form up to n tile-channel pairs), ``:nohalowide`` (no 8-wave halo forms), ``:torchstem`` (the stem's
input/weight casts and weight transform as torch ops) and/or ``:nomask`` (the last BN writes
dy * mask for the residual join instead of parking (dy, bits)) and/or ``:finP<n>`` (at most n
level-1 blocks per channel group in the BN finalize kernels) and/or ``:redG<b>x<r>`` (BN reduction grid) and/or ``:accP<n>`` (conv-epilogue
BN statistics as fp64 sums up to n tile-channel pairs) and/or ``:finbwd0`` (BN backward sums
from the pool plus a finalize launch) and/or
``:nostempool`` (stem BN and max pool unfused) and/or ``:noxsel`` (stem backward sums per pixel
over x instead of from the saved argmax inputs) and/or ``:noressums`` (down_bn's backward sums
by its own reduction, not in bn3's dx pass) and/or ``:downfirst`` (downsample shortcut built
before the main path: its strided dgrad completes the join, no BN link there) and/or ``:ebk<n>`` (at most n blocks per BN apply pass), ``:dxb<n>`` (per dx pass), ``:noslice`` (flat
grids for C > 256 instead of 256-channel slices),
joined with ``+``.
Prints one JSON line per variant: median / min ms per step, images/s.

    python tools/cnn_ab.py --modes miopen,auto --batch 128 > gpurun_out/cnn_ab.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from arena_amd.examples import cnn_bench  # noqa: E402
from arena_amd.ops import conv  # noqa: E402
from arena_amd.parallel import hvd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="miopen,auto")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = True
    hvd.init("gloo")
    args = cnn_bench.parse(["--model", a.model, "--batch_size", str(a.batch)])
    variants = {}
    conv_acc_default = conv._ACC_MAX_PAIRS
    link_acc_default = conv._LINK_ACC_MAX_PAIRS
    for i, name in enumerate(a.modes.split(",")):
        mode, _, opt_s = name.partition(":")
        conv.set_mode(mode)
        conv.set_async_wgrad("async" in opt_s.split("+"))
        opts = opt_s.split("+")
        # BN-backward partials in the dgrad epilogue: on by default, "nolink" turns them off
        conv.set_bn_links("nolink" not in opts if "link" not in opts else True)
        conv.set_stem_fused("torchstem" not in opt_s.split("+"))
        conv.set_halo_wide("nohalowide" not in opt_s.split("+"))   # the 8-wave halo forms
        conv.set_masked_join("nomask" not in opt_s.split("+"))
        # finP<n>: at most n level-1 blocks per channel group in the BN finalize kernels (the
        # grid is baked into this variant's captured graph)
        finp = [int(o[4:]) for o in opt_s.split("+") if o.startswith("finP")]
        from arena_amd.ops import _ext as _e
        _e.load().bn_set_fin_max_blocks(finp[0] if finp else 64)
        _e.load().bn_set_nt(0 if "bnnt0" in opt_s.split("+") else 1)   # BN non-temporal loads
        # redG<blocks>x<rounds>: BN reduction grid (at most <blocks> blocks, >= <rounds> row rounds
        # per block); default 512x8
        redg = [o[4:].split("x") for o in opt_s.split("+") if o.startswith("redG")]
        _e.load().bn_set_reduce_geometry(*(map(int, redg[0]) if redg else (512, 8)))
        # pqm<n>: stem-pool quad reduction grid at n x the usual reduction grid (default 2)
        pqm = [int(o[3:]) for o in opt_s.split("+") if o.startswith("pqm")]
        _e.load().bn_set_pool_quad_mult(pqm[0] if pqm else 2)
        # accP<n>: conv-epilogue BN statistics as fp64 sums up to n (tile, channel) pairs
        accp = [int(o[4:]) for o in opt_s.split("+") if o.startswith("accP")]
        conv.set_acc_max_pairs(accp[0] if accp else conv_acc_default)
        # laccP<n>: the same for the linked dgrad epilogue's BN-backward sums
        laccp = [int(o[5:]) for o in opt_s.split("+") if o.startswith("laccP")]
        conv.set_link_acc_max_pairs(laccp[0] if laccp else link_acc_default)
        # finbwd0: BN backward sums from the pool + a finalize launch (not the layer's own set)
        from arena_amd.ops import batchnorm as _bn
        _bn.set_fin_bwd("finbwd0" not in opt_s.split("+"))
        # nostempool: stem BN apply + max pool kernels instead of the fused pass
        _bn.set_stem_pool_fused("nostempool" not in opt_s.split("+"))
        _bn.set_stem_xsel("noxsel" not in opt_s.split("+"))   # stem sums per pixel over x
        _bn.set_res_sums("noressums" not in opt_s.split("+"))   # down_bn reduces itself
        from arena_amd.models import resnet as _rn
        _rn.set_downsample_last("downfirst" not in opt_s.split("+"))   # shortcut built first
        # ebk<n>: at most n blocks per BN apply pass (grid baked into the captured graph)
        ebk = [int(o[3:]) for o in opt_s.split("+") if o.startswith("ebk")]
        _e.load().bn_set_elem_max_blocks(ebk[0] if ebk else 1024)
        # dxb<n>: at most n blocks per BN dx pass; noslice: flat grids for C > 256 (no channel
        # slices in the apply / dx passes)
        dxb = [int(o[3:]) for o in opt_s.split("+") if o.startswith("dxb")]
        _e.load().bn_set_dx_max_blocks(dxb[0] if dxb else 1024)
        _e.load().bn_set_slice(0 if "noslice" in opt_s.split("+") else 1)
        # st1p: conv-epilogue BN statistics in one pass (the launch args bake the switch)
        _e.load().conv_set_stats_one_pass("st1p" in opt_s.split("+"))
        model, opt, x, y = cnn_bench.build(args, dev, 1)
        for _ in range(a.warmup):
            cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
        torch.cuda.synchronize()
        g, loss = cnn_bench.capture_step(model, opt, x, y, torch.bfloat16)
        g.replay()
        torch.cuda.synchronize()
        # the graph holds raw pointers into this model's parameters, optimizer state and batch:
        # keep them alive (rebinding the names would free them into the next variant's use)
        variants[f"{name}" if name not in variants else f"{name}#{i}"] = (g, loss,
                                                                          (model, opt, x, y))
        print(f"[ab] {name}: captured, loss {float(loss):.4f}", file=sys.stderr, flush=True)
    conv.set_mode(None)
    times = {m: [] for m in variants}
    for r in range(a.rounds):
        for m, (g, _, _) in variants.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.chunk):
                g.replay()
            torch.cuda.synchronize()
            times[m].append((time.perf_counter() - t0) / a.chunk * 1e3)
        print(f"[ab] round {r}: " + " ".join(
            f"{m}={times[m][-1]:.3f}ms/loss {float(variants[m][1]):.4f}" for m in times),
            file=sys.stderr, flush=True)
    for m, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"variant": m, "model": a.model, "batch": a.batch,
                          "ms_per_step_median": round(med, 3), "ms_per_step_min": round(min(ts), 3),
                          "images_per_s": round(a.batch / med * 1e3, 1),
                          "loss": round(float(variants[m][1]), 4), "rounds": a.rounds,
                          "chunk": a.chunk}), flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
