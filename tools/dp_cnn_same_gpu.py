#!/usr/bin/env python3
"""Rehearse the data-parallel ResNet step on ONE GPU: W ranks share GPU 0, gloo process group for
setup (RCCL refuses two ranks on one device). Default: bf16 weights with the sharded xGMI SGD
(arena_amd.parallel.zero); --master_weights off: fp32 weights + hvd.DistributedOptimizer.

What it checks:

* gradient buckets (12 MB default, in model order: each bucket's bf16 conv weights travel with
  the fp32 BN/bias parameters of the same blocks; the input-side bucket is a quarter size)
  through the registered xGMI staging buffer, issued on the comm stream while backward is
  still running;
* fused BN kernels under bf16 autocast in every rank;
* that all replicas stay bit-identical after the steps (same averaged gradient everywhere).

The ranks time-share the CUs, so images/s is a lower bound of what W GPUs do; the allreduce
runs over same-device hipIpc mappings (protocol cost, not xGMI bandwidth).

    python tools/dp_cnn_same_gpu.py --world 2 --model resnet50 --batch_size 32 --steps 20
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
import types

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def trace_overlap(model, opt, x, y, path):
    """One eager DP step with HIP events: a start event on the main stream before the forward,
    one on the comm stream right after every bucket's optimizer kernel (ShardedMasterSGD:
    ``xgmi_sgd_*``), and one on the main stream when backward has issued its last kernel. A bucket
    whose completion time is earlier than the backward's end ran concurrently with backward.
    Writes the per-bucket times (ms after the forward's start) to ``path``."""
    from arena_amd.examples import cnn_bench
    from arena_amd.parallel.zero import ShardedMasterSGD
    assert isinstance(opt, ShardedMasterSGD)
    marks = []
    orig = opt._launch

    def launch(b):
        orig(b)
        e = torch.cuda.Event(enable_timing=True)
        e.record(opt.stream)
        marks.append((len(marks), str(b.dtype).replace("torch.", ""),
                      {str(r.dtype).replace("torch.", ""): r.end - r.start for r in b.ranges}, e))

    opt._launch = launch
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    bwd_end = torch.cuda.Event(enable_timing=True)
    step_end = torch.cuda.Event(enable_timing=True)
    start.record()
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        loss = torch.nn.functional.cross_entropy(model(x), y)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    bwd_end.record()
    opt.step()
    step_end.record()
    torch.cuda.synchronize()
    opt._launch = orig
    t_bwd = start.elapsed_time(bwd_end)
    rows = [{"bucket": i, "dtype": dt, "elems": n, "done_ms": round(start.elapsed_time(e), 3)}
            for i, dt, n, e in marks]
    with open(path, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
        f.write(json.dumps({"backward_end_ms": round(t_bwd, 3),
                            "step_end_ms": round(start.elapsed_time(step_end), 3)}) + "\n")
    return {"buckets": len(rows), "finished_before_backward_end":
            sum(1 for r in rows if r["done_ms"] < t_bwd),
            "backward_end_ms": round(t_bwd, 3),
            "bucket_done_ms": [r["done_ms"] for r in rows]}


def rank_main(rank, world, port, a, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from arena_amd.examples import cnn_bench
    from arena_amd.parallel import hvd
    hvd.init()
    torch.backends.cudnn.benchmark = True
    args = types.SimpleNamespace(model=a.model, batch_size=a.batch_size, image_size=a.image_size,
                                 num_classes=1000, width=64, learning_rate=0.1, momentum=0.9,
                                 weight_decay=4e-5, bucket_mb=a.bucket_mb, comm="xgmi",
                                 data_format="NHWC", dtype="bf16", master_weights=a.master_weights)
    model, opt, x, y = cnn_bench.build(args, torch.device("cuda", 0), world)
    name = cnn_bench.comm_name(opt)
    assert name.startswith("xgmi"), name
    for i in range(a.warmup):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
        torch.cuda.synchronize()
        if rank == 0:  # the first steps include the solver search: show progress
            print(f"warmup {i + 1}/{a.warmup}", file=sys.stderr, flush=True)
    overlap = None
    if a.trace:   # a collective step: every rank runs it, rank 0 under the profiler
        if rank == 0:
            overlap = trace_overlap(model, opt, x, y, a.trace)
        else:
            cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
            torch.cuda.synchronize()
        dist.barrier()
    graph = None
    if a.graph:  # the whole DP step (bucket hooks + xGMI kernels on the comm stream) as a hipGraph
        graph, g_loss = cnn_bench.capture_step(model, opt, x, y, torch.bfloat16)
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if graph is not None:
            graph.replay()
            loss = g_loss
        else:
            loss = cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for c in cnn_bench.comms_of(opt):
        if c is not None:
            c.check()
    flat = torch.cat([p.detach().double().reshape(-1) for p in model.parameters()])
    digest = float(flat.sum().item()), float(flat.abs().sum().item())
    q.put((rank, dt, float(loss), digest, len(opt.buckets), name, overlap))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--image_size", type=int, default=224)
    ap.add_argument("--bucket_mb", type=float, default=12.0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--graph", type=int, default=0, help="1: replay the whole step as a hipGraph")
    ap.add_argument("--trace", default="", help="rank 0 times one eager step with HIP events "
                    "(per-bucket optimizer-kernel completion vs the end of backward), writes them "
                    "here and reports how many buckets finished while backward was running")
    ap.add_argument("--master_weights", choices=["auto", "on", "off"], default="auto",
                    help="auto/on: bf16 weights + ShardedMasterSGD (xGMI reduce-scatter / SGD / "
                         "all-gather); off: fp32 weights + DistributedOptimizer buckets")
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, a.world, port, a, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=900) for _ in range(a.world))
    for p in ps:
        p.join(60)
    dt = max(r[1] for r in res)
    same = all(r[3] == res[0][3] for r in res)
    print(json.dumps({"world": a.world, "same_gpu": True, "model": a.model,
                      "batch_per_rank": a.batch_size, "steps": a.steps,
                      "exec": "hipgraph" if a.graph else "eager", "buckets": res[0][4],
                      "comm": res[0][5],
                      "images_per_s_all_ranks": round(a.world * a.batch_size * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1e3, 3), "final_loss": round(res[0][2], 4),
                      "replicas_identical": same, "overlap": res[0][6]}), flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
