#!/usr/bin/env python3
"""Rehearse the data-parallel MNIST step on ONE GPU: W ranks share GPU 0, gradients go through the
xGMI collective's hipIpc protocol (gloo process group for setup only; RCCL refuses two ranks on
one device). The ranks time-share the GPU's CUs, so ms/step is an upper bound of what W GPUs do;
it checks that the DP path (graph-captured fused reduce-scatter/Adam/all-gather) runs end to end.

    python tools/dp_same_gpu.py --world 2 --steps 600 --warmup 60
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(rank, world, port, steps, warmup, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    from arena_amd.data.mnist import load_mnist
    from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig
    data = load_mnist()
    tr = FusedMLPTrainer(MLPConfig(), data.train_images, data.train_labels, device="cuda",
                         process_group=dist.group.WORLD, rank=rank, world=world, comm="xgmi")
    spg = tr.pick_steps_per_graph()
    tr.enable_graphs(spg)
    tr.train_steps(warmup)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    tr.train_steps(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tr.xgmi.check()
    loss, acc = tr.recent_metrics(100)
    tl, ta = tr.evaluate(data.test_images, data.test_labels)
    q.put((rank, dt, tr.graph_mode, spg, loss, acc, ta))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=60)
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, a.world, port, a.steps, a.warmup, q))
          for r in range(a.world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in range(a.world))
    for p in ps:
        p.join(60)
    dt = max(r[1] for r in res)
    print(json.dumps({"world": a.world, "same_gpu": True, "steps": a.steps,
                      "ms_per_step": round(dt / a.steps * 1e3, 5),
                      "samples_per_s": round(a.world * 100 * a.steps / dt, 1),
                      "graph_mode": res[0][2], "steps_per_graph": res[0][3],
                      "train_loss_last100": round(res[0][4], 5), "train_acc_last100": round(res[0][5], 4),
                      "test_acc": [round(r[6], 4) for r in res]}), flush=True)


if __name__ == "__main__":
    main()
