"""MNIST MLP trainer -- the workload of the reference's standalone and Horovod demos.

Equivalent of the ``mnist_with_summaries`` image the reference runs
(docs/userguide/1-tfjob-standalone.md:178-186: 784-500-10 MLP, ReLU, dropout keep 0.9,
softmax cross-entropy, Adam 1e-3, batch 100; prints ``Accuracy at step N: acc`` every 10 steps
and ``Adding run metadata for N`` at N % 100 == 99; TensorBoard summaries under --log_dir).

    python -m arena_amd.examples.mnist --max_steps 1000 [--data_dir DIR] [--log_dir DIR]

With ``WORLD_SIZE > 1`` (an ``arena submit mpijob`` rank, or torchrun) it trains data-parallel:
per-rank batch 100 on a rank-sharded dataset, flat-gradient all-reduce (RCCL over xGMI on
MI355X, gloo on CPU) inside the captured step, Adam on every rank.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

from .common import (default_log_dir, load_checkpoint, pick_device, save_checkpoint,
                     share_cpu_threads)


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--max_steps", type=int, default=1000)
    ap.add_argument("--learning_rate", type=float, default=0.001)
    ap.add_argument("--dropout", type=float, default=0.9, help="keep probability")
    ap.add_argument("--batch_size", type=int, default=100, help="per-rank batch")
    ap.add_argument("--hidden", type=int, default=500)
    ap.add_argument("--data_dir", default=os.environ.get("ARENA_MNIST_DIR", ""),
                    help="directory with the MNIST IDX files; synthetic MNIST when absent")
    ap.add_argument("--log_dir", default="", help="TensorBoard dir (default $ARENA_TRAINING_LOGDIR)")
    ap.add_argument("--eval_every", type=int, default=10)
    ap.add_argument("--checkpoint", default="", help="save here at the end; resume if present")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--n_train", type=int, default=60000)
    ap.add_argument("--fake_data", action="store_true", help="accepted for compatibility")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse(argv)
    from ..data.mnist import load_mnist
    from ..models.mlp import FusedMLPTrainer, MLPConfig
    from ..parallel import hvd
    from ..tb.writer import SummaryWriter

    world = int(os.environ.get("WORLD_SIZE", "1"))
    dev = pick_device(args.device)
    pg = None
    if world > 1:
        pg = hvd.init("nccl" if dev.type == "cuda" else "gloo")
    rank = hvd.rank()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    else:
        share_cpu_threads(int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    data = load_mnist(args.data_dir or None, n_train=args.n_train)
    cfg = MLPConfig(hidden=args.hidden, batch=args.batch_size, lr=args.learning_rate,
                    keep_prob=args.dropout, seed=args.seed)
    tr = FusedMLPTrainer(cfg, data.train_images, data.train_labels, device=dev,
                         process_group=pg, rank=rank, world=world)
    start = 0
    ck = load_checkpoint(args.checkpoint)
    if ck is not None:
        tr.load_state_dict(ck)
        start = int(ck["step"])
        if rank == 0:
            print(f"Restored checkpoint {args.checkpoint} at step {start}", flush=True)
    log_dir = default_log_dir(args.log_dir)
    tw = te = None
    if rank == 0:
        tw = SummaryWriter(os.path.join(log_dir, "train"))
        te = SummaryWriter(os.path.join(log_dir, "test"))
        print(f"arena_amd mnist: device={dev} world={world} data={data.source} "
              f"steps={args.max_steps}", flush=True)
    every = max(1, args.eval_every)
    if dev.type == "cuda":
        # one hipGraph per eval interval (divides the epoch length, so no reshuffle inside)
        spe = tr.steps_per_epoch
        tr.enable_graphs(every if spe % every == 0 else tr.pick_steps_per_graph(every))
    t0 = time.time()
    i = start
    while i < args.max_steps:
        if (i % every == 0) and rank == 0:
            loss, acc = tr.evaluate(data.test_images, data.test_labels)
            te.add_scalars({"accuracy": acc, "cross_entropy": loss}, i)
            print(f"Accuracy at step {i}: {acc:.4f}", flush=True)
        n = min(every - i % every, args.max_steps - i)
        tr.train_steps(n)
        i += n
        if i % 100 == 0 or i == args.max_steps:
            tl, ta = tr.recent_metrics(min(100, i - start))
            if rank == 0:
                tw.add_scalars({"accuracy": ta, "cross_entropy": tl}, i - 1)
                if (i - 1) % 100 == 99:
                    print(f"Adding run metadata for {i - 1}", flush=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    loss, acc = tr.evaluate(data.test_images, data.test_labels)
    if rank == 0:
        te.add_scalars({"accuracy": acc, "cross_entropy": loss}, args.max_steps)
        tw.close()
        te.close()
        done = args.max_steps - start
        print(f"Final test accuracy: {acc:.4f} (loss {loss:.4f}) after {args.max_steps} steps; "
              f"{done * cfg.batch * world / max(dt, 1e-9):.0f} samples/s", flush=True)
        if args.checkpoint:
            save_checkpoint(args.checkpoint, tr.state_dict())
    if world > 1:
        hvd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
