"""MNIST with a plain ``torch.nn`` model and the Horovod-style API (arena_amd.parallel.hvd).

The shape of the reference's Horovod demo (charts/tf-horovod/README.md:66-69, hvd-distribute.sh):
``hvd.init()``, pin one GPU per rank by local rank, broadcast the initial variables from rank 0,
wrap the optimizer in ``DistributedOptimizer`` (bucketed, backward-overlapped gradient
all-reduce). Layers are the fused HIP ``FusedLinear`` modules, the loss is the fused
softmax-xent kernel; on CPU the same code runs on the reference ops over gloo.

    arena submit mpijob --name hvd --workers 2 --gpus 1 "python -m arena_amd.examples.mnist_hvd"
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
from torch import nn

from .common import pick_device, share_cpu_threads


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--max_steps", type=int, default=1000)
    ap.add_argument("--learning_rate", type=float, default=0.001)
    ap.add_argument("--batch_size", type=int, default=100)
    ap.add_argument("--dropout", type=float, default=0.9)
    ap.add_argument("--data_dir", default=os.environ.get("ARENA_MNIST_DIR", ""))
    ap.add_argument("--bucket_mb", type=float, default=32.0)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--n_train", type=int, default=60000)
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse(argv)
    from ..data.mnist import load_mnist
    from ..ops import FusedLinear, fused_cross_entropy
    from ..parallel import hvd

    dev = pick_device(args.device)
    hvd.init("nccl" if dev.type == "cuda" else "gloo")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    else:
        share_cpu_threads(int(os.environ.get("LOCAL_WORLD_SIZE", hvd.size())))
    torch.manual_seed(1234 + hvd.rank())        # different init per rank: broadcast fixes it
    model = nn.Sequential(FusedLinear(784, 500, activation="relu", keep_prob=args.dropout,
                                      seed=hvd.rank()),
                          FusedLinear(500, 10, activation="none")).to(dev)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    opt = torch.optim.Adam(model.parameters(), lr=args.learning_rate)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(),
                                   bucket_mb=args.bucket_mb)
    data = load_mnist(args.data_dir or None, n_train=args.n_train).to(dev)
    x_all = data.train_images[hvd.rank()::hvd.size()]
    y_all = data.train_labels[hvd.rank()::hvd.size()]
    g = torch.Generator(device=dev).manual_seed(hvd.rank())
    t0 = time.time()
    for step in range(args.max_steps):
        idx = torch.randint(0, x_all.shape[0], (args.batch_size,), device=dev, generator=g)
        x = x_all[idx].float().mul_(1.0 / 255.0)
        loss = fused_cross_entropy(model(x), y_all[idx].long())
        opt.zero_grad()
        loss.backward()
        opt.step()
        if step % 100 == 0 or step == args.max_steps - 1:
            l_avg = hvd.allreduce(loss.detach().reshape(1))
            if hvd.rank() == 0:
                print(f"step {step}: loss {float(l_avg):.4f}", flush=True)
    model.eval()
    with torch.no_grad():
        xt = data.test_images.float().mul_(1.0 / 255.0)
        pred = model(xt).argmax(1)
        acc = (pred == data.test_labels.long()).float().mean().reshape(1)
    acc = hvd.allreduce(acc)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    if hvd.rank() == 0:
        print(f"Final test accuracy: {float(acc):.4f}; "
              f"{args.max_steps * args.batch_size * hvd.size() / dt:.0f} samples/s over "
              f"{hvd.size()} ranks", flush=True)
    hvd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
