"""PS/worker MNIST -- the workload of the reference's distributed TFJob demos.

Equivalent of the TF dist-mnist image (docs/userguide/3-tfjob-distributed.md,
4-tfjob-distributed-data.md:168-187): variables live on the parameter servers, workers compute
gradients and push them; the cluster layout comes from TF_CONFIG / MX_CLUSTER_SPEC, which
``arena submit tfjob`` injects into every task.

    arena submit tfjob --name dist --ps 1 --workers 2 --gpus 1 \\
        "python -m arena_amd.examples.mnist_ps --max_steps 1000"

* ``ps`` tasks run the native parameter server (csrc/runtime/ps_server.cpp) on their port;
* ``worker`` tasks run forward+backward with the fused HIP kernels (one launch pair per step)
  into a flat gradient, then one PUSHPULL round trip per PS shard returns fresh parameters.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

from .common import default_log_dir, pick_device, share_cpu_threads


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--max_steps", type=int, default=1000, help="global updates to run")
    ap.add_argument("--learning_rate", type=float, default=0.001)
    ap.add_argument("--optimizer", choices=["adam", "sgd"], default="adam")
    ap.add_argument("--dropout", type=float, default=0.9)
    ap.add_argument("--batch_size", type=int, default=100)
    ap.add_argument("--hidden", type=int, default=500)
    ap.add_argument("--sync_replicas", action="store_true",
                    help="average one gradient per worker per update (default: async)")
    ap.add_argument("--data_dir", default=os.environ.get("ARENA_MNIST_DIR", ""))
    ap.add_argument("--log_dir", default="")
    ap.add_argument("--eval_every", type=int, default=10)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--n_train", type=int, default=60000)
    return ap.parse_args(argv)


def run_ps(args, spec) -> int:
    from ..parallel.ps import run_server
    port = int(spec.ps[spec.task_index].rsplit(":", 1)[1])
    print(f"PS {spec.task_index}: serving shard on port {port} for {len(spec.worker)} workers",
          flush=True)
    return run_server(port, len(spec.worker), sync=args.sync_replicas, optimizer=args.optimizer,
                      lr=args.learning_rate)


def run_worker(args, spec) -> int:
    from ..data.mnist import load_mnist
    from ..models.mlp import FusedMLPTrainer, MLPConfig
    from ..parallel.ps import PSClient
    from ..tb.writer import SummaryWriter

    dev = pick_device(args.device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    else:
        local = [a for a in spec.worker if a.split(":")[0] in ("127.0.0.1", "localhost")]
        share_cpu_threads(len(local))
    widx, nw = spec.task_index, len(spec.worker)
    data = load_mnist(args.data_dir or None, n_train=args.n_train)
    cfg = MLPConfig(hidden=args.hidden, batch=args.batch_size, lr=args.learning_rate,
                    keep_prob=args.dropout, seed=0)
    # rank-sharded data like the DP path, but every worker starts from the chief's weights
    tr = FusedMLPTrainer(cfg, data.train_images, data.train_labels, device=dev, rank=widx,
                         world=1, external_update=True)
    if nw > 1:
        n_all = tr.train_x.shape[0]
        tr.shard = torch.arange(widx, n_all, nw, dtype=torch.int64, device=dev)
        tr.perm = torch.empty(tr.shard.numel(), dtype=torch.int32, device=dev)
        tr._reshuffle()
    n = tr.layout.total
    pin = dev.type == "cuda"
    host_p = torch.empty(n, dtype=torch.float32, pin_memory=pin)
    host_g = torch.empty(n, dtype=torch.float32, pin_memory=pin)
    np_p, np_g = host_p.numpy(), host_g.numpy()
    client = PSClient(spec.ps, n)
    if spec.is_chief:
        host_p.copy_(tr.P)
        client.init(np_p)
    gstep = client.pull(np_p)
    tr.P.copy_(host_p, non_blocking=pin)
    if dev.type == "cuda":
        tr.enable_graphs(1)
    te = None
    if spec.is_chief:
        te = SummaryWriter(os.path.join(default_log_dir(args.log_dir), "test"))
    print(f"Worker {widx}: device={dev} ps={len(spec.ps)} workers={nw} "
          f"mode={'sync' if args.sync_replicas else 'async'} data={data.source}", flush=True)
    t0, local, last_eval = time.time(), 0, -1
    while gstep < args.max_steps:
        tr.train_steps(1)                      # fwd + bwd -> tr.G (device)
        host_g.copy_(tr.G, non_blocking=pin)
        if pin:
            torch.cuda.current_stream().synchronize()
        gstep = client.push_pull(np_g, np_p)
        tr.P.copy_(host_p, non_blocking=pin)
        local += 1
        if spec.is_chief and gstep // args.eval_every != last_eval:
            last_eval = gstep // args.eval_every
            loss, acc = tr.evaluate(data.test_images, data.test_labels)
            te.add_scalars({"accuracy": acc, "cross_entropy": loss}, gstep)
            print(f"Accuracy at step {gstep}: {acc:.4f}", flush=True)
        if local % 100 == 0:
            print(f"Worker {widx}: training step {local} done (global step: {gstep})", flush=True)
    dt = time.time() - t0
    loss, acc = tr.evaluate(data.test_images, data.test_labels)
    print(f"Worker {widx}: done, {local} local steps in {dt:.2f}s "
          f"({local * cfg.batch / max(dt, 1e-9):.0f} samples/s); test accuracy {acc:.4f}",
          flush=True)
    if te is not None:
        te.close()
    client.done()
    return 0


def main(argv=None) -> int:
    args = parse(argv)
    from ..parallel.ps import ClusterSpec
    spec = ClusterSpec.from_env()
    if not spec.ps:
        print("mnist_ps: no 'ps' tasks in TF_CONFIG/MX_CLUSTER_SPEC", file=sys.stderr)
        return 2
    if spec.task_type == "ps":
        return run_ps(args, spec)
    return run_worker(args, spec)


if __name__ == "__main__":
    sys.exit(main())
