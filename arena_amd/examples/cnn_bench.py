"""Synthetic-ImageNet CNN training benchmark with the Horovod-style API (tf_cnn_benchmarks shape).

The reference's MPI demo runs the Horovod TF image's ``hvd-distribute.sh``
(charts/tf-horovod/README.md:66-69). That image benchmarks the ResNet family on synthetic data
with Horovod allreduce. The script is not in the reference repo, so exact flags are unpinned.
This is the same workload, built for MI355X:

* ResNet v1.5 (``arena_amd.models.resnet``), NHWC (``channels_last``), bf16 autocast on the MFMA
  conv/GEMM paths, fp32 master weights;
* momentum SGD with weight decay, as in tf_cnn_benchmarks;
* one process per GPU: ``hvd.DistributedOptimizer`` buckets (RCCL or the xGMI kernel on a comm
  stream) overlap the gradient allreduce with backward;
* output lines shaped like tf_cnn_benchmarks' ``images/sec`` and ``total images/sec``.

    arena submit mpijob --name r50 --workers 8 --gpus 1 \\
        "python -m arena_amd.examples.cnn_bench --model resnet50 --batch_size 128"
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

from ..runtime import heartbeat
from .common import pick_device, share_cpu_threads


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch_size", type=int, default=128, help="per-rank batch")
    ap.add_argument("--image_size", type=int, default=224)
    ap.add_argument("--num_classes", type=int, default=1000)
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--num_batches", type=int, default=100)
    ap.add_argument("--num_warmup_batches", type=int, default=10)
    ap.add_argument("--display_every", type=int, default=10)
    ap.add_argument("--learning_rate", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight_decay", type=float, default=4e-5)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--data_format", choices=["NHWC", "NCHW"], default="NHWC")
    ap.add_argument("--bucket_mb", type=float, default=12.0,
                    help="gradient bucket size (Horovod fusion buffer). 12 MB splits ResNet-50's "
                         "51 MB of bf16 gradients into 5 buckets, so the first buckets' "
                         "collectives run while backward is still producing the rest")
    ap.add_argument("--comm", choices=["auto", "xgmi", "rccl", "hier"], default="auto",
                    help="DP gradient path: xgmi kernels (one node), rccl (flat), hier (node-level "
                         "then inter-node RCCL on 1/local_size of the bytes); auto picks")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: capture the whole training step (fwd, bwd, optimizer) in one hipGraph "
                         "and replay it (single rank; DP ranks run eagerly)")
    ap.add_argument("--master_weights", choices=["auto", "on", "off"], default="auto",
                    help="bf16 conv/linear weights with fp32 master copies updated by one "
                         "multi-tensor HIP kernel; with several ranks by the sharded xGMI "
                         "reduce-scatter/SGD/all-gather kernel (auto: on for bf16 GPU runs, "
                         "data parallel only when the xGMI collective is usable)")
    ap.add_argument("--async_wgrad", choices=["on", "off"], default="off",
                    help="conv weight gradients on a second HIP stream, concurrent with the "
                         "backward-data/BatchNorm chain (single rank; measured slower on "
                         "ResNet-50 bs128: 16.18 vs 15.49 ms/step, docs/perf.md)")
    ap.add_argument("--verify_every", type=int, default=0,
                    help="data parallel: every K steps check that all replicas hold bit-identical "
                         "parameters (and that no xGMI barrier timed out); abort if not. The "
                         "replicas are always verified once at the end")
    ap.add_argument("--json", action="store_true", help="print one JSON summary line at the end")
    return ap.parse_args(argv)


def build(args, dev, world):
    """Model, optimizer (wrapped for DP) and one synthetic batch, ready to step."""
    from ..models.resnet import resnet
    from ..parallel import hvd
    torch.manual_seed(1234)
    model = resnet(args.model, num_classes=args.num_classes, width=args.width).to(dev)
    nhwc = dev.type == "cuda" and args.data_format == "NHWC"
    if nhwc:
        model = model.to(memory_format=torch.channels_last)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    decay, no_decay = [], []
    for n, p in model.named_parameters():
        (no_decay if p.ndim <= 1 else decay).append(p)   # no decay on BN / bias
    mw = getattr(args, "master_weights", "auto")
    master = mw == "on" or (
        mw == "auto" and dev.type == "cuda"
        and getattr(args, "dtype", "bf16") == "bf16" and all(p.numel() % 4 == 0 for p in decay))
    if master and (getattr(args, "dtype", "bf16") != "bf16" or dev.type != "cuda"):
        raise SystemExit("--master_weights on needs --dtype bf16 on a GPU (the weights become "
                         "bf16 and the update runs in the HIP multi-tensor kernel)")
    opt = None
    if master and world > 1:
        # data parallel keeps the bf16-weight design: ShardedMasterSGD over the xGMI kernels
        # where every rank's GPU is mapped into every rank (one node), else over RCCL
        # reduce-scatter / shard update / all-gather (decided collectively: all ranks agree)
        from ..parallel.zero import ShardedMasterSGD
        comm = getattr(args, "comm", "auto")
        opt = ShardedMasterSGD(
            [{"params": decay, "weight_decay": args.weight_decay},
             {"params": no_decay, "weight_decay": 0.0, "weights": "fp32"}],
            lr=args.learning_rate, momentum=args.momentum, bucket_mb=args.bucket_mb,
            backend=comm, order=list(model.parameters()))
        if hvd.rank() == 0 and opt.backend != "xgmi" and comm == "auto":
            print(f"[rank 0] ShardedMasterSGD over RCCL, {opt.backend} (ranks cannot map each "
                  "other's GPUs)", file=sys.stderr, flush=True)
    if opt is not None:
        pass                   # data parallel, sharded
    elif master:
        # conv/fc weights live in bf16 (fp32 masters inside MasterSGD): no per-step casts
        from ..ops.optim import MasterSGD, OptimizerGroup
        opt = OptimizerGroup(
            MasterSGD(decay, lr=args.learning_rate, momentum=args.momentum,
                      weight_decay=args.weight_decay),
            # BN scales / shifts and biases (fp32): torch's fused multi-tensor SGD, one launch
            # instead of the five of the foreach form
            torch.optim.SGD(no_decay, lr=args.learning_rate, momentum=args.momentum,
                            fused=dev.type == "cuda", foreach=None if dev.type == "cuda" else True))
    else:
        opt = torch.optim.SGD([{"params": decay, "weight_decay": args.weight_decay},
                               {"params": no_decay, "weight_decay": 0.0}],
                              lr=args.learning_rate, momentum=args.momentum,
                              foreach=dev.type == "cuda")
    if world > 1 and not master:
        opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(),
                                       bucket_mb=args.bucket_mb, comm=args.comm)
    g = torch.Generator(device=dev).manual_seed(hvd.rank())
    x = torch.randn(args.batch_size, 3, args.image_size, args.image_size, device=dev, generator=g)
    if nhwc:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, args.num_classes, (args.batch_size,), device=dev, generator=g)
    return model, opt, x, y


def comm_name(opt) -> str:
    """How the optimizer moves gradients (for logs and the JSON line)."""
    from ..parallel.zero import ShardedMasterSGD
    if isinstance(opt, ShardedMasterSGD):
        red = ""
        if opt.backend in ("rccl", "hier"):
            red = ",fp32-reduce" if opt.rccl_reduce_fp32 else ",bf16-ring-reduce"
        return f"{opt.backend}-sharded-sgd[{len(opt.buckets)} buckets{red}]"
    c = getattr(opt, "comm", None)
    return c if isinstance(c, str) else "none"


def comms_of(opt) -> list:
    """The xGMI communicators an optimizer owns (for ReplicaCheck's barrier-timeout check)."""
    from ..parallel.zero import ShardedMasterSGD
    if isinstance(opt, ShardedMasterSGD):
        return [opt.comm]       # None on the RCCL backend (ReplicaCheck skips it)
    return [getattr(opt, "xgmi", None)]


def train_step(model, opt, x, y, amp_dtype, zero_grad=True):
    with torch.autocast(device_type=x.device.type, dtype=amp_dtype, enabled=amp_dtype is not None,
                        cache_enabled=False):
        logits = model(x)
    # (outside autocast: the fused loss takes the bf16 logits as they are and sums in fp32, as
    # autocast's fp32 cross_entropy does after its upcast copy)
    if x.is_cuda:
        from ..ops.pool import cross_entropy
        loss = cross_entropy(logits, y)
    else:
        loss = F.cross_entropy(logits.float(), y)
    if zero_grad:
        opt.zero_grad(set_to_none=True)
    loss.backward()
    if x.is_cuda:
        from ..ops import conv
        conv.sync_wgrad()   # weight gradients computed on the side stream (if enabled)
    opt.step()
    return loss.detach()


def capture_step(model, opt, x, y, amp_dtype):
    """The whole step as one hipGraph: ~800 kernels per ResNet-50 step replay without host
    launches or inter-kernel gaps. Gradients are None at capture, so the captured backward writes
    (not accumulates) them, and every replay reuses the same memory (static x, y)."""
    opt.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        loss = train_step(model, opt, x, y, amp_dtype, zero_grad=False)
    return g, loss


def main(argv=None) -> int:
    args = parse(argv)
    from ..parallel import hvd
    dev = pick_device(args.device)
    hvd.init("nccl" if dev.type == "cuda" else "gloo")
    world, rank = hvd.size(), hvd.rank()
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        torch.backends.cudnn.benchmark = True      # MIOpen: pick the fastest conv solvers once
    else:
        share_cpu_threads(int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    amp = torch.bfloat16 if args.dtype == "bf16" else None
    if dev.type == "cuda":
        from ..ops import conv
        if args.async_wgrad == "on" and world > 1:
            raise SystemExit("--async_wgrad on is single-rank only (DP hooks read gradients "
                             "as soon as autograd produces them)")
        conv.set_async_wgrad(args.async_wgrad == "on")
    model, opt, x, y = build(args, dev, world)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    if rank == 0:
        print(f"Model: {args.model}  Batch size: {args.batch_size} per device, "
              f"{args.batch_size * world} global  Devices: {world} x {dev.type}  "
              f"Data: synthetic  dtype: {args.dtype}  graph: {args.graph}  comm: "
              f"{comm_name(opt)}", flush=True)
    for i in range(args.num_warmup_batches):
        t = time.perf_counter()
        train_step(model, opt, x, y, amp)
        sync()
        if rank == 0:   # the first steps include MIOpen's solver search: show progress
            print(f"warmup {i + 1}/{args.num_warmup_batches}: {time.perf_counter() - t:.2f} s",
                  flush=True)
    sync()
    graph = None
    if args.graph and dev.type == "cuda":
        # Data parallel too: the bucket hooks fire during the captured backward, so the graph
        # holds the pack + collective (xGMI kernel on the comm stream, or RCCL) of every bucket
        # exactly where eager mode issues them; all ranks replay the same collective sequence.
        ok = True
        try:
            graph, g_loss = capture_step(model, opt, x, y, amp)
        except RuntimeError as e:  # capture refused by a library call: run eagerly
            graph, ok = None, False
            print(f"[rank {rank}] hipGraph capture failed, running eagerly: {e}", flush=True)
        if world > 1:  # every rank replays, or none does (a lone eager rank would still match
            # the collective sequence, but the timing would not be one mode)
            t = torch.tensor([1 if ok else 0], device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
            if not int(t.item()):
                graph = None
            torch.distributed.barrier()
        if graph is not None:
            graph.replay()  # one untimed replay: the step the capture recorded is now executed
            sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    check = None
    if world > 1:
        from ..parallel.verify import ReplicaCheck
        check = ReplicaCheck(args.verify_every, lambda: list(model.parameters()),
                             comms=comms_of(opt))
    t0 = t_last = time.perf_counter()
    loss = None
    for i in range(1, args.num_batches + 1):
        if graph is not None:
            graph.replay()
            loss = g_loss
        else:
            loss = train_step(model, opt, x, y, amp)
        heartbeat.beat(i)
        if check is not None:
            check.maybe(i)
        if i % args.display_every == 0 or i == args.num_batches:
            sync()
            now = time.perf_counter()
            n = args.display_every if i % args.display_every == 0 else i % args.display_every
            if rank == 0:
                ips = n * args.batch_size / (now - t_last)
                print(f"{i}\timages/sec: {ips:.1f} (per device)  loss {float(loss):.3f}",
                      flush=True)
            t_last = now
    sync()
    elapsed = time.perf_counter() - t0
    if check is not None:
        check.verify(args.num_batches)   # every rank raises on divergence: no number printed
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    total = args.num_batches * args.batch_size * world / elapsed
    if rank == 0:
        print("-" * 64)
        print(f"total images/sec: {total:.2f}", flush=True)
        print("-" * 64)
        if args.json:
            print(json.dumps({"model": args.model, "images_per_s": round(total, 2),
                              "ms_per_step": round(elapsed / args.num_batches * 1e3, 3),
                              "batch_per_device": args.batch_size, "devices": world,
                              "dtype": args.dtype, "comm": comm_name(opt),
                              "exec": "hipgraph" if graph is not None else "eager",
                              "final_loss": round(float(loss), 4)}), flush=True)
    if rank == 0 and os.environ.get("ARENA_CONV_LOG"):
        from ..ops import conv
        for key, plan in conv.plans().items():
            print(f"conv {key[0]} w{key[1]} s{key[2]} p{key[3]}: fwd={plan.fwd} bwd={plan.bwd} "
                  f"bwd_bn={plan.bwd_bn} wgrad={plan.wgrad} {plan.times}", file=sys.stderr)
    hvd.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
