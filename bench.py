#!/usr/bin/env python3
"""Flagship benchmark: MNIST MLP data-parallel training throughput on MI355X.

Metric/config: the reference publishes no perf numbers (BASELINE.json is N/A); its headline
workload is the MNIST demo job (784-500-10 MLP, ReLU, dropout keep 0.9, softmax-xent, Adam 1e-3,
batch 100; docs/userguide/1-tfjob-standalone.md:178-186), which BASELINE.md adopts as the
north-star. We measure whole-job training throughput (samples/s, all ranks) with a FIXED per-GPU
batch of 100 (weak scaling), full fp32 compute, every step complete (forward, loss, backward,
gradient all-reduce when N>1, Adam update, device-side data gather + epoch reshuffles).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

``--gpus N`` is honoured either way. Under torchrun (``WORLD_SIZE`` set) every rank is already a
process. Without it and N > 1, this process becomes the launcher before it imports torch or touches
a GPU: it starts N copies of itself, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE /
LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT (``runtime.podlaunch``'s gang: the
first failing rank takes the others down, the launcher exits with its code; never exec), and relays
their output -- rank 0's JSON line is the launcher's stdout. That is the reference's launcher role
(``mpirun`` over the hostfile, charts/tf-horovod/templates/config.yaml:67-84,
charts/tf-horovod/README.md:66-69 ``hvd-distribute.sh <hosts> <gpus>``).

``--same-gpu`` (or ``ARENA_BENCH_SAME_GPU=1``) emulates an N-GPU node on one GPU: all ranks on
device 0, a gloo process group (RCCL refuses two ranks per device), the xGMI collectives over
same-device hipIpc mappings. It exercises the whole N > 1 path (sharded optimizers at W = N,
hipGraph-captured collectives, replica verification); its throughput is N ranks time-sharing one
GPU, so the line says ``"emulated"`` and is NOT a scaling number.

The MNIST steps run as replays of one hipGraph whose length divides the warmup, the timed step
count and the epoch; ``config.exec`` reports how many timed steps were replayed vs run eagerly.
The same line also carries ``resnet50_images_per_s`` (all ranks) / ``resnet50_ms_per_step``
(ResNet-50 bs128 per GPU, bf16, whole training step in one hipGraph, data parallel over the
sharded xGMI optimizer at N>1; ``--resnet 0`` skips it). At N>1 it also carries ``ccl``: xGMI vs
RCCL time and bus bandwidth per collective and size, the xGMI self-test outcome per kernel and the
protocol form in use (``--ccl 0`` skips it). A failed ResNet or collective run at N>1 is reported
in the line (``failed``) and the process exits 3.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); started by this script unless under torchrun")
    ap.add_argument("--same-gpu", action="store_true",
                    default=os.environ.get("ARENA_BENCH_SAME_GPU", "0") == "1",
                    help="emulate --gpus N on one GPU (all ranks on device 0, gloo + xGMI "
                         "same-device mappings): a correctness run of the N>1 path, not a "
                         "scaling number")
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--impl", choices=["fused", "torch"], default="fused",
                    help="fused = arena_amd HIP kernels + hipGraph; torch = eager PyTorch baseline")
    ap.add_argument("--hidden", type=int, default=500)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--steps-per-graph", type=int, default=0, help="0 = auto")
    ap.add_argument("--eval", action="store_true", help="report test accuracy after timing")
    ap.add_argument("--comm", choices=["auto", "xgmi", "rccl"], default="auto",
                    help="DP gradient path: fused xGMI reduce-scatter/Adam/all-gather kernel or "
                         "RCCL all_reduce + flat Adam (auto = xgmi when its self-test passes)")
    ap.add_argument("--verify-every", type=int, default=0,
                    help="N>1: every K timed steps, compare a parameter checksum across ranks "
                         "(and the xGMI barrier flags) and abort on divergence; adds a host sync "
                         "per check. The replicas are always verified once after timing.")
    ap.add_argument("--resnet", type=int, default=1,
                    help="1: also time ResNet-50 training (bs128/GPU, bf16, hipGraph; data "
                         "parallel over all ranks at N>1) and report it as extra resnet50_* keys "
                         "of the same JSON line")
    ap.add_argument("--resnet-steps", type=int, default=20)
    ap.add_argument("--resnet-batch", type=int, default=128)
    ap.add_argument("--ccl", type=int, default=1,
                    help="N>1: also time allreduce 4 KB..256 MB, all-gather, broadcast and one "
                         "ResNet-sized sharded-SGD bucket through xGMI and RCCL (key 'ccl')")
    ap.add_argument("--resnet-verify-every", type=int, default=10,
                    help="N>1: replica bit-identity check every K timed ResNet steps (untimed)")
    return ap.parse_args()


def max_over_ranks(x: float, dev) -> float:
    """MAX of a host float over all ranks (the slowest rank sets a synchronous step). gloo (the
    same-GPU emulation) reduces on the host, RCCL on the device."""
    import torch
    import torch.distributed as dist
    on_dev = dist.get_backend() == "nccl"
    e = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(e.item())


def _plan_stats() -> dict:
    """How the conv plans were decided (tuned here / received from rank 0 / from the plan file)
    and the seconds spent timing candidates."""
    from arena_amd.ops import planstore
    st = planstore.stats()
    st["tune_s"] = round(st["tune_s"], 2)
    return st


def bench_resnet50(dev, steps: int, batch: int, world: int = 1, verify_every: int = 10) -> dict:
    """ResNet-50 v1.5 training step (fwd + bwd + momentum-SGD on fp32 masters, bf16 MFMA convs,
    synthetic 224x224 ImageNet batch of ``batch`` per GPU) as ONE hipGraph: 8 eager warmup steps
    (the conv kernels' per-shape autotuning runs in the first), capture, five untimed replays,
    then ``steps`` timed replays bracketed by barrier + device synchronisation, max over ranks.
    Same code path as ``arena_amd.examples.cnn_bench``.

    Data parallel (world > 1, one process per GPU): on one node the optimizer is
    ``ShardedMasterSGD`` -- gradient buckets reduce-scattered, applied and all-gathered by one
    xGMI kernel each, on a comm stream overlapping backward, captured in the same graph; where
    the ranks cannot map each other's GPUs, fp32 weights + ``hvd.DistributedOptimizer`` over
    RCCL. Every ``verify_every`` timed steps (and once after) all replicas must hold
    bit-identical parameters (``ReplicaCheck``) or the run fails; the checks run outside the
    timed segments."""
    import torch
    import torch.distributed as dist
    from arena_amd.examples import cnn_bench
    from arena_amd.parallel import hvd
    if os.environ.get("ARENA_BENCH_FAIL_RESNET") == "1":
        # test hook (tests/test_bench_gpu.py): a failed N > 1 ResNet run must fail the process
        raise RuntimeError("injected ResNet-50 failure (ARENA_BENCH_FAIL_RESNET=1)")
    args = cnn_bench.parse(["--model", "resnet50", "--batch_size", str(batch), "--dtype", "bf16"])
    torch.backends.cudnn.benchmark = True
    if world > 1:
        hvd.init()
    model, opt, x, y = cnn_bench.build(args, dev, world)
    amp = torch.bfloat16
    for _ in range(8):
        cnn_bench.train_step(model, opt, x, y, amp)
    torch.cuda.synchronize()
    graph, g_loss = cnn_bench.capture_step(model, opt, x, y, amp)
    if world > 1:
        dist.barrier()
    for _ in range(5):   # untimed replays, so the timed ones start from a steady state
        graph.replay()
    torch.cuda.synchronize()
    check = None
    if world > 1:
        from arena_amd.parallel.verify import ReplicaCheck
        check = ReplicaCheck(verify_every, lambda: list(model.parameters()),
                             comms=cnn_bench.comms_of(opt))
    dt, done = 0.0, 0
    seg = verify_every if (world > 1 and verify_every > 0) else steps
    while done < steps:
        k = min(seg, steps - done)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            graph.replay()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt += time.perf_counter() - t0
        done += k
        if check is not None:
            check.maybe(done)
    if world > 1:
        dt = max_over_ranks(dt, dev)
        check.verify(steps)
    loss = float(g_loss)
    if not loss == loss:
        raise RuntimeError("ResNet-50 bench: non-finite loss")
    out = {"resnet50_images_per_s": round(steps * batch * world / dt, 1),
           "resnet50_ms_per_step": round(dt / steps * 1e3, 3),
           "resnet50_config": {"batch_per_gpu": batch, "global_batch": batch * world,
                               "image": 224, "dtype": "bf16", "parallelism": f"dp{world}",
                               "optimizer": "momentum-sgd fp32 masters", "timed_steps": steps,
                               "comm": cnn_bench.comm_name(opt) if world > 1 else "none",
                               "exec": f"hipgraph[whole step] {steps}/{steps} replays",
                               "final_loss": round(loss, 4),
                               "conv_plan": _plan_stats()}}
    if check is not None:
        out["resnet50_config"]["replicas_verified"] = check.checks
    return out


def launch_ranks(args, argv=None) -> int:
    """Launcher mode (``--gpus N > 1`` and no ``WORLD_SIZE``): start N ranks of this script and
    supervise them as a gang. Runs before torch is imported (no GPU call in this process)."""
    from arena_amd.runtime.podlaunch import local_world_envs, run_gang
    envs = local_world_envs(args.gpus)
    for e in envs:
        e["ARENA_BENCH_LAUNCHED"] = "1"
        if args.same_gpu:
            e["ARENA_BENCH_SAME_GPU"] = "1"
    argv = [sys.executable, os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None
                                                               else argv)
    print(f"[bench] launching {args.gpus} ranks (127.0.0.1:{envs[0]['MASTER_PORT']}"
          f"{', same GPU' if args.same_gpu else ''})", file=sys.stderr, flush=True)
    return run_gang([argv] * args.gpus, envs, grace_s=15.0)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if os.environ.get("ARENA_BENCH_ENV_PROBE") == "1":
        # test hook (tests/test_bench_launch.py): report the rank environment, touch no GPU
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                "MASTER_PORT", "ARENA_BENCH_SAME_GPU", "ARENA_BENCH_LAUNCHED")
        print(json.dumps({k: os.environ.get(k) for k in keys}), flush=True)
        if os.environ.get("ARENA_BENCH_PROBE_FAIL_RANK") == os.environ.get("RANK"):
            sys.exit(3)
        time.sleep(float(os.environ.get("ARENA_BENCH_PROBE_SLEEP", "0")))
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    same_gpu = args.same_gpu and world > 1
    if world != args.gpus and rank == 0:
        print(f"[bench] note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE",
              file=sys.stderr)
    dev_index = 0 if same_gpu else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    pg = None
    if world > 1:
        if same_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        pg = dist.group.WORLD

    from arena_amd.data.mnist import load_mnist
    from arena_amd.models.mlp import FusedMLPTrainer, MLPConfig

    data = load_mnist()
    cfg = MLPConfig(hidden=args.hidden, batch=args.batch)

    if args.impl == "fused":
        tr = FusedMLPTrainer(cfg, data.train_images, data.train_labels, device=dev,
                             process_group=pg, rank=rank, world=world, comm=args.comm)
        # the graph length divides the timed steps and the epoch, and its baked-in step parity is
        # the parity of the first timed step, so every timed step is a replay of the graph
        # captured here, before the warmup (warmup steps that do not fit replays run eagerly)
        spg = args.steps_per_graph or tr.pick_steps_per_graph(runs=(args.steps,))
        graphs = tr.enable_graphs(spg, start_parity=args.warmup & 1)
        run = tr.train_steps
        mode = f"hipgraph[{tr.graph_mode},{spg} steps/graph]" if graphs else "eager"
        if world > 1:
            mode += f",comm={tr.comm}"
    else:
        from arena_amd.models.torch_mlp import EagerMLPTrainer
        tr = EagerMLPTrainer(cfg, data.train_images, data.train_labels, device=dev,
                             process_group=pg, rank=rank, world=world)
        run = tr.train_steps
        mode = "eager-pytorch"

    run(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    check = None
    if world > 1:
        from arena_amd.parallel.verify import ReplicaCheck
        check = ReplicaCheck(args.verify_every,
                             lambda: [tr.P] if hasattr(tr, "P") else list(tr.model.parameters()),
                             group=pg,
                             comms=[getattr(tr, "xgmi", None)])
    g0, e0 = getattr(tr, "graph_steps", 0), getattr(tr, "eager_steps", 0)
    t0 = time.perf_counter()
    if check is not None and args.verify_every > 0:
        done = 0
        while done < args.steps:
            k = min(args.verify_every, args.steps - done)
            run(k)
            done += k
            check.maybe(done)
    else:
        run(args.steps)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if args.impl == "fused":
        # what the timed region actually executed (not what was configured)
        mode += f"; timed: {tr.graph_steps - g0}/{args.steps} graph-replayed, " \
                f"{tr.eager_steps - e0} eager"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = t1 - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev)

    extra = {}
    if check is not None:
        # replicas bit-identical on every rank and no xGMI barrier timed out, or every rank
        # raises (ReplicaMismatch) and the run fails loudly instead of printing a number
        check.verify(args.steps)
        extra["replicas_verified"] = check.checks
    loss, acc = tr.recent_metrics(100)
    extra["train_loss_last100"] = round(loss, 5)
    extra["train_acc_last100"] = round(acc, 5)
    if args.eval:
        tl, ta = tr.evaluate(data.test_images, data.test_labels)
        extra["test_loss"] = round(tl, 5)
        extra["test_acc"] = round(ta, 5)

    failed = []
    if args.resnet and args.impl == "fused":
        del tr
        torch.cuda.empty_cache()
        try:
            extra.update(bench_resnet50(dev, args.resnet_steps, args.resnet_batch, world,
                                        args.resnet_verify_every))
        except Exception as e:   # reported in the line, then the run fails (exit 3)
            print(f"[bench] ResNet-50 failed: {e!r}", file=sys.stderr)
            extra["resnet50_error"] = repr(e)[:300]
            failed.append("resnet50")
    if world > 1 and args.ccl:
        # north-star #2: xGMI vs RCCL collective bandwidth on this node
        from arena_amd.parallel import cclbench
        torch.cuda.empty_cache()
        try:
            extra["ccl"] = cclbench.north_star(world)
        except Exception as e:
            print(f"[bench] collective benchmark failed: {e!r}", file=sys.stderr)
            extra["ccl_error"] = repr(e)[:300]
            failed.append("ccl")

    samples = world * cfg.batch * args.steps
    value = samples / elapsed
    if rank == 0:
        out = {
            "metric": "mnist_mlp_train_throughput",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": f"synthetic ({data.source} MNIST-shaped uint8 60k/10k, device-resident)",
            "config": {"model": f"mnist_mlp_784-{args.hidden}-10 (relu, dropout 0.9, adam 1e-3)",
                       "global_batch": world * cfg.batch, "seq_len": None,
                       "parallelism": f"dp{world}", "impl": args.impl, "exec": mode,
                       "launch": "bench.py" if os.environ.get("ARENA_BENCH_LAUNCHED") else
                       ("torchrun" if world > 1 else "single")},
            **extra,
        }
        if same_gpu:
            out["emulated"] = (f"{world} ranks time-sharing ONE GPU (gloo + same-device xGMI "
                               f"mappings): checks the N>1 path, not a scaling number")
        if failed:
            out["failed"] = failed
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if failed:
        # the line above still reports what was measured, but a diverged or broken N > 1 run
        # must not look like a success to whoever checks the exit code
        sys.exit(3)


if __name__ == "__main__":
    main()
