#!/usr/bin/env python3
"""Collective microbenchmark: xGMI one-kernel allreduce / fused Adam / broadcast (direct pull and
scatter + all-gather) / all-gather / sharded bf16 SGD vs RCCL.

    # 8x MI355X node: one rank per GPU, RCCL process group
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/ccl_bench.py
    # 1-GPU box: W ranks share GPU 0 (gloo process group, xGMI path only; "remote" reads are
    # local HBM, so this measures the protocol's barrier + launch cost, not link bandwidth)
    python tools/ccl_bench.py --same-gpu 2

``--forms pull,push`` times both xGMI protocol forms (the push form only if its self-test passes).
Prints one JSON line per (op, size) from rank 0: time per call (graph-replayed, 50 calls per
graph) and algorithm / bus bandwidth. busbw uses the ring-equivalent factor of each op: allreduce
2 (W-1)/W, broadcast 1, all-gather (W-1)/W (of the gathered bytes).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


from arena_amd.parallel.cclbench import timed  # noqa: E402


def bench(rank: int, world: int, sizes, rccl: bool,
          block_sweep=(1024, 2048, 4096, 8192, 16384), form: str = "pull") -> None:
    from arena_amd.parallel.xgmi import XgmiComm
    maxn = max(sizes) // 4
    # the push form is requested through the environment and kept only if its self-test passes
    os.environ["ARENA_XGMI_PUSH"] = "1" if form == "push" else "0"
    comm = XgmiComm(staging_elems=maxn, param_elems=397520, timeout_s=30.0)
    if comm.form != form:
        raise RuntimeError(f"asked for the {form} form, the self-test chose {comm.form}")
    rows = []
    comm.all_reduce_(comm.buffer()[:1024])  # first-call warm-up (code object load), untimed
    torch.cuda.synchronize()
    for nbytes in sizes:
        n = nbytes // 4
        x = torch.randn(n, device="cuda")
        stage = comm.buffer()[:n]
        t = timed(lambda: comm.all_reduce_(stage, scale=1.0 / world))
        rows.append(("xgmi_allreduce_zero_copy", nbytes, t))
        y = torch.empty_like(x)
        t = timed(lambda: comm.all_reduce_(x, out=y))
        rows.append(("xgmi_allreduce", nbytes, t))
        if n <= comm.ext.ccl_oneshot_elems:  # A/B: one-shot vs two-shot kernel at this size
            default = comm.ext.ccl_get_oneshot_max()
            for kind, cap in (("one_shot", comm.ext.ccl_oneshot_elems), ("two_shot", 0)):
                comm.ext.ccl_set_oneshot_max(cap)
                t = timed(lambda: comm.all_reduce_(stage, scale=1.0 / world))
                rows.append((f"xgmi_allreduce_zero_copy(forced_{kind})", nbytes, t))
            comm.ext.ccl_set_oneshot_max(default)
        if rccl:
            t = timed(lambda: dist.all_reduce(x))
            rows.append(("rccl_allreduce", nbytes, t))
    # broadcast (both algorithms forced, then the default switch) and all-gather
    for nbytes in sizes:
        n = nbytes // 4
        x = torch.randn(n, device="cuda")
        for kind, cap in (("direct", 1 << 40), ("scatter_allgather", 0)):
            comm.ext.ccl_set_bcast_direct_max(cap)
            t = timed(lambda: comm.broadcast_(x, 0))
            rows.append((f"xgmi_broadcast({kind})", nbytes, t))
        comm.ext.ccl_set_bcast_direct_max(128 << 10)
        if rccl:
            t = timed(lambda: dist.broadcast(x, 0))
            rows.append(("rccl_broadcast", nbytes, t))
        m = max(4, n // world // 4 * 4)
        shard = x[:m]
        if m <= comm.staging_elems:
            t = timed(lambda: comm.all_gather(shard))
            rows.append(("xgmi_allgather", m * 4 * world, t))
            if rccl:
                out = torch.empty(m * world, device="cuda")
                t = timed(lambda: dist.all_gather_into_tensor(out, shard))
                rows.append(("rccl_allgather", m * 4 * world, t))
    # the sharded bf16 SGD step of data-parallel ResNet-50 (25.5 M bf16 weights in 32 MB buckets)
    from arena_amd.parallel.xgmi import XgmiComm as _C
    nw = 25_557_032 // 8 * 8
    zc = _C(staging_elems=nw // 2, param_elems=nw // 2, timeout_s=30.0)
    master = torch.zeros(nw, device="cuda")
    mom = torch.zeros(nw, device="cuda")
    bucket = 16 << 20
    t = timed(lambda: [zc.peers.sgd_bf16(master, mom, o, min(bucket, nw - o), 0.1, 0.9, 4e-5,
                                         1.0 / world) for o in range(0, nw, bucket)], iters=10)
    rows.append(("xgmi_sharded_sgd_bf16(resnet50, 32MB buckets)", nw * 2, t))
    zc.close()
    # the DP trainer's fused step collective on the MNIST MLP's flat parameter vector, swept over
    # the per-block chunk size (fewer, fatter blocks = fewer barrier fences)
    n = 397520
    M = torch.zeros(n, device="cuda")
    V = torch.zeros(n, device="cuda")
    tt = torch.ones(1, dtype=torch.int64, device="cuda")
    for be in block_sweep:
        comm.ext.ccl_set_block_elems(be)
        t = timed(lambda: comm.adam_(M, V, n, t_step=tt, grad_scale=1.0 / world))
        rows.append((f"xgmi_rs_adam_ag(mnist_mlp,block_elems={be})", n * 4, t))
        stage = comm.buffer()[:n]
        t = timed(lambda: comm.all_reduce_(stage, scale=1.0 / world))
        rows.append((f"xgmi_allreduce_zero_copy(block_elems={be})", n * 4, t))
    comm.ext.ccl_set_block_elems(4096)
    comm.check()
    if rank == 0:
        for op, nb, t in rows:
            algbw = nb / t / 1e9
            f = 1.0 if "broadcast" in op else ((world - 1) / world if "allgather" in op
                                               else 2 * (world - 1) / world)
            print(json.dumps({"op": op, "form": form, "bytes": nb, "world": world,
                              "us": round(t * 1e6, 2),
                              "algbw_GBs": round(algbw, 2),
                              "busbw_GBs": round(algbw * f, 2)}), flush=True)
    comm.close()


def _same_gpu_rank(rank, world, port, sizes, forms):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    for form in forms:
        bench(rank, world, sizes, rccl=False, form=form)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-gpu", type=int, default=0, help="W ranks sharing GPU 0 (gloo PG)")
    ap.add_argument("--sizes", default="4096,65536,1048576,1590080,8388608,33554432")
    ap.add_argument("--forms", default="pull",
                    help="comma list of xGMI protocol forms to time: pull (default), push")
    args = ap.parse_args()
    sizes = [int(s) for s in args.sizes.split(",")]
    forms = args.forms.split(",")
    if args.same_gpu:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        mp.start_processes(_same_gpu_rank, args=(args.same_gpu, port, sizes, forms),
                           nprocs=args.same_gpu, start_method="spawn")
        return
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    for form in forms:
        bench(dist.get_rank(), dist.get_world_size(), sizes, rccl=True, form=form)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
