"""Collective bandwidth measurement: xGMI kernels vs RCCL at the sizes a DP job moves.

North-star #2 of BASELINE.md ("xGMI custom allreduce bus bandwidth vs RCCL, 1 KB-256 MB",
SURVEY.md §6) measured by the driver-run ``bench.py --gpus N`` itself, so the first real 8-GPU
run records it next to the training throughput. The reference's counterpart is Horovod's NCCL
allreduce inside the hvd image (charts/tf-horovod/README.md:66-69, values.yaml:14); this module
times OUR two paths for the same operation:

* ``xgmi``: :class:`~arena_amd.parallel.xgmi.XgmiComm` kernels (one kernel per call, every peer
  link used at once, pull protocol unless the self-test promoted the push form);
* ``rccl``: ``torch.distributed`` over the ``nccl`` (= RCCL) process group -- skipped, with the
  reason, when the group is gloo (same-GPU rehearsal, where RCCL refuses two ranks per device).

Each call is replayed from a hipGraph (launch cost excluded), best of ``reps`` windows, MAX over
ranks. busbw uses the ring-equivalent factors: allreduce 2(W-1)/W, broadcast 1, all-gather (W-1)/W.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

DEFAULT_SIZES = (4 << 10, 256 << 10, 4 << 20, 64 << 20, 256 << 20)
# one ResNet-50 bucket of the sharded bf16 SGD (ShardedMasterSGD's default 32 MB bucket)
RESNET_BUCKET_ELEMS = 16 << 20


def timed(fn: Callable[[], object], iters: int = 50, reps: int = 5) -> float:
    """Seconds per call of ``fn`` (graph-replayed ``iters`` times; eager if capture is refused),
    best of ``reps`` windows, MAX over the ranks of the default group."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(iters):
                fn()
        run = g.replay
    except Exception:  # noqa: BLE001 - e.g. a collective that refuses capture: time eagerly
        torch.cuda.synchronize()

        def run():
            for _ in range(iters):
                fn()
    run()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.barrier()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / 1e3 / iters)
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([best], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        best = float(t.item())
    return best


def bus_factor(op: str, world: int) -> float:
    if op.startswith("broadcast"):
        return 1.0
    if op.startswith("allgather"):
        return (world - 1) / world
    return 2.0 * (world - 1) / world


def _row(op: str, nbytes: int, world: int, xgmi_s: Optional[float], rccl_s: Optional[float],
         rccl_note: str = "") -> dict:
    f = bus_factor(op, world)
    r = {"op": op, "bytes": nbytes}
    for k, t in (("xgmi", xgmi_s), ("rccl", rccl_s)):
        if t is None:
            continue
        r[f"{k}_us"] = round(t * 1e6, 2)
        r[f"{k}_busbw_GBs"] = round(nbytes / t / 1e9 * f, 2)
    if rccl_s is None:
        r["rccl"] = rccl_note or "skipped"
    if xgmi_s is not None and rccl_s is not None:
        r["xgmi_speedup"] = round(rccl_s / xgmi_s, 3)
    return r


def north_star(world: int, sizes=DEFAULT_SIZES, comm_timeout_s: float = 60.0,
               sgd_bucket_elems: int = RESNET_BUCKET_ELEMS) -> Dict[str, object]:
    """Collective over the default group (every rank calls it). Returns
    ``{"rows": [...], "xgmi": {...choice...}, "rccl": "nccl" | reason}``."""
    from .xgmi import XgmiComm, XgmiUnavailable, usable
    rccl_ok = dist.get_backend() == "nccl"
    rccl_note = "" if rccl_ok else f"process group is {dist.get_backend()} (same-GPU rehearsal)"
    maxn = max(sizes) // 4
    comm, why = None, ""
    if usable():
        try:
            comm = XgmiComm(staging_elems=maxn, param_elems=sgd_bucket_elems // 2,
                            timeout_s=comm_timeout_s)
        except XgmiUnavailable as e:
            why = str(e)
    else:
        why = "xgmi.usable() is false (not one node / extension missing / ARENA_XGMI=0)"
    rows: List[dict] = []
    dev = torch.device("cuda", torch.cuda.current_device())
    for nbytes in sizes:
        n = nbytes // 4
        iters = 50 if nbytes <= (4 << 20) else 10
        x = torch.randn(n, device=dev)
        tx = None
        if comm is not None:
            y = torch.empty_like(x)
            tx = timed(lambda: comm.all_reduce_(x, out=y), iters=iters)
        tr = timed(lambda: dist.all_reduce(x), iters=iters) if rccl_ok else None
        rows.append(_row("allreduce", nbytes, world, tx, tr, rccl_note))
        del x
    # all-gather and broadcast at the middle size (the bucket scale of a DP step)
    nbytes = 4 << 20
    n = nbytes // 4
    m = n // world // 4 * 4
    shard = torch.randn(m, device=dev)
    tx = timed(lambda: comm.all_gather(shard)) if comm is not None else None
    tr = None
    if rccl_ok:
        out = torch.empty(m * world, device=dev)
        tr = timed(lambda: dist.all_gather_into_tensor(out, shard))
    rows.append(_row("allgather", m * 4 * world, world, tx, tr, rccl_note))
    x = torch.randn(n, device=dev)
    tx = timed(lambda: comm.broadcast_(x, 0)) if comm is not None else None
    tr = timed(lambda: dist.broadcast(x, 0)) if rccl_ok else None
    rows.append(_row("broadcast", nbytes, world, tx, tr, rccl_note))
    # one ResNet-50-sized sharded-SGD bucket: fused RS + SGD + AG (xGMI) vs RCCL reduce-scatter +
    # the same SGD on the shard + all-gather of the bf16 weights (what the RCCL backend runs)
    ne = sgd_bucket_elems
    tx = None
    if comm is not None:
        master = torch.zeros(ne, device=dev)
        mom = torch.zeros(ne, device=dev)
        tx = timed(lambda: comm.peers.sgd_bf16(master, mom, 0, ne, 0.1, 0.9, 4e-5, 1.0 / world),
                   iters=10)
        del master, mom
    tr = None
    if rccl_ok:
        g = torch.zeros(ne, dtype=torch.bfloat16, device=dev)
        gs = torch.zeros(ne // world, dtype=torch.bfloat16, device=dev)
        w = torch.zeros(ne, dtype=torch.bfloat16, device=dev)
        ws = torch.zeros(ne // world, dtype=torch.bfloat16, device=dev)

        def rccl_sgd():
            dist.reduce_scatter_tensor(gs, g)
            ws.add_(gs, alpha=-0.1)
            dist.all_gather_into_tensor(w, ws)
        tr = timed(rccl_sgd, iters=10)
    rows.append(_row("sharded_sgd_bf16_bucket", ne * 2, world, tx, tr, rccl_note))
    info: Dict[str, object] = {"world": world, "rows": rows,
                               "rccl": "nccl" if rccl_ok else rccl_note}
    if comm is not None:
        comm.check()
        info["xgmi"] = {"form": comm.form, "selftest": comm.selftest_result,
                        "shared_gpu": bool(comm.shared_gpu)}
        comm.close()
    else:
        info["xgmi"] = {"unavailable": why}
    return info
