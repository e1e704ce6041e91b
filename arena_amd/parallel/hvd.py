"""Horovod-style data-parallel API on torch.distributed (RCCL over xGMI on MI355X, gloo on CPU).

The reference's allreduce jobs run Horovod images (DistributedOptimizer
gradient allreduce with a 64 MB tensor-fusion buffer, broadcast_global_variables(0), allgather).
This module provides the same user-facing calls, designed for one process per GPU:

    import arena_amd.parallel.hvd as hvd
    hvd.init()                                   # env:// rendezvous (RANK/WORLD_SIZE/MASTER_*)
    torch.cuda.set_device(hvd.local_rank())
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters())

``broadcast_parameters`` / ``broadcast_`` / ``allgather`` run the xGMI copy kernels when every
rank's GPU is mapped into every rank (single node, ``xgmi.usable``), else RCCL (gloo on CPU).
``DistributedOptimizer`` packs gradients into flat fp32 buckets with the native multi-tensor
kernel as soon as each bucket's last gradient is produced (post-accumulate hooks), launches an
async all_reduce per bucket so communication overlaps the rest of backward, and unpacks the
averaged result (the 1/N scale fused into the unpack kernel) in ``step()``. Bucket size defaults
to 32 MB: on a fully connected 8x MI355X node each ring hop is one ~153 GB/s xGMI link, so
32-64 MB buckets amortise the per-collective latency while leaving several buckets to overlap.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..runtime import heartbeat

_STATE = {"pg": None, "local_rank": 0, "local_size": 1, "xgmi": None}
# staging floats of the communicator used by broadcast/allgather (64 MB; larger tensors go
# through it in pieces)
_XGMI_STAGING = 16 << 20


def _new_comm(staging_elems: int):
    """A fresh xGMI communicator (collective), or None when the ranks cannot map each other."""
    from . import xgmi
    if not xgmi.usable():
        return None
    try:
        return xgmi.XgmiComm(staging_elems=staging_elems)
    except xgmi.XgmiUnavailable:
        return None


def _xgmi_comm(t: Optional[torch.Tensor] = None):
    """The job's xGMI communicator for broadcast/allgather (collective on first use), or None to
    use RCCL/gloo: CPU tensors, ``ARENA_XGMI=0``, or ranks that cannot map each other's GPUs."""
    if t is not None and not t.is_cuda:
        return None
    c = _STATE["xgmi"]
    if c is None:
        c = _new_comm(_XGMI_STAGING) or False
        _STATE["xgmi"] = c
    return c or None


def init(backend: Optional[str] = None, timeout_s: float = 600.0):
    """Initialise the default process group from the environment (idempotent)."""
    if not dist.is_initialized():
        if "WORLD_SIZE" not in os.environ:  # plain `python script.py`: a world of one
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                              MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                              MASTER_PORT=os.environ.get("MASTER_PORT", str(port)))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        import datetime
        kwargs = {}
        if backend == "nccl":
            lr = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(lr)
            kwargs["device_id"] = torch.device("cuda", lr)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    _STATE["local_rank"] = int(os.environ.get("LOCAL_RANK", "0"))
    _STATE["local_size"] = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return dist.group.WORLD


def is_initialized() -> bool:
    return dist.is_initialized()


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def local_rank() -> int:
    return _STATE["local_rank"]


def local_size() -> int:
    return _STATE["local_size"]


def shutdown() -> None:
    c = _STATE["xgmi"]
    if c:
        c.close()
    _STATE["xgmi"] = None
    if dist.is_initialized():
        dist.destroy_process_group()


def allreduce(tensor: torch.Tensor, average: bool = True, op=None) -> torch.Tensor:
    """Out-of-place allreduce (Horovod semantics: returns a new tensor)."""
    out = tensor.detach().clone()
    allreduce_(out, average=average, op=op)
    return out


def allreduce_(tensor: torch.Tensor, average: bool = True, op=None) -> torch.Tensor:
    if size() == 1:
        return tensor
    dist.all_reduce(tensor, op=op or dist.ReduceOp.SUM)
    if average and (op is None or op == dist.ReduceOp.SUM):
        tensor.div_(size())
    return tensor


def allgather(tensor: torch.Tensor) -> torch.Tensor:
    """Concatenate along dim 0 across ranks (first dims may differ, like hvd.allgather)."""
    if size() == 1:
        return tensor.clone()
    n = torch.tensor([tensor.shape[0]], device=tensor.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(size())]
    dist.all_gather(sizes, n)
    mx = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((mx,) + tuple(tensor.shape[1:]), device=tensor.device, dtype=tensor.dtype)
    pad[: tensor.shape[0]] = tensor
    comm = _xgmi_comm(tensor)
    if comm is not None:
        outs = list(comm.all_gather(pad))      # one copy kernel over xGMI
    else:
        outs = [torch.empty_like(pad) for _ in range(size())]
        dist.all_gather(outs, pad)
    return torch.cat([o[: int(s.item())] for o, s in zip(outs, sizes)], dim=0)


def broadcast_(tensor: torch.Tensor, root_rank: int = 0) -> torch.Tensor:
    if size() > 1:
        comm = _xgmi_comm(tensor)
        if comm is not None:
            comm.broadcast_(tensor, root_rank)
        else:
            dist.broadcast(tensor, root_rank)
    return tensor


def broadcast_parameters(params, root_rank: int = 0) -> None:
    """Broadcast a state_dict / named_parameters / list of tensors from root (in place), packed
    into one flat buffer per dtype so it is a handful of collectives, not one per tensor.

    Runs before training, when no job communicator exists yet: the xGMI path then uses a
    temporary communicator whose staging buffer is sized to the largest flat buffer (capped at
    the job communicator's 64 MB) and released right after, instead of keeping a 64 MB
    registered buffer alive next to the optimizer's own communicator for the whole job."""
    if size() == 1:
        return
    if isinstance(params, dict):
        tensors = list(params.values())
    else:
        tensors = [p[1] if isinstance(p, tuple) else p for p in params]
    by_dtype: Dict[Tuple[torch.dtype, torch.device], List[torch.Tensor]] = {}
    for t in tensors:
        if torch.is_tensor(t):
            by_dtype.setdefault((t.dtype, t.device), []).append(t)
    flats = {k: torch.cat([t.detach().reshape(-1) for t in ts]) for k, ts in by_dtype.items()}
    comm, temp = _STATE["xgmi"] or None, False
    if _STATE["xgmi"] is None:
        # whether to build a temporary xGMI communicator is decided COLLECTIVELY: building it is
        # a collective (xgmi.usable, XgmiComm), so a rank whose list happens to hold no GPU
        # tensor must still take part, or the ranks that do would wait for it forever
        words = max([((f.numel() * f.element_size() + 15) // 16 * 4) for (_, dev), f in
                     flats.items() if dev.type == "cuda"] + [0])
        allw: List[Optional[int]] = [None] * size()
        dist.all_gather_object(allw, words)
        if max(allw) > 0:
            comm, temp = _new_comm(min(max(allw), _XGMI_STAGING)), True
    try:
        for (dt, dev), ts in by_dtype.items():
            flat = flats[(dt, dev)]
            if comm is not None and flat.is_cuda:
                comm.broadcast_(flat, root_rank)   # xGMI direct pull / scatter + all-gather
            elif not flat.is_cuda and dist.get_backend() == "nccl":
                # host tensors (e.g. torch Adam's CPU "step") through the device for RCCL
                dflat = flat.cuda()
                dist.broadcast(dflat, root_rank)
                flat.copy_(dflat.cpu())
            else:
                dist.broadcast(flat, root_rank)
            off = 0
            with torch.no_grad():
                for t in ts:
                    n = t.numel()
                    t.copy_(flat[off:off + n].view_as(t))
                    off += n
        if comm is not None:
            # a barrier that timed out leaves the copies incomplete: fail here, before training
            # starts from weights that silently differ between ranks
            comm.check()
    finally:
        if temp and comm is not None:
            comm.close()


def _leaf_optimizers(optimizer) -> list:
    """The torch-style optimizers inside ``optimizer`` (OptimizerGroup members, the one a
    DistributedOptimizer wraps), in a fixed order."""
    subs = getattr(optimizer, "opts", None)          # OptimizerGroup: its members, in order
    if subs is not None:
        return [o for s in subs for o in _leaf_optimizers(s)]
    inner = getattr(optimizer, "opt", None)          # DistributedOptimizer wraps one
    if inner is not None and not hasattr(optimizer, "param_groups"):
        return _leaf_optimizers(inner)
    return [optimizer]


def _state_layout(opt) -> list:
    """[(group, param, key, kind, meta)] of a torch-style optimizer's per-parameter state: kind
    "t" for tensors (meta = shape, dtype name), "v" for plain values (meta = the value)."""
    state = getattr(opt, "state", None)
    if not state or not hasattr(opt, "param_groups"):
        return []
    out = []
    for gi, group in enumerate(opt.param_groups):
        for pi, p in enumerate(group["params"]):
            st = state.get(p, {})
            for k in sorted(st, key=str):
                v = st[k]
                if torch.is_tensor(v):
                    out.append((gi, pi, k, "t", (tuple(v.shape), str(v.dtype).split(".")[-1],
                                                 v.device.type)))
                else:
                    out.append((gi, pi, k, "v", v))
    return out


def _optimizer_state_tensors(optimizer) -> List[torch.Tensor]:
    out = []
    for opt in _leaf_optimizers(optimizer):
        state = getattr(opt, "state", None)
        if not state:        # nothing to send (e.g. ShardedMasterSGD: masters derive from weights)
            continue
        for group in opt.param_groups:
            for p in group["params"]:
                st = state.get(p, {})
                for k in sorted(st, key=str):
                    if torch.is_tensor(st[k]):
                        out.append(st[k])
    return out


def broadcast_optimizer_state(optimizer, root_rank: int = 0) -> None:
    """Broadcast the root's optimizer state (momentum buffers, Adam moments, step counts) in
    place. Recurses into ``OptimizerGroup`` members; optimizers without per-parameter state are
    skipped. The usual Horovod pattern works -- a checkpoint loaded on the root only: the root's
    state LAYOUT is broadcast first, and every other rank creates whatever state it lacks (zeros
    of the root's shape and dtype, the root's plain values) before the tensors move, so every
    rank enters the same collectives."""
    if size() == 1:
        return
    leaves = _leaf_optimizers(optimizer)
    box = [[_state_layout(o) for o in leaves] if rank() == root_rank else None]
    dist.broadcast_object_list(box, src=root_rank)
    layouts = box[0]
    if len(layouts) != len(leaves):
        raise RuntimeError(f"broadcast_optimizer_state: root has {len(layouts)} optimizers, "
                           f"rank {rank()} has {len(leaves)}")
    for opt, layout in zip(leaves, layouts):
        for gi, pi, k, kind, meta in layout:
            p = opt.param_groups[gi]["params"][pi]
            st = opt.state[p]          # torch optimizers' state is a defaultdict(dict)
            if kind == "v":
                st[k] = meta
                continue
            shape, dtname, devtype = meta
            have = st.get(k)
            dt = getattr(torch, dtname)
            # the ROOT's device type decides where the tensor lives (torch keeps Adam's scalar
            # "step" on the CPU unless fused/capturable, then on the parameter's device): the
            # broadcast groups tensors by (dtype, device), so a rank whose copy lives elsewhere
            # would enter collectives of different sizes than the root
            dev = torch.device("cpu") if devtype == "cpu" else (
                p.device if p.device.type == devtype else torch.device(devtype))
            if not (torch.is_tensor(have) and tuple(have.shape) == shape and have.dtype == dt
                    and have.device.type == devtype):
                st[k] = (have.to(dev) if torch.is_tensor(have) and tuple(have.shape) == shape
                         and have.dtype == dt else torch.zeros(shape, dtype=dt, device=dev))
    broadcast_parameters(_optimizer_state_tensors(optimizer), root_rank)


def _raw(t: torch.Tensor) -> Optional[torch.Tensor]:
    """1-D view of a dense tensor's memory: contiguous, or channels_last (NHWC conv weights and
    their gradients). Averaging is elementwise and every rank has the same layout for the same
    parameter, so buckets can hold the memory order directly (no layout copies). None for any
    other stride pattern."""
    if t.is_contiguous():
        return t.view(-1)
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).reshape(-1)  # NHWC order == memory order: a view
    return None


class _Bucket:
    def __init__(self, params: List[torch.nn.Parameter], device):
        self.params = params
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += (p.numel() + 3) // 4 * 4
        self.flat = torch.zeros(off, device=device, dtype=torch.float32)
        self.pending = set(id(p) for p in params)
        self.work = None


class _Done:
    @staticmethod
    def wait():
        return None


_DONE = _Done()


class DistributedOptimizer:
    """Wraps a torch optimizer: bucketed async gradient allreduce overlapped with backward."""

    def __init__(self, optimizer: torch.optim.Optimizer, named_parameters=None,
                 bucket_mb: float = 32.0, process_group=None, comm: str = "auto"):
        """``comm``: "xgmi" (single-node fused xGMI kernel), "rccl" (torch.distributed),
        "auto" (xgmi when its self-test passes on every rank, else rccl)."""
        self.opt = optimizer
        self.pg = process_group
        params = [p for _, p in named_parameters] if named_parameters is not None else \
            [p for g in optimizer.param_groups for p in g["params"]]
        params = [p for p in params if p.requires_grad]
        if any(p.dtype != torch.float32 for p in params):
            raise TypeError("DistributedOptimizer buckets are fp32 (master weights)")
        # reverse registration order ~ the order gradients become ready in backward
        cap = int(bucket_mb * 2**20 / 4)
        self.buckets: List[_Bucket] = []
        cur: List[torch.nn.Parameter] = []
        n = 0
        for p in reversed(params):
            cur.append(p)
            n += p.numel()
            if n >= cap:
                self.buckets.append(_Bucket(cur, p.device))
                cur, n = [], 0
        if cur:
            self.buckets.append(_Bucket(cur, cur[0].device))
        self._owner = {}
        for b in self.buckets:
            for p in b.params:
                self._owner[id(p)] = b
        self._hooks = []
        self.xgmi = None
        if size() > 1 and comm in ("auto", "xgmi") and params and params[0].is_cuda:
            from . import xgmi
            if xgmi.usable(process_group):
                try:
                    self.xgmi = xgmi.XgmiComm(process_group,
                                              staging_elems=max(b.flat.numel() for b in self.buckets))
                except xgmi.XgmiUnavailable:
                    if comm == "xgmi":
                        raise
            elif comm == "xgmi":
                raise xgmi.XgmiUnavailable("xGMI collective not usable for this process group")
        self.comm = "xgmi" if self.xgmi is not None else "rccl"
        # xGMI buckets run on their own stream (RCCL's async_op already has one), ordered after
        # the gradients through an event, so the collective overlaps the rest of backward
        self._stream = torch.cuda.Stream() if self.xgmi is not None else None
        if size() > 1:
            for p in params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    @property
    def param_groups(self):
        return self.opt.param_groups

    @property
    def state(self):
        return self.opt.state

    def _launch(self, b: _Bucket) -> None:
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in b.params]
        grads = [r if (r := _raw(g)) is not None else g.contiguous().view(-1) for g in grads]
        if self.xgmi is not None:
            # pack straight into the registered staging buffer (zero-copy input), average on the
            # way out. Comm stream: waits for the grads (event), then buckets run in launch order,
            # so the shared staging buffer is never overwritten while a reduction still reads it.
            ready = torch.cuda.current_stream()
            self._stream.wait_stream(ready)
            with torch.cuda.stream(self._stream):
                for g in grads:
                    g.record_stream(self._stream)
                stage = self.xgmi.buffer()[: b.flat.numel()]
                ops.flatten_into(grads, b.offsets, stage, 1.0)
                self.xgmi.all_reduce_(stage, scale=1.0 / size(), out=b.flat)
            b.work = _DONE
            return
        ops.flatten_into(grads, b.offsets, b.flat, 1.0)
        b.work = dist.all_reduce(b.flat, group=self.pg, async_op=True)

    def _on_grad(self, p) -> None:
        b = self._owner[id(p)]
        b.pending.discard(id(p))
        if not b.pending and b.work is None:
            self._launch(b)

    def synchronize(self) -> None:
        if size() == 1:
            return
        inv = 1.0 if self.xgmi is not None else 1.0 / size()
        for b in self.buckets:
            if b.work is None:  # some grads never arrived (unused params): reduce anyway
                self._launch(b)
        if self._stream is not None:
            torch.cuda.current_stream().wait_stream(self._stream)
        for b in self.buckets:
            b.work.wait()
            grads, strided = [], []
            for p in b.params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                r = _raw(p.grad)
                if r is None:  # exotic strides: unpack in logical order, then copy in
                    r = torch.empty(p.numel(), device=p.device, dtype=p.grad.dtype)
                    strided.append((p.grad, r))
                grads.append(r)
            ops.unflatten_from(grads, b.offsets, b.flat, inv)
            for g, r in strided:
                g.copy_(r.view(g.shape))
            b.work = None
            b.pending = set(id(p) for p in b.params)

    def step(self, closure=None):
        self.synchronize()
        out = self.opt.step(closure)
        heartbeat.beat()  # training progress: a rank hung in a collective stops beating
        return out

    def zero_grad(self, set_to_none: bool = True):
        self.opt.zero_grad(set_to_none=set_to_none)

    def state_dict(self):
        return self.opt.state_dict()

    def load_state_dict(self, sd):
        self.opt.load_state_dict(sd)
