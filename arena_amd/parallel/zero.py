"""Sharded mixed-precision momentum SGD for data-parallel CNN training over xGMI.

The single-GPU ResNet path keeps conv/linear weights in bf16 with fp32 masters updated by one
multi-tensor kernel (:class:`arena_amd.ops.optim.MasterSGD`). Data parallel used to give that up:
Horovod's ``DistributedOptimizer`` moves fp32 gradients of fp32 weights, so every step cast the
weights to bf16, the gradients back to fp32, and pushed twice the bytes over xGMI.

:class:`ShardedMasterSGD` keeps the single-GPU design across ranks (ZeRO-1 style):

* the bf16 weights of every rank live in that rank's registered xGMI parameter buffer and the
  model's parameters are views into it (no casts in forward or backward);
* gradient buckets (reverse registration order, ~``bucket_mb`` of bf16) are packed into the
  registered staging buffer as soon as their last gradient is produced (post-accumulate hooks, on
  a comm stream, overlapped with the rest of backward);
* one ``xgmi_sgd_bf16`` kernel per bucket then reduce-scatters the bf16 gradients (fp32 sums in a
  fixed rank order), applies momentum SGD with weight decay to the rank's chunk of the fp32
  masters, and all-gathers the rounded bf16 weights into every rank's weight buffer -- the bytes
  of one bf16 allreduce, no separate optimizer pass, no fp32 weight traffic;
* every rank ends each step with bit-identical bf16 weights (``--verify_every`` checks it).

Masters and momentum are full-length fp32 arrays of which each rank updates only the chunks it
owns; :meth:`state_dict` reassembles them. Requires the xGMI collective (``xgmi.usable``); the CNN
bench falls back to fp32 weights + ``DistributedOptimizer`` (RCCL) elsewhere.
"""
from __future__ import annotations

from typing import Iterable, List

import torch
import torch.distributed as dist

from ..ops.optim import _same_memory_order
from ..runtime import heartbeat

Tensor = torch.Tensor


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


class _Bucket:
    def __init__(self, params, offsets, start, end):
        self.params, self.offsets = params, offsets
        self.start, self.end = start, end
        self.pending = set(id(p) for p in params)
        self.launched = False


class ShardedMasterSGD:
    def __init__(self, params: Iterable[Tensor], lr: float, momentum: float = 0.0,
                 weight_decay: float = 0.0, bucket_mb: float = 32.0, group=None,
                 timeout_s: float = 60.0):
        from .xgmi import XgmiComm
        self.params: List[Tensor] = [p for p in params]
        if not self.params:
            raise ValueError("ShardedMasterSGD needs at least one parameter")
        self.lr, self.momentum, self.weight_decay = float(lr), float(momentum), float(weight_decay)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        for p in self.params:
            if not p.is_cuda:
                raise ValueError("ShardedMasterSGD runs on GPU parameters")
            if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                raise ValueError("parameters must be contiguous or channels_last")
        # layout: gradient-readiness order (reverse registration), 8-element aligned slots
        cap = max(8, int(bucket_mb * 2**20 / 2))
        self.offsets = {}
        self.buckets: List[_Bucket] = []
        off = 0
        cur, cur_offs, start = [], [], 0
        for p in reversed(self.params):
            self.offsets[id(p)] = off
            cur.append(p)
            cur_offs.append(off)
            off += _pad8(p.numel())
            if off - start >= cap:
                self.buckets.append(_Bucket(cur, cur_offs, start, off))
                cur, cur_offs, start = [], [], off
        if cur:
            self.buckets.append(_Bucket(cur, cur_offs, start, off))
        self.total = off
        floats = (self.total + 1) // 2
        self.comm = XgmiComm(group, staging_elems=floats, param_elems=floats,
                             timeout_s=timeout_s)
        dev = self.params[0].device
        self.wbf = self.comm.params().view(torch.bfloat16)[: self.total]
        self.stage = self.comm.buffer().view(torch.bfloat16)[: self.total]
        self.master = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.mom = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self._owner = {}
        with torch.no_grad():
            self.wbf.zero_()
            self.stage.zero_()
            for b in self.buckets:
                for p in b.params:
                    self._owner[id(p)] = b
            for p in self.params:
                o = self.offsets[id(p)]
                self._view(self.master, p, o).copy_(p)
                v = self._view(self.wbf, p, o)
                v.copy_(p)
                p.data = v
                p.grad = None
        self.stream = torch.cuda.Stream(device=dev)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.param_groups = [{"params": self.params, "lr": self.lr, "momentum": self.momentum,
                              "weight_decay": self.weight_decay}]

    # ----------------------------------------------------------------------------------------
    @staticmethod
    def _view(flat: Tensor, p: Tensor, off: int) -> Tensor:
        return torch.as_strided(flat, p.shape, p.stride(), flat.storage_offset() + off)

    def _launch(self, b: _Bucket) -> None:
        main = torch.cuda.current_stream()
        self.stream.wait_stream(main)
        with torch.cuda.stream(self.stream):
            dst, src = [], []
            for p, o in zip(b.params, b.offsets):
                v = self._view(self.stage, p, o)
                if p.grad is None:
                    v.zero_()          # unused parameter this step: zero gradient (Horovod)
                    continue
                g = p.grad
                if g.dtype != torch.bfloat16 or not _same_memory_order(g, p):
                    raise RuntimeError("ShardedMasterSGD: gradients must be bf16 in the "
                                       f"parameter's memory order (param {tuple(p.shape)} "
                                       f"{p.stride()}, grad {g.dtype} {g.stride()})")
                g.record_stream(self.stream)
                dst.append(v)
                src.append(g)
            if dst:
                torch._foreach_copy_(dst, src)
            self.comm.peers.sgd_bf16(self.master, self.mom, b.start, b.end - b.start, self.lr,
                                     self.momentum, self.weight_decay, 1.0 / self.world)
        b.launched = True

    def _on_grad(self, p) -> None:
        b = self._owner[id(p)]
        b.pending.discard(id(p))
        if not b.pending and not b.launched:
            self._launch(b)

    # ------------------------------------------------------------------------- optimizer API
    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        for b in self.buckets:   # same launch order on every rank: bucket order
            if not b.launched:
                self._launch(b)
        torch.cuda.current_stream().wait_stream(self.stream)
        for b in self.buckets:
            b.launched = False
            b.pending = set(id(p) for p in b.params)
        heartbeat.beat()
        return None

    def shard_ranges(self, rank: int | None = None):
        r = self.rank if rank is None else rank
        return [tuple(self.comm.ext.ccl_sgd_shard(b.start, b.end - b.start, self.world, r))
                for b in self.buckets]

    @torch.no_grad()
    def _gathered(self, flat: Tensor) -> Tensor:
        """Full-length copy of a sharded fp32 array: owned chunks from every rank (sum of the
        rank-masked arrays over xGMI)."""
        mine = torch.zeros_like(flat)
        for lo, hi in self.shard_ranges():
            mine[lo:hi] = flat[lo:hi]
        self.comm.all_reduce_(mine)
        return mine

    def state_dict(self) -> dict:
        """fp32 masters + momentum per parameter in logical layout (collective)."""
        master, mom = self._gathered(self.master), self._gathered(self.mom)
        return {"master": [self._view(master, p, self.offsets[id(p)]).contiguous()
                           for p in self.params],
                "momentum_buffer": [self._view(mom, p, self.offsets[id(p)]).contiguous()
                                    for p in self.params],
                "lr": self.lr, "momentum": self.momentum, "weight_decay": self.weight_decay}

    @torch.no_grad()
    def load_state_dict(self, state: dict) -> None:
        for p, a, b in zip(self.params, state["master"], state["momentum_buffer"]):
            o = self.offsets[id(p)]
            self._view(self.master, p, o).copy_(a)
            self._view(self.mom, p, o).copy_(b)
            self._view(self.wbf, p, o).copy_(a)
        self.lr = float(state["lr"])

    def close(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        torch.cuda.synchronize()
        self.comm.close()
