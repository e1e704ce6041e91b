"""Sharded mixed-precision momentum SGD for data-parallel CNN training over xGMI.

The single-GPU ResNet path keeps conv/linear weights in bf16 with fp32 masters updated by one
multi-tensor kernel (:class:`arena_amd.ops.optim.MasterSGD`). Data parallel used to give that up:
Horovod's ``DistributedOptimizer`` moves fp32 gradients of fp32 weights, so every step cast the
weights to bf16, the gradients back to fp32, and pushed twice the bytes over xGMI.

:class:`ShardedMasterSGD` keeps the single-GPU design across ranks (ZeRO-1 style), for every
parameter of the model on ONE registered communicator:

* bf16 parameters (conv/fc weights) live in that rank's registered xGMI weight buffer (the
  model's parameters are views into it); fp32 parameters (BatchNorm scales/shifts, biases) live in
  an fp32 tail region of the same buffer;
* gradient buckets (reverse registration order, ~``bucket_mb`` each, never mixing dtypes or
  param groups) are packed into the registered staging buffer as soon as their last gradient is
  produced (post-accumulate hooks, on a comm stream, overlapped with the rest of backward);
* one kernel per bucket then reduce-scatters the gradients (fp32 sums in a fixed rank order),
  applies momentum SGD with weight decay to the rank's chunk (``xgmi_sgd_bf16``: fp32 masters,
  rounded bf16 weights all-gathered; ``xgmi_sgd_f32``: the fp32 weights are the masters) and
  all-gathers the result into every rank's weight buffer -- the bytes of one allreduce, no
  separate optimizer pass;
* every rank ends each step with bit-identical weights (``--verify_every`` checks it).

Update timing. With ``overlap=True`` (default) a bucket's update runs during ``backward()`` as
soon as its gradients are complete; ``step()`` only launches buckets whose gradients never
arrived (unused parameters: zero gradient, as Horovod) and joins the comm stream. Consequences:

* gradient accumulation must run its extra backwards inside :meth:`no_sync` (the hooks stay
  silent there, the final backward outside launches the updates on the accumulated gradients);
  a second backward that reaches an already-updated bucket before ``step()``/``zero_grad()``
  raises instead of silently dropping its gradients;
* to be able to skip a step after seeing the loss (non-finite loss, warmup), construct with
  ``overlap=False``: hooks only record readiness and ``step()`` launches every bucket;
* hyperparameters are read from ``param_groups`` at launch time (an lr schedule works eagerly;
  a captured hipGraph bakes the values in at capture).

Masters and momentum are full-length arrays of which each rank updates only the chunks it
owns; :meth:`state_dict` reassembles them. Requires the xGMI collective (``xgmi.usable``); the CNN
bench falls back to fp32 weights + ``DistributedOptimizer`` (RCCL) elsewhere.
"""
from __future__ import annotations

import contextlib
from typing import Iterable, List

import torch
import torch.distributed as dist

from ..ops.optim import _same_memory_order
from ..runtime import heartbeat

Tensor = torch.Tensor
_BF16, _F32 = torch.bfloat16, torch.float32


def _pad(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class _Bucket:
    def __init__(self, dtype, gi, params, offsets, start, end):
        self.dtype, self.gi = dtype, gi            # element dtype and param-group index
        self.params, self.offsets = params, offsets
        self.start, self.end = start, end          # region-relative, element units of `dtype`
        self.pending = set(id(p) for p in params)
        self.launched = False


class ShardedMasterSGD:
    """Momentum SGD (torch.optim.SGD semantics, dampening 0) sharded over the xGMI ranks.

    ``params``: tensors, or torch-style param-group dicts (``{"params": [...], "weight_decay":
    0.0, "weights": "fp32"}``) whose ``lr`` / ``momentum`` / ``weight_decay`` override the
    defaults. ``weights`` (default ``"bf16"``) is the dtype the group's parameters are kept in:
    bf16 weights with fp32 masters (the parameters are converted in place), or fp32 weights that
    are their own masters. Parameters must be CUDA tensors, contiguous or channels_last."""

    def __init__(self, params: Iterable, lr: float, momentum: float = 0.0,
                 weight_decay: float = 0.0, bucket_mb: float = 16.0, group=None,
                 timeout_s: float = 60.0, overlap: bool = True):
        from .xgmi import XgmiComm
        plist = list(params)
        if plist and isinstance(plist[0], dict):
            raw_groups = plist
        else:
            raw_groups = [{"params": plist}]
        self.param_groups = []
        for g in raw_groups:
            ps = [p for p in g["params"]]
            self.param_groups.append({"params": ps, "lr": float(g.get("lr", lr)),
                                      "momentum": float(g.get("momentum", momentum)),
                                      "weight_decay": float(g.get("weight_decay", weight_decay))})
        self.params: List[Tensor] = [p for g in self.param_groups for p in g["params"]]
        if not self.params:
            raise ValueError("ShardedMasterSGD needs at least one parameter")
        if len({id(p) for p in self.params}) != len(self.params):
            raise ValueError("a parameter appears in more than one param group")
        self.state: dict = {}   # Horovod's broadcast_optimizer_state finds nothing to send: the
        #                         masters are derived from the (already broadcast) weights
        self.group = group
        self.overlap = bool(overlap)
        self._no_sync = False
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        kind_of = {}
        for gi, g in enumerate(self.param_groups):
            kind = {"bf16": _BF16, "fp32": _F32}.get(raw_groups[gi].get("weights", "bf16"))
            if kind is None:
                raise ValueError("param group 'weights' must be 'bf16' or 'fp32'")
            g["weights"] = "bf16" if kind == _BF16 else "fp32"
            for p in g["params"]:
                kind_of[id(p)] = (kind, gi)
                if not p.is_cuda:
                    raise ValueError("ShardedMasterSGD runs on GPU parameters")
                if not p.is_floating_point():
                    raise TypeError(f"ShardedMasterSGD takes floating-point parameters, got "
                                    f"{p.dtype}")
                if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                    raise ValueError("parameters must be contiguous or channels_last")
        # Layout: gradient-readiness order (reverse registration). bf16 region [0, T16) in bf16
        # elements (16-byte aligned slots), fp32 region [F0, F0 + T32) in floats behind it. One
        # open bucket per weight dtype; it closes once it holds ~bucket_mb, or when the next
        # parameter of that dtype belongs to another param group (a bucket's range is contiguous
        # and its hyperparameters are one group's).
        cap = {_BF16: max(8, int(bucket_mb * 2**20 / 2)), _F32: max(4, int(bucket_mb * 2**20 / 4))}
        align = {_BF16: 8, _F32: 4}
        self.offsets = {}
        self.buckets: List[_Bucket] = []
        size = {_BF16: 0, _F32: 0}
        open_ = {}

        def close(dt):
            gi, ps, offs, start = open_.pop(dt)
            self.buckets.append(_Bucket(dt, gi, ps, offs, start, size[dt]))

        for p in reversed(self.params):
            dt, gi = kind_of[id(p)]
            if dt in open_ and open_[dt][0] != gi:
                close(dt)
            if dt not in open_:
                open_[dt] = (gi, [], [], size[dt])
            off = size[dt]
            self.offsets[id(p)] = off
            open_[dt][1].append(p)
            open_[dt][2].append(off)
            size[dt] = off + _pad(p.numel(), align[dt])
            if size[dt] - open_[dt][3] >= cap[dt]:
                close(dt)
        for dt in list(open_):
            close(dt)
        self.t16, self.t32 = size[_BF16], size[_F32]
        self.f0 = _pad((self.t16 + 1) // 2, 4)            # fp32 region start (floats)
        floats = self.f0 + self.t32
        self.comm = XgmiComm(group, staging_elems=floats, param_elems=floats,
                             timeout_s=timeout_s)
        dev = self.params[0].device
        buf, wbuf = self.comm.buffer(), self.comm.params()
        self.wbf = wbuf.view(_BF16)[: self.t16]
        self.stage = buf.view(_BF16)[: self.t16]
        self.w32 = wbuf[self.f0: self.f0 + self.t32]
        self.stage32 = buf[self.f0: self.f0 + self.t32]
        self.master = torch.zeros(self.t16, dtype=_F32, device=dev)
        self.mom = torch.zeros(self.t16, dtype=_F32, device=dev)
        self.mom32 = torch.zeros(self.t32, dtype=_F32, device=dev)
        self._owner = {}
        with torch.no_grad():
            wbuf.zero_()
            buf.zero_()
            for b in self.buckets:
                for p in b.params:
                    self._owner[id(p)] = b
            for p in self.params:
                o = self.offsets[id(p)]
                if kind_of[id(p)][0] == _BF16:
                    self._view(self.master, p, o).copy_(p)
                    v = self._view(self.wbf, p, o)
                else:
                    v = self._view(self.w32, p, o)
                v.copy_(p)
                p.data = v          # bf16 group: the parameter becomes bf16 (weights in the
                p.grad = None       # registered buffer, fp32 master in self.master)
        self.stream = torch.cuda.Stream(device=dev)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    # ----------------------------------------------------------------------------------------
    @staticmethod
    def _view(flat: Tensor, p: Tensor, off: int) -> Tensor:
        return torch.as_strided(flat, p.shape, p.stride(), flat.storage_offset() + off)

    def _launch(self, b: _Bucket) -> None:
        main = torch.cuda.current_stream()
        self.stream.wait_stream(main)
        g = self.param_groups[b.gi]
        stage = self.stage if b.dtype == _BF16 else self.stage32
        with torch.cuda.stream(self.stream):
            dst, src = [], []
            for p, o in zip(b.params, b.offsets):
                v = self._view(stage, p, o)
                if p.grad is None:
                    v.zero_()          # unused parameter this step: zero gradient (Horovod)
                    continue
                gr = p.grad
                if gr.dtype != p.dtype or not _same_memory_order(gr, p):
                    raise RuntimeError("ShardedMasterSGD: gradients must have the parameter's "
                                       f"dtype and memory order (param {p.dtype} "
                                       f"{tuple(p.shape)} {p.stride()}, grad {gr.dtype} "
                                       f"{gr.stride()})")
                gr.record_stream(self.stream)
                dst.append(v)
                src.append(gr)
            if dst:
                torch._foreach_copy_(dst, src)
            lr, mu, wd = float(g["lr"]), float(g["momentum"]), float(g["weight_decay"])
            if b.dtype == _BF16:
                self.comm.peers.sgd_bf16(self.master, self.mom, b.start, b.end - b.start, lr, mu,
                                         wd, 1.0 / self.world)
            else:
                self.comm.peers.sgd_f32(self.mom32[b.start:b.end], self.f0 + b.start,
                                        b.end - b.start, lr, mu, wd, 1.0 / self.world)
        b.launched = True

    def _on_grad(self, p) -> None:
        if self._no_sync:
            return
        b = self._owner[id(p)]
        if b.launched:
            raise RuntimeError(
                "ShardedMasterSGD: a second backward reached a bucket whose update already ran "
                "this step; call step() and zero_grad() between backwards, or accumulate the "
                "extra backwards inside `with opt.no_sync():`")
        b.pending.discard(id(p))
        if not b.pending and self.overlap:
            self._launch(b)

    def _reset(self) -> None:
        if any(b.launched for b in self.buckets):
            # updates already issued on the comm stream: later work on the main stream (the
            # next forward reads the weights) must be ordered after them
            torch.cuda.current_stream().wait_stream(self.stream)
        for b in self.buckets:
            b.launched = False
            b.pending = set(id(p) for p in b.params)

    # ------------------------------------------------------------------------- optimizer API
    @contextlib.contextmanager
    def no_sync(self):
        """Backwards inside only accumulate ``.grad`` (gradient accumulation): no bucket update."""
        prev, self._no_sync = self._no_sync, True
        try:
            yield
        finally:
            self._no_sync = prev

    def zero_grad(self, set_to_none: bool = True) -> None:
        self._reset()
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

    # ----------------------------------------------------------------------- state / sharding
    def shard_ranges(self, rank: int | None = None, dtype=_BF16):
        """Region-relative [lo, hi) element ranges this rank owns, one per bucket of ``dtype``."""
        r = self.rank if rank is None else rank
        out = []
        for b in self.buckets:
            if b.dtype != dtype:
                continue
            if dtype == _BF16:
                out.append(tuple(self.comm.ext.ccl_sgd_shard(b.start, b.end - b.start,
                                                             self.world, r)))
            else:
                lo, hi = self.comm.ext.ccl_sgd_f32_shard(self.f0 + b.start, b.end - b.start,
                                                         self.world, r)
                out.append((lo - self.f0, hi - self.f0))
        return out

    @torch.no_grad()
    def _gathered(self, flat: Tensor, dtype) -> Tensor:
        """Full-length copy of a sharded fp32 array: owned chunks from every rank (sum of the
        rank-masked arrays over xGMI; collective)."""
        mine = torch.zeros_like(flat)
        for lo, hi in self.shard_ranges(dtype=dtype):
            mine[lo:hi] = flat[lo:hi]
        if mine.numel():
            self.comm.all_reduce_(mine)
        return mine

    def _logical(self, flat: Tensor, p: Tensor) -> Tensor:
        return self._view(flat, p, self.offsets[id(p)]).contiguous()

    def state_dict(self) -> dict:
        """fp32 masters + momentum per parameter in logical layout, and the param groups'
        hyperparameters (collective: every rank must call it)."""
        torch.cuda.current_stream().wait_stream(self.stream)
        master = self._gathered(self.master, _BF16) if self.t16 else self.master
        mom = self._gathered(self.mom, _BF16) if self.t16 else self.mom
        mom32 = self._gathered(self.mom32, _F32) if self.t32 else self.mom32
        masters, moms = [], []
        for p in self.params:
            if p.dtype == _BF16:
                masters.append(self._logical(master, p))
                moms.append(self._logical(mom, p))
            else:
                masters.append(self._logical(self.w32, p).clone())
                moms.append(self._logical(mom32, p))
        return {"master": masters, "momentum_buffer": moms,
                "shapes": [tuple(p.shape) for p in self.params],
                "param_groups": [{k: v for k, v in g.items() if k != "params"}
                                 for g in self.param_groups]}

    @torch.no_grad()
    def load_state_dict(self, state: dict) -> None:
        masters, moms = state["master"], state["momentum_buffer"]
        if isinstance(masters, Tensor) or isinstance(moms, Tensor):
            raise ValueError("ShardedMasterSGD state must hold one tensor per parameter")
        n = len(self.params)
        if len(masters) != n or len(moms) != n:
            raise ValueError(f"ShardedMasterSGD state holds {len(masters)} masters / {len(moms)} "
                             f"momentum buffers for {n} parameters")
        for i, (p, a, b) in enumerate(zip(self.params, masters, moms)):
            if tuple(a.shape) != tuple(p.shape) or tuple(b.shape) != tuple(p.shape):
                raise ValueError(f"ShardedMasterSGD state: parameter {i} has shape "
                                 f"{tuple(p.shape)}, state has {tuple(a.shape)} / {tuple(b.shape)}")
        groups = state.get("param_groups")
        if groups is not None and len(groups) != len(self.param_groups):
            raise ValueError(f"ShardedMasterSGD state has {len(groups)} param groups, the "
                             f"optimizer {len(self.param_groups)}")
        torch.cuda.current_stream().wait_stream(self.stream)
        for p, a, b in zip(self.params, masters, moms):
            o = self.offsets[id(p)]
            if p.dtype == _BF16:
                self._view(self.master, p, o).copy_(a)
                self._view(self.mom, p, o).copy_(b)
                self._view(self.wbf, p, o).copy_(a)
            else:
                self._view(self.w32, p, o).copy_(a)
                self._view(self.mom32, p, o).copy_(b)
        for g, st in zip(self.param_groups, groups or []):
            for k in ("lr", "momentum", "weight_decay"):
                if k in st:
                    g[k] = float(st[k])
        self._rebind()

    @torch.no_grad()
    def _rebind(self) -> None:
        """Make every parameter a view into the registered weight buffer again (after a
        ``p.data = t`` re-binding), keeping the buffer's values."""
        for p in self.params:
            o = self.offsets[id(p)]
            v = self._view(self.wbf if p.dtype == _BF16 else self.w32, p, o)
            if p.data_ptr() != v.data_ptr():
                p.data = v

    @torch.no_grad()
    def sync_from_params(self) -> None:
        """Re-derive the masters from the current parameter values (call after
        ``model.load_state_dict(...)`` on a model whose optimizer already exists; otherwise the
        next update overwrites the loaded weights with stale masters). A parameter whose data
        was re-bound (``p.data = t``) is copied back into the registered buffer and re-bound to
        it, so the all-gathered weights reach the model again. Momentum is kept."""
        torch.cuda.current_stream().wait_stream(self.stream)
        for p in self.params:
            o = self.offsets[id(p)]
            v = self._view(self.wbf if p.dtype == _BF16 else self.w32, p, o)
            if p.data_ptr() != v.data_ptr():
                v.copy_(p)
                p.data = v
            if p.dtype == _BF16:
                self._view(self.master, p, o).copy_(v)

    def close(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        torch.cuda.synchronize()
        self.comm.close()
