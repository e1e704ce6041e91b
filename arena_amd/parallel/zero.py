"""Sharded mixed-precision momentum SGD for data-parallel CNN training (xGMI or RCCL).

The single-GPU ResNet path keeps conv/linear weights in bf16 with fp32 masters updated by one
multi-tensor kernel (:class:`arena_amd.ops.optim.MasterSGD`). Data parallel used to give that up:
Horovod's ``DistributedOptimizer`` moves fp32 gradients of fp32 weights, so every step cast the
weights to bf16, the gradients back to fp32, and pushed twice the bytes over the links.

:class:`ShardedMasterSGD` keeps the single-GPU design across ranks (ZeRO-1 style), for every
parameter of the model:

* bf16 parameters (conv/fc weights) live in one flat bf16 weight buffer (the model's parameters
  are views into it); fp32 parameters (BatchNorm scales/shifts, biases) live in an fp32 region
  behind it;
* gradient buckets of ~``bucket_mb`` are formed in gradient-readiness order (reverse model
  order, ``order=``). A bucket may hold a bf16 and an fp32 sub-range side by side, so a block's
  BN parameters travel with the conv weights whose gradients become ready at the same time
  instead of in one fp32 tail bucket that can only launch after the whole backward. The
  input-side bucket -- the last one ready, whose update nothing can overlap -- is capped at
  ``last_bucket_mb``;
* each bucket is packed as soon as its last gradient is produced (post-accumulate hooks, on a
  comm stream, overlapped with the rest of backward) and updated by a reduce-scatter -> fp32
  shard update -> all-gather, the bytes of one allreduce and no separate optimizer pass:

  - ``backend="xgmi"`` (one node, every rank's GPU mapped into every rank): one kernel per
    sub-range over hipIpc peer memory (``xgmi_sgd_bf16`` / ``xgmi_sgd_f32``: fp32 sums in a fixed
    rank order, the rank's chunk updated in its own buffer, every rank then pulling the other
    ranks' rounded weights -- no kernel stores into a peer's memory);
  - ``backend="rccl"`` (ranks that cannot map each other: multi-pod, multi-node):
    ``reduce_scatter_tensor`` of the bucket's bf16 (or fp32) range, the ``shard_sgd`` HIP kernel
    on the owned equal-size shard, ``all_gather_into_tensor`` of the updated weights. bf16 buckets
    reduce in bf16 by default (the bytes the xGMI path moves); ``rccl_reduce_fp32=True`` reduces
    fp32 copies instead (exact sums, twice the bytes; the default on ``hier``, whose two levels
    would round a bf16 sum twice). Buckets launch strictly in index order on every rank, even
    when a rank's gradients become ready in another order;
  - ``backend="hier"`` (several nodes of ``local_size`` ranks each, consecutive ranks per node):
    the same three steps in two levels -- reduce-scatter inside the node (RCCL rides xGMI there),
    reduce-scatter of that 1/L chunk between nodes, ``shard_sgd`` on the 1/W shard, all-gather
    between nodes, all-gather inside the node. Each rank sends 1/L of the bucket over the
    inter-node network instead of all of it (Horovod's hierarchical allreduce, sharded);
  - ``"auto"``: xgmi when ``xgmi.usable`` and the communicator comes up on every rank; else hier
    when the job spans several nodes of more than one rank each (``local_size`` or
    ``LOCAL_WORLD_SIZE``); else rccl;
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
owns; :meth:`state_dict` reassembles them.
"""
from __future__ import annotations

import contextlib
import os
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

from ..ops.optim import _same_memory_order
from ..runtime import heartbeat

Tensor = torch.Tensor
_BF16, _F32 = torch.bfloat16, torch.float32
_ALIGN = {_BF16: 8, _F32: 4}          # 16-byte slots


def _pad(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class _Range:
    """One dtype's part of a bucket: its parameters' slots in that dtype's region."""

    def __init__(self, dtype, gi, params, offsets, start, end):
        self.dtype, self.gi = dtype, gi            # element dtype and param-group index
        self.params, self.offsets = params, offsets
        self.start, self.end = start, end          # region-relative, element units of `dtype`


class _Bucket:
    def __init__(self, ranges: List[_Range]):
        self.ranges = ranges                        # bf16 first, then fp32 (each optional)
        self.params = [p for r in ranges for p in r.params]
        self.pending = set(id(p) for p in self.params)
        self.launched = False

    @property
    def dtypes(self):
        return {r.dtype for r in self.ranges}

    @property
    def dtype(self):
        """The bucket's element dtype if it has one sub-range (else "mixed")."""
        return self.ranges[0].dtype if len(self.ranges) == 1 else "mixed"


class ShardedMasterSGD:
    """Momentum SGD (torch.optim.SGD semantics, dampening 0) sharded over the data-parallel ranks.

    ``params``: tensors, or torch-style param-group dicts (``{"params": [...], "weight_decay":
    0.0, "weights": "fp32"}``) whose ``lr`` / ``momentum`` / ``weight_decay`` override the
    defaults. ``weights`` (default ``"bf16"``) is the dtype the group's parameters are kept in:
    bf16 weights with fp32 masters (the parameters are converted in place), or fp32 weights that
    are their own masters. Parameters must be contiguous or channels_last; CUDA tensors (CPU
    tensors with ``backend="rccl"`` over gloo, for tests). ``order``: the parameters in model
    (registration) order, which decides the buckets (default: the param groups' order)."""

    def __init__(self, params: Iterable, lr: float, momentum: float = 0.0,
                 weight_decay: float = 0.0, bucket_mb: float = 16.0, group=None,
                 timeout_s: float = 60.0, overlap: bool = True, backend: str = "auto",
                 order: Optional[Iterable[Tensor]] = None, last_bucket_mb: Optional[float] = None,
                 rccl_reduce_fp32: Optional[bool] = None, local_size: Optional[int] = None):
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
        if backend not in ("auto", "xgmi", "rccl", "hier"):
            raise ValueError(f"backend must be auto, xgmi, rccl or hier (got {backend!r})")
        self.state: dict = {}   # Horovod's broadcast_optimizer_state finds nothing to send: the
        #                         masters are derived from the (already broadcast) weights
        self.group = group
        self.overlap = bool(overlap)
        self._no_sync = False
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = self.params[0].device
        self.device = dev
        kind_of = {}
        for gi, g in enumerate(self.param_groups):
            kind = {"bf16": _BF16, "fp32": _F32}.get(raw_groups[gi].get("weights", "bf16"))
            if kind is None:
                raise ValueError("param group 'weights' must be 'bf16' or 'fp32'")
            g["weights"] = "bf16" if kind == _BF16 else "fp32"
            for p in g["params"]:
                kind_of[id(p)] = (kind, gi)
                if p.device != dev:
                    raise ValueError("ShardedMasterSGD parameters must share one device")
                if not p.is_floating_point():
                    raise TypeError(f"ShardedMasterSGD takes floating-point parameters, got "
                                    f"{p.dtype}")
                if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                    raise ValueError("parameters must be contiguous or channels_last")
        if dev.type != "cuda" and backend == "xgmi":
            raise ValueError("ShardedMasterSGD on CPU tensors runs over gloo: backend 'rccl', "
                             "'hier' or 'auto'")
        requested = backend
        self.local_size = self._local_size(local_size, strict=backend == "hier")
        if backend == "auto":
            from . import xgmi
            backend = "xgmi" if dev.type == "cuda" and xgmi.usable(group) else self._flat_or_hier()
        self._intra = self._inter = None
        if backend == "hier":
            self._make_level_groups()
        model_order = self._model_order(order)
        last_mb = bucket_mb / 4 if last_bucket_mb is None else last_bucket_mb
        self.comm = None
        if backend == "xgmi":
            from .xgmi import XgmiComm, XgmiUnavailable
            self._form_buckets(model_order, kind_of, bucket_mb, last_mb, pad_to=1)
            floats = self.f0 + self.t32
            try:
                # collective: every rank learns together whether the peer mappings came up
                self.comm = XgmiComm(group, staging_elems=floats, param_elems=floats,
                                     timeout_s=timeout_s)
            except XgmiUnavailable:
                if requested == "xgmi":
                    raise
                backend = self._flat_or_hier()
                if backend == "hier":
                    self._make_level_groups()
        self.backend = backend
        # default: bf16 ring sums on the flat RCCL backend (the bytes xGMI moves), fp32 on the
        # hierarchical one, whose two levels would otherwise round the sum twice
        self.rccl_reduce_fp32 = (backend == "hier") if rccl_reduce_fp32 is None \
            else bool(rccl_reduce_fp32)
        if self.comm is None:
            # RCCL layout: sub-ranges padded to world x 16-byte slots (equal, aligned shards)
            self._form_buckets(model_order, kind_of, bucket_mb, last_mb, pad_to=self.world)
            floats = self.f0 + self.t32
            wbuf = torch.zeros(floats, dtype=_F32, device=dev)
            buf = torch.zeros(floats, dtype=_F32, device=dev)
            self._rs_out = torch.zeros(self._max_shard_words(), dtype=_F32, device=dev)
            self._rs_wide = (torch.zeros(self._max_range_elems(_BF16), dtype=_F32, device=dev)
                             if self.rccl_reduce_fp32 else None)
            self._rs_mid = (torch.zeros(self._max_chunk_words(), dtype=_F32, device=dev)
                            if self._intra is not None else None)
        else:
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
                p.grad = None       # flat buffer, fp32 master in self.master)
        self._next = 0          # index of the next bucket to launch (strict bucket order)
        self.stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    # ------------------------------------------------------------------------------- layout
    def _model_order(self, order) -> List[Tensor]:
        if order is None:
            return list(self.params)
        mine = {id(p) for p in self.params}
        seen, out = set(), []
        for p in order:
            if id(p) in mine and id(p) not in seen:
                out.append(p)
                seen.add(id(p))
        out += [p for p in self.params if id(p) not in seen]   # not in `order`: appended
        return out

    def _form_buckets(self, model_order, kind_of, bucket_mb, last_mb, pad_to):
        """Buckets in readiness order. Built from the INPUT side (model order): the first group
        closes at ``last_mb`` (it is ready last and nothing overlaps its update), the others at
        ``bucket_mb``; a group also closes when a parameter's param group differs from the one
        its dtype's sub-range already has (one set of hyperparameters per sub-range). With
        ``pad_to`` > 1 every sub-range is padded to a multiple of pad_to slots, so RCCL's
        reduce-scatter splits it into equal, aligned shards."""
        cap = max(1, int(bucket_mb * 2**20))
        first_cap = max(1, int(last_mb * 2**20))
        groups, cur, cur_bytes, cur_gi = [], [], 0, {}
        for p in model_order:
            dt, gi = kind_of[id(p)]
            if cur and cur_gi.get(dt, gi) != gi:
                groups.append(cur)
                cur, cur_bytes, cur_gi = [], 0, {}
            cur.append(p)
            cur_gi[dt] = gi
            cur_bytes += p.numel() * (2 if dt == _BF16 else 4)
            if cur_bytes >= (first_cap if not groups else cap):
                groups.append(cur)
                cur, cur_bytes, cur_gi = [], 0, {}
        if cur:
            groups.append(cur)
        self.offsets = {}
        self.buckets: List[_Bucket] = []
        size = {_BF16: 0, _F32: 0}
        for grp in reversed(groups):                 # readiness order
            ranges = []
            for dt in (_BF16, _F32):
                ps = [p for p in reversed(grp) if kind_of[id(p)][0] == dt]
                if not ps:
                    continue
                start, offs = size[dt], []
                for p in ps:
                    offs.append(size[dt])
                    self.offsets[id(p)] = size[dt]
                    size[dt] += _pad(p.numel(), _ALIGN[dt])
                size[dt] = start + _pad(size[dt] - start, _ALIGN[dt] * pad_to)
                ranges.append(_Range(dt, kind_of[id(ps[0])][1], ps, offs, start, size[dt]))
            self.buckets.append(_Bucket(ranges))
        self.t16, self.t32 = size[_BF16], size[_F32]
        self.f0 = _pad((self.t16 + 1) // 2, 4)            # fp32 region start (floats)

    def _local_size(self, local_size, strict: bool) -> int:
        """Ranks per node for the hierarchical backend (``LOCAL_WORLD_SIZE`` by default: torchrun
        numbers a node's ranks consecutively). Only ``backend='hier'`` requires it to divide the
        world; otherwise a non-dividing value (uneven nodes) just rules the hierarchy out."""
        if local_size is None:
            local_size = int(os.environ.get("LOCAL_WORLD_SIZE", self.world))
        local_size = int(local_size)
        if local_size < 1 or self.world % local_size:
            if strict:
                raise ValueError(f"local_size {local_size} must divide the world size "
                                 f"{self.world}")
            return self.world
        return local_size

    def _flat_or_hier(self) -> str:
        """The RCCL form ``auto`` picks: two-level when the job spans several equal nodes."""
        return "hier" if 1 < self.local_size < self.world else "rccl"

    def _make_level_groups(self) -> None:
        """One group per node (its L consecutive ranks) and one per local rank (the same local
        rank on every node). Collective: every rank creates every group, in the same order."""
        L, W = self.local_size, self.world
        if not 1 < L < W:
            raise ValueError(f"backend='hier' needs 1 < local_size < world (got local_size {L}, "
                             f"world {W})")
        granks = (dist.get_process_group_ranks(self.group) if self.group is not None
                  else list(range(W)))
        self.nodes = W // L
        self.node, self.lrank = self.rank // L, self.rank % L
        for k in range(self.nodes):
            g = dist.new_group([granks[k * L + l] for l in range(L)])
            if k == self.node:
                self._intra = g
        for l in range(L):
            g = dist.new_group([granks[k * L + l] for k in range(self.nodes)])
            if l == self.lrank:
                self._inter = g

    def _shard_index(self, rank: int) -> int:
        """Which 1/W slice of every sub-range ``rank`` owns: the flat backend slices in rank
        order; the hierarchical one gives local rank l the node-level chunk l, of which node k
        owns slice k."""
        if self._intra is None:
            return rank
        return (rank % self.local_size) * self.nodes + rank // self.local_size

    def _max_chunk_words(self) -> int:
        """fp32 words of the largest node-level (1/L) reduce-scatter output."""
        L = self.local_size
        m16 = self._max_range_elems(_BF16) // L
        m32 = self._max_range_elems(_F32) // L
        return max(4, m16 if self.rccl_reduce_fp32 else (m16 + 1) // 2, m32)

    def _max_range_elems(self, dtype) -> int:
        return max([r.end - r.start for b in self.buckets for r in b.ranges if r.dtype == dtype]
                   + [0])

    def _max_shard_words(self) -> int:
        """fp32 words of the largest reduce-scatter output (a bf16 shard fits in half)."""
        m16 = self._max_range_elems(_BF16) // max(1, self.world)
        m32 = self._max_range_elems(_F32) // max(1, self.world)
        return max(4, m16 if self.rccl_reduce_fp32 else (m16 + 1) // 2, m32)

    # ----------------------------------------------------------------------------------------
    @staticmethod
    def _view(flat: Tensor, p: Tensor, off: int) -> Tensor:
        return torch.as_strided(flat, p.shape, p.stride(), flat.storage_offset() + off)

    def _stream_ctx(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else \
            contextlib.nullcontext()

    def _launch(self, b: _Bucket) -> None:
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream())
        with self._stream_ctx():
            dst, src = [], []
            for r in b.ranges:
                stage = self.stage if r.dtype == _BF16 else self.stage32
                for p, o in zip(r.params, r.offsets):
                    v = self._view(stage, p, o)
                    if p.grad is None:
                        v.zero_()          # unused parameter this step: zero gradient (Horovod)
                        continue
                    gr = p.grad
                    if gr.dtype != p.dtype or not _same_memory_order(gr, p):
                        raise RuntimeError(
                            "ShardedMasterSGD: gradients must have the parameter's dtype and "
                            f"memory order (param {p.dtype} {tuple(p.shape)} {p.stride()}, grad "
                            f"{gr.dtype} {gr.stride()})")
                    if self.stream is not None:
                        gr.record_stream(self.stream)
                    dst.append(v)
                    src.append(gr)
            if dst:
                torch._foreach_copy_(dst, src)
            for r in b.ranges:
                g = self.param_groups[r.gi]
                lr, mu, wd = float(g["lr"]), float(g["momentum"]), float(g["weight_decay"])
                if self.comm is not None:
                    self._update_xgmi(r, lr, mu, wd)
                else:
                    self._update_rccl(r, lr, mu, wd)
        b.launched = True

    def _update_xgmi(self, r: _Range, lr, mu, wd) -> None:
        if r.dtype == _BF16:
            self.comm.peers.sgd_bf16(self.master, self.mom, r.start, r.end - r.start, lr, mu, wd,
                                     1.0 / self.world)
        else:
            self.comm.peers.sgd_f32(self.mom32[r.start:r.end], self.f0 + r.start,
                                    r.end - r.start, lr, mu, wd, 1.0 / self.world)

    def _update_rccl(self, r: _Range, lr, mu, wd) -> None:
        """reduce-scatter -> shard_sgd on the owned shard -> all-gather, on the current (comm)
        stream. Sub-ranges are padded to world x 16-byte slots: equal, aligned shards. The
        hierarchical backend does each collective in two levels (node, then between nodes)."""
        from ..ops import fused
        n = r.end - r.start
        sl = n // self.world
        lo = r.start + self._shard_index(self.rank) * sl
        scale = 1.0 / self.world
        if r.dtype == _BF16:
            if self.rccl_reduce_fp32:
                wide = self._rs_wide[:n]
                wide.copy_(self.stage[r.start:r.end])
                out = self._rs_out[:sl]
                self._reduce_scatter(out, wide)
            else:
                out = self._rs_out.view(_BF16)[:sl]
                self._reduce_scatter(out, self.stage[r.start:r.end])
            fused.shard_sgd(out, self.master[lo:lo + sl], self.mom[lo:lo + sl],
                            self.wbf[lo:lo + sl], lr=lr, momentum=mu, weight_decay=wd,
                            scale=scale)
            self._all_gather(self.wbf, r.start, n, lo, sl)
        else:
            out = self._rs_out[:sl]
            self._reduce_scatter(out, self.stage32[r.start:r.end])
            fused.shard_sgd(out, self.w32[lo:lo + sl], self.mom32[lo:lo + sl], None, lr=lr,
                            momentum=mu, weight_decay=wd, scale=scale)
            self._all_gather(self.w32, r.start, n, lo, sl)

    def _reduce_scatter(self, out: Tensor, inp: Tensor) -> None:
        if self._intra is None:
            dist.reduce_scatter_tensor(out, inp, group=self.group)
            return
        # node level: local rank l gets chunk l (summed over the node); then the nodes
        # reduce-scatter that chunk, node k keeping slice k of it
        mid = self._rs_mid.view(inp.dtype)[: inp.numel() // self.local_size]
        dist.reduce_scatter_tensor(mid, inp, group=self._intra)
        dist.reduce_scatter_tensor(out, mid, group=self._inter)

    def _all_gather(self, flat: Tensor, start: int, n: int, lo: int, sl: int) -> None:
        """Every rank's updated slice [lo, lo + sl) into ``flat[start:start + n]``."""
        def gather(out, mine, group):
            # in place on RCCL (the send buffer is this rank's slot of the receive buffer);
            # gloo gets a copy
            dist.all_gather_into_tensor(out, mine.clone() if out.device.type == "cpu" else mine,
                                        group=group)
        if self._intra is None:
            gather(flat[start:start + n], flat[lo:lo + sl], self.group)
            return
        chunk = n // self.local_size
        c0 = start + self.lrank * chunk
        gather(flat[c0:c0 + chunk], flat[lo:lo + sl], self._inter)
        gather(flat[start:start + n], flat[c0:c0 + chunk], self._intra)

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
            self._launch_ready_prefix()

    def _launch_ready_prefix(self) -> None:
        """Launch buckets strictly in index order: bucket i only once 0..i-1 have launched. The
        RCCL / hier backends need every rank to issue its collectives in the same order, and a
        rank whose gradients arrive in another order (data-dependent control flow, an unused
        parameter) would otherwise reduce one bucket against a peer's different one."""
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if b.pending or b.launched:
                if b.launched:
                    self._next += 1
                    continue
                return
            self._launch(b)
            self._next += 1

    def _join(self) -> None:
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)

    def _reset(self) -> None:
        if any(b.launched for b in self.buckets):
            # updates already issued on the comm stream: later work on the main stream (the
            # next forward reads the weights) must be ordered after them
            self._join()
        for b in self.buckets:
            b.launched = False
            b.pending = set(id(p) for p in b.params)
        self._next = 0

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
        self._join()
        for b in self.buckets:
            b.launched = False
            b.pending = set(id(p) for p in b.params)
        self._next = 0
        heartbeat.beat()
        return None

    # ----------------------------------------------------------------------- state / sharding
    def shard_ranges(self, rank: int | None = None, dtype=_BF16):
        """Region-relative [lo, hi) element ranges this rank owns, one per sub-range of
        ``dtype``."""
        r = self.rank if rank is None else rank
        out = []
        for b in self.buckets:
            for rg in b.ranges:
                if rg.dtype != dtype:
                    continue
                n = rg.end - rg.start
                if self.comm is None:
                    sl = n // self.world
                    s = self._shard_index(r)
                    out.append((rg.start + s * sl, rg.start + (s + 1) * sl))
                elif dtype == _BF16:
                    out.append(tuple(self.comm.ext.ccl_sgd_shard(rg.start, n, self.world, r)))
                else:
                    lo, hi = self.comm.ext.ccl_sgd_f32_shard(self.f0 + rg.start, n, self.world, r)
                    out.append((lo - self.f0, hi - self.f0))
        return out

    @torch.no_grad()
    def _gathered(self, flat: Tensor, dtype) -> Tensor:
        """Full-length copy of a sharded fp32 array: owned chunks from every rank (sum of the
        rank-masked arrays; collective)."""
        mine = torch.zeros_like(flat)
        for lo, hi in self.shard_ranges(dtype=dtype):
            mine[lo:hi] = flat[lo:hi]
        if mine.numel():
            if self.comm is not None:
                self.comm.all_reduce_(mine)
            elif self.world > 1:
                dist.all_reduce(mine, group=self.group)
        return mine

    def _logical(self, flat: Tensor, p: Tensor) -> Tensor:
        return self._view(flat, p, self.offsets[id(p)]).contiguous()

    def state_dict(self) -> dict:
        """fp32 masters + momentum per parameter in logical layout, and the param groups'
        hyperparameters (collective: every rank must call it)."""
        self._join()
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
        self._join()
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
        """Make every parameter a view into the flat weight buffer again (after a
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
        was re-bound (``p.data = t``) is copied back into the flat buffer and re-bound to
        it, so the all-gathered weights reach the model again. Momentum is kept."""
        self._join()
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
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        if self.comm is not None:
            self.comm.close()
