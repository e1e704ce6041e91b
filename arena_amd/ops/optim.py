"""Mixed-precision optimizers over the native multi-tensor kernels.

:class:`MasterSGD` keeps conv/linear weights as bf16 parameters (views into one flat bf16 buffer)
and their fp32 master copies + momentum in flat fp32 buffers. The bf16 weights feed the MFMA
convolutions directly, so a bf16-autocast step has no per-weight fp32->bf16 cast in the forward
and no bf16->fp32 gradient cast in the backward; the update is one multi-tensor kernel
(``mt_sgd_master`` in ``csrc/ops/mlp_kernels.hip``). The reference trains through TF inside its
Horovod image (``charts/tf-horovod/values.yaml``); tf_cnn_benchmarks' fp16 mode keeps fp32
master variables the same way.
"""
from __future__ import annotations

from typing import Iterable, List

import torch

from . import fused

Tensor = torch.Tensor


class MasterSGD:
    """Momentum SGD (torch.optim.SGD semantics, dampening 0) with fp32 master weights.

    Converts every parameter in ``params`` to bf16 in place (``p.data`` becomes a view into the
    flat bf16 buffer with the parameter's own strides, so channels_last weights stay
    channels_last)."""

    def __init__(self, params: Iterable[Tensor], lr: float, momentum: float = 0.0,
                 weight_decay: float = 0.0):
        self.params: List[Tensor] = list(params)
        if not self.params:
            raise ValueError("MasterSGD needs at least one parameter")
        self.lr, self.momentum, self.weight_decay = float(lr), float(momentum), float(weight_decay)
        self.offsets: List[int] = []
        total = 0
        for p in self.params:
            if not (p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)):
                raise ValueError("MasterSGD parameters must be contiguous or channels_last")
            if p.numel() % 4:
                raise ValueError(f"MasterSGD needs numel % 4 == 0 (got {tuple(p.shape)})")
            self.offsets.append(total)
            total += p.numel()
        dev = self.params[0].device
        self.master = torch.empty(total, dtype=torch.float32, device=dev)
        self.mom = torch.zeros(total, dtype=torch.float32, device=dev)
        self.wbf = torch.empty(total, dtype=torch.bfloat16, device=dev)
        with torch.no_grad():
            for p, off in zip(self.params, self.offsets):
                self.master.as_strided(p.shape, p.stride(), off).copy_(p)
                v = self.wbf.as_strided(p.shape, p.stride(), off)
                v.copy_(p)
                p.data = v
                p.grad = None

    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    @torch.no_grad()
    def step(self) -> None:
        grads, offs = [], []
        for p, off in zip(self.params, self.offsets):
            g = p.grad
            if g is None:
                continue
            if g.dtype != torch.bfloat16 or not _same_memory_order(g, p):
                raise RuntimeError("MasterSGD: gradient must be bf16 with the parameter's strides "
                                   f"(param {tuple(p.shape)} strides {p.stride()}, grad "
                                   f"{g.dtype} strides {g.stride()})")
            grads.append(g)
            offs.append(off)
        if grads:
            fused.mt_sgd_master(grads, offs, self.master, self.mom, self.wbf, lr=self.lr,
                                momentum=self.momentum, weight_decay=self.weight_decay)

    def _views(self, flat: Tensor):
        return [flat.as_strided(p.shape, p.stride(), off) for p, off in zip(self.params,
                                                                            self.offsets)]

    @torch.no_grad()
    def sync_from_params(self) -> None:
        """Re-derive the fp32 masters from the current (bf16) parameter values.

        Call this after ``model.load_state_dict(...)`` on a model whose optimizer already exists:
        otherwise the next :meth:`step` overwrites the loaded weights with the stale masters.
        (Momentum is left as is; load the optimizer state too to restore it.)"""
        for p, m, w in zip(self.params, self._views(self.master), self._views(self.wbf)):
            if p.data_ptr() != w.data_ptr():
                # the parameter's data was re-bound (``p.data = t``): adopt its values and
                # make it a view into the flat bf16 buffer again. (``load_state_dict(...,
                # assign=True)`` replaces the Parameter objects themselves; like any torch
                # optimizer, MasterSGD must then be rebuilt.)
                w.copy_(p)
                p.data = w
            m.copy_(p)

    def master_params(self) -> List[Tensor]:
        """fp32 master weights, one tensor per parameter in logical (contiguous) layout."""
        return [m.contiguous() for m in self._views(self.master)]

    def state_dict(self) -> dict:
        """fp32 masters + momentum, one tensor per parameter in LOGICAL layout (independent of
        channels_last strides), so a checkpoint moves between NHWC and NCHW runs and CPU/GPU."""
        return {"master": self.master_params(),
                "momentum_buffer": [m.contiguous() for m in self._views(self.mom)],
                "shapes": [tuple(p.shape) for p in self.params],
                "lr": self.lr, "momentum": self.momentum, "weight_decay": self.weight_decay}

    @torch.no_grad()
    def load_state_dict(self, state: dict) -> None:
        masters, moms = state["master"], state["momentum_buffer"]
        if isinstance(masters, Tensor) or isinstance(moms, Tensor):
            raise ValueError("MasterSGD state is in the old flat format (memory-order dependent); "
                             "re-save it with this version")
        n = len(self.params)
        if len(masters) != n or len(moms) != n:
            raise ValueError(f"MasterSGD state holds {len(masters)} masters / {len(moms)} momentum "
                             f"buffers for {n} parameters")
        for i, (p, a, b) in enumerate(zip(self.params, masters, moms)):
            if tuple(a.shape) != tuple(p.shape) or tuple(b.shape) != tuple(p.shape):
                raise ValueError(f"MasterSGD state: parameter {i} has shape {tuple(p.shape)}, "
                                 f"state has {tuple(a.shape)} / {tuple(b.shape)}")
        for m, a in zip(self._views(self.master), masters):
            m.copy_(a)
        for m, b in zip(self._views(self.mom), moms):
            m.copy_(b)
        self.lr = float(state["lr"])
        self.momentum = float(state.get("momentum", self.momentum))
        self.weight_decay = float(state.get("weight_decay", self.weight_decay))
        self.wbf.copy_(self.master)   # bf16 weights are views into wbf


def _same_memory_order(g: Tensor, p: Tensor) -> bool:
    """True if ``g`` is dense and walks memory in the same element order as ``p``.

    Strides of size-1 dims are irrelevant (autograd's AccumulateGrad keeps such gradients as they
    come: a channels_last gradient of a [Cout, Cin, 1, 1] weight is contiguous in both senses)."""
    if g.shape != p.shape:
        return False
    if not (g.is_contiguous() or g.is_contiguous(memory_format=torch.channels_last)):
        return False
    return all(gs == ps for gs, ps, n in zip(g.stride(), p.stride(), p.shape) if n > 1)


class OptimizerGroup:
    """Steps several optimizers as one (e.g. MasterSGD for weights + torch SGD for BN/bias)."""

    def __init__(self, *opts):
        self.opts = opts

    def zero_grad(self, set_to_none: bool = True) -> None:
        for o in self.opts:
            o.zero_grad(set_to_none=set_to_none)

    def step(self) -> None:
        for o in self.opts:
            o.step()

    def state_dict(self) -> dict:
        return {"opts": [o.state_dict() for o in self.opts]}

    def load_state_dict(self, state: dict) -> None:
        if len(state["opts"]) != len(self.opts):
            raise ValueError(f"OptimizerGroup state holds {len(state['opts'])} optimizers, "
                             f"this group has {len(self.opts)}")
        for o, st in zip(self.opts, state["opts"]):
            o.load_state_dict(st)
