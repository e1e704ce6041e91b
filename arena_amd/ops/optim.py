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
            if g.dtype != torch.bfloat16 or g.stride() != p.stride():
                raise RuntimeError("MasterSGD: gradient must be bf16 with the parameter's strides")
            grads.append(g)
            offs.append(off)
        if grads:
            fused.mt_sgd_master(grads, offs, self.master, self.mom, self.wbf, lr=self.lr,
                                momentum=self.momentum, weight_decay=self.weight_decay)

    def state_dict(self) -> dict:
        """fp32 masters + momentum (the bf16 parameters are derived from the masters)."""
        return {"master": self.master.clone(), "momentum_buffer": self.mom.clone(),
                "lr": self.lr, "momentum": self.momentum, "weight_decay": self.weight_decay}

    @torch.no_grad()
    def load_state_dict(self, state: dict) -> None:
        if state["master"].numel() != self.master.numel():
            raise ValueError("MasterSGD state does not match this parameter set")
        self.master.copy_(state["master"])
        self.mom.copy_(state["momentum_buffer"])
        self.lr = float(state["lr"])
        self.momentum = float(state.get("momentum", self.momentum))
        self.weight_decay = float(state.get("weight_decay", self.weight_decay))
        self.wbf.copy_(self.master)   # bf16 weights are views into wbf


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
        for o, st in zip(self.opts, state["opts"]):
            o.load_state_dict(st)
