"""Autograd wrappers so ordinary PyTorch models can use the fused HIP kernels.

``FusedLinear``: y = dropout(relu(x @ Wᵀ + b)) with W stored [out, in]. Forward = one linear_fwd launch; backward = wgrad_grouped (dW, db in one
launch) + a plain library GEMM for dX (hipBLASLt via torch.mm). W is [out, in] (nn.Linear).
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import fused


def _kernel_ok(x: torch.Tensor, W: torch.Tensor) -> bool:
    return (x.dim() == 2 and W.shape[1] % 4 == 0 and x.dtype in (torch.float32, torch.uint8)
            and W.dtype == torch.float32)


class _FusedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, act, keep_prob, seed, step):
        x = x.contiguous()
        Y = torch.empty(x.shape[0], W.shape[0], device=x.device, dtype=torch.float32)
        fused.linear_fwd(x, W, Y, b, act=act, keep_prob=keep_prob, seed=seed, step=step)
        ctx.save_for_backward(x, W, Y)
        ctx.act, ctx.keep_prob, ctx.has_bias = act, keep_prob, b is not None
        return Y

    @staticmethod
    def backward(ctx, dY):
        x, W, Y = ctx.saved_tensors
        inv_keep = 1.0 / ctx.keep_prob if ctx.keep_prob < 1.0 else 1.0
        if ctx.act == 1:
            # Y = relu(z)*mask/keep  ->  Y > 0 exactly where both relu' and the keep mask are 1.
            dZ = torch.where(Y > 0, dY * inv_keep, torch.zeros_like(dY)).contiguous()
        else:
            dZ = dY.contiguous()
        dW = torch.empty_like(W)
        db = torch.empty(W.shape[0], device=W.device, dtype=torch.float32) if ctx.has_bias else None
        fused.wgrad_grouped([x], [dZ], [dW], [db], x_scales=[1.0], gather=[False], mode=0)
        dx = dZ @ W if ctx.needs_input_grad[0] else None
        return dx, dW, db, None, None, None, None


def fused_linear(x, W, b=None, act: int = 1, keep_prob: float = 1.0, seed: int = 0,
                 step: torch.Tensor | None = None):
    if act == 0 and keep_prob < 1.0:
        raise ValueError("fused dropout requires act=relu (mask is recovered from the output)")
    if not _kernel_ok(x, W):
        z = x.float() @ W.t()
        if b is not None:
            z = z + b
        if act == 1:
            z = torch.relu(z)
        return z
    return _FusedLinearFn.apply(x, W, b, act, keep_prob, seed, step)


class FusedLinear(nn.Module):
    """Linear(+ReLU)(+dropout) layer on the fused HIP kernels; weight is [out, in]."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 activation: str = "relu", keep_prob: float = 1.0, seed: int = 0):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        self.act = {"relu": 1, "none": 0, None: 0}[activation]
        self.keep_prob = keep_prob
        self.seed = seed
        self.register_buffer("step", torch.zeros(1, dtype=torch.int64), persistent=False)
        bound = 1.0 / math.sqrt(in_features)
        nn.init.uniform_(self.weight, -bound, bound)

    def forward(self, x):
        keep = self.keep_prob if self.training else 1.0
        y = fused_linear(x, self.weight, self.bias, self.act, keep, self.seed, self.step)
        if self.training and keep < 1.0:
            self.step.add_(1)
        return y


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.contiguous().float()
        n = logits.shape[0]
        loss, dl = fused.softmax_xent(logits, labels.contiguous().long(), 1.0 / n, True)
        ctx.save_for_backward(dl)
        return loss.mean()

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None


def fused_cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy; forward+backward computed by one HIP launch."""
    return _XentFn.apply(logits, labels)
