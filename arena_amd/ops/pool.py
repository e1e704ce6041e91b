"""NHWC max pooling with a saved in-window argmax (``csrc/ops/pool_kernels.hip``).

``MaxPool2dNHWC`` is a drop-in ``nn.MaxPool2d`` (dilation 1, floor mode). On an MI355X with a
channels_last bf16/fp32 input whose C is a multiple of 8 it runs the HIP kernels: the forward
stores a uint8 window position per output element, and the backward gathers each input's
gradient from the windows that picked it (no atomics, no zero-fill). Anything else, including
CPU tensors, runs ``F.max_pool2d``, which is also the numerics reference.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import _ext


def kernel_ok(x: torch.Tensor, k: int, s: int, p: int) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.numel() > 0 and x.shape[1] % 8 == 0
            and x.dtype in (torch.bfloat16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last)
            and 1 <= k <= 15 and s >= 1 and 0 <= 2 * p <= k
            and (k + s - 1) // s <= 3   # <= 3x3 windows cover an input (backward instantiations)
            and x.shape[2] + 2 * p >= k and x.shape[3] + 2 * p >= k)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, pos = _ext.load().maxpool_fwd(x, k, s, p)
        ctx.save_for_backward(pos)
        ctx.geom = (x.shape[2], x.shape[3], k, s, p)
        ctx.mark_non_differentiable(pos)
        return y

    @staticmethod
    def backward(ctx, dy):
        (pos,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        return _ext.load().maxpool_bwd(dy, pos, *ctx.geom), None, None, None


def max_pool2d(x: torch.Tensor, kernel_size: int, stride: int, padding: int = 0) -> torch.Tensor:
    if kernel_ok(x, kernel_size, stride, padding):
        return _MaxPoolFn.apply(x, kernel_size, stride, padding)
    return F.max_pool2d(x, kernel_size, stride, padding)


class MaxPool2dNHWC(nn.Module):
    """``nn.MaxPool2d(k, stride, padding)`` with the fused NHWC kernels on MI355X."""

    def __init__(self, kernel_size: int, stride: int | None = None, padding: int = 0):
        super().__init__()
        self.kernel_size = kernel_size
        self.stride = stride if stride is not None else kernel_size
        self.padding = padding

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return max_pool2d(x, self.kernel_size, self.stride, self.padding)

    def extra_repr(self) -> str:
        return f"kernel_size={self.kernel_size}, stride={self.stride}, padding={self.padding}"


class _GlobalAvgPoolFn(torch.autograd.Function):
    """Mean over H, W of a channels_last activation, [N, C, H, W] -> [N, C]. The backward writes
    the (broadcast) gradient straight into a channels_last tensor: the stock adaptive-pool
    backward materialises it NCHW and the next layer's channels_last conversion then transposes
    25.7 MB at ResNet-50 bs128 (14 + 45.5 us per step; a broadcast copy into channels_last 5 + 22
    us, profiles/r6_kernel_neighbors.txt; gap_bwd's single write pass replaces both)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        n, c, h, w = ctx.shape
        if c % 8 == 0 and g.dtype in (torch.bfloat16, torch.float32):
            return _ext.load().gap_bwd(g.contiguous(), h, w)   # one write pass (pool_kernels.hip)
        return (g * (1.0 / (h * w)))[:, :, None, None].expand(n, c, h, w).contiguous(
            memory_format=torch.channels_last)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)`` for channels_last GPU tensors; anything
    else runs the stock op."""
    if x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        loss, lse = _ext.load().xent_fwd(logits, labels)
        ctx.save_for_backward(logits, labels, lse)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse = ctx.saved_tensors
        return _ext.load().xent_bwd(logits, labels, lse, g.float().reshape(1)), None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """``F.cross_entropy(logits, labels)`` (mean reduction, fp32 result, no ignore_index / label
    smoothing) on the GPU through the ``pool_kernels.hip`` xent kernels: forward per-row loss +
    log-sum-exp (one wave per row) and their mean, backward one elementwise pass in the logits'
    dtype. Anything else runs the stock op."""
    if (logits.is_cuda and logits.dim() == 2 and labels.dim() == 1
            and labels.dtype == torch.int64 and logits.dtype in (torch.bfloat16, torch.float32)):
        return _SoftmaxXentFn.apply(logits.contiguous(), labels.contiguous())
    return F.cross_entropy(logits.float(), labels)
