"""NHWC bf16 convolutions on the hand-written MFMA implicit-GEMM kernel (``conv_kernels.hip``).

The ResNet family of the reference's Horovod benchmark image (charts/tf-horovod/README.md:66-69)
spends half its step in convolutions. ``conv2d_fwd`` runs one on the gfx950 kernel;
``conv2d_bwd_data`` runs the backward-data pass of a stride-1 convolution through the SAME kernel:

    dX = conv(dY, W'),  W'[ci][r][s][co] = W[co][R-1-r][S-1-s][ci],  padding R-1-pad

(``flip_weight``), so one tuned GEMM serves both directions. Shapes the kernel does not cover
(C or Cout not a multiple of 64, e.g. the 3-channel stem) belong to MIOpen: ``kernel_ok`` says
which. The variant picks the block's output tile (0: 128x128, 1: 128x64, 2: 64x128, 3: 64x64);
``pick_variant`` is the fill-the-chip heuristic, ``Conv2dNHWC`` autotunes per shape.
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _ext

Tensor = torch.Tensor
TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64)}
_CUS = 256


def out_hw(h: int, w: int, r: int, s: int, stride: int, pad: int) -> Tuple[int, int]:
    return (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1


def kernel_ok(x: Tensor, w: Tensor, stride: int, pad: int) -> bool:
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and w.shape[1] == x.shape[1] and stride >= 1 and pad >= 0
            and x.shape[2] + 2 * pad >= w.shape[2] and x.shape[3] + 2 * pad >= w.shape[3])


def variants_for(cout: int):
    return [v for v, (_, bn) in TILES.items() if cout % bn == 0]


def pick_variant(m: int, cout: int) -> int:
    """Largest tile that still gives every CU at least two blocks; else the most blocks."""
    best, best_blocks = None, 0
    for v in (0, 1, 2, 3):
        bm, bn = TILES[v]
        if cout % bn:
            continue
        blocks = -(-m // bm) * (cout // bn)
        if blocks >= 2 * _CUS:
            return v
        if blocks > best_blocks:
            best, best_blocks = v, blocks
    return best


def conv2d_fwd(x: Tensor, w: Tensor, stride: int = 1, pad: int = 0, variant: int = -1) -> Tensor:
    """y = conv2d(x, w) for channels_last bf16 x [N,C,H,W] and w [Cout,C,R,S]."""
    x = x.contiguous(memory_format=torch.channels_last)
    w = w.contiguous(memory_format=torch.channels_last)
    if variant < 0:
        ho, wo = out_hw(x.shape[2], x.shape[3], w.shape[2], w.shape[3], stride, pad)
        variant = pick_variant(x.shape[0] * ho * wo, w.shape[0])
    return _ext.load().conv_fwd(x, w, int(stride), int(pad), int(variant))


def flip_weight(w: Tensor) -> Tensor:
    """W' [Cin, Cout, R, S] (channels_last) with W'[ci, co, r, s] = W[co, ci, R-1-r, S-1-s]."""
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


def conv2d_bwd_data(dy: Tensor, w: Tensor, pad: int, variant: int = -1) -> Tensor:
    """dX of a stride-1 convolution (same spatial size when pad = (R-1)/2)."""
    r = w.shape[2]
    return conv2d_fwd(dy, flip_weight(w), 1, r - 1 - pad, variant)
