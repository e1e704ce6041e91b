"""NHWC bf16 convolutions on the hand-written MFMA implicit-GEMM kernel (``conv_kernels.hip``).

The ResNet family of the reference's Horovod benchmark image (charts/tf-horovod/README.md:66-69)
spends half its step in convolutions. ``conv2d_fwd`` runs one on the gfx950 kernel;
``conv2d_bwd_data`` runs the backward-data pass of a stride-1 convolution through the SAME kernel:

    dX = conv(dY, W'),  W'[ci][r][s][co] = W[co][R-1-r][S-1-s][ci],  padding R-1-pad

(``flip_weight``), so one tuned GEMM serves both directions. Shapes the kernel does not cover
(C or Cout not a multiple of 64) fall back to MIOpen: ``kernel_ok`` says which. Strided
backward-data runs as parity-class phase convolutions (``conv2d_bwd_data_strided``) and the
3-channel 7x7/2 stem as a space-to-depth 4x4 convolution (``StemConv2d``), so a ResNet step needs
no MIOpen convolution at all -- which matters for hipGraph capture (docs/perf.md "MIOpen inside a
captured step"). The variant picks the block's output tile (0: 128x128, 1: 128x64, 2: 64x128,
3: 64x64); ``pick_variant`` is the fill-the-chip heuristic, ``Conv2dNHWC`` autotunes per shape
among the kernel variants (ARENA_CONV=miopen selects the library instead, for comparisons).
"""
from __future__ import annotations

import os
from typing import Tuple

import torch

from . import _ext, planstore

Tensor = torch.Tensor
TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64)}
# + 4: four-stage K pipeline (3 steps in flight); + 8: single stage buffer, serial K loop, high
# occupancy
TILES.update({v + d: t for v, t in list(TILES.items()) for d in (4, 8)})
# 12 / 13: 256x128 / 256x64 tiles on 8 waves, two stage buffers; 14 / 15: three
TILES.update({12: (256, 128), 13: (256, 64), 14: (256, 128), 15: (256, 64)})
# + 16 * (k - 1): the same tile with its K steps split over k blocks (in-kernel ticket reduction,
# bit-reproducible): for the layers whose tile count leaves CUs idle (14x14 / 7x7 at batch 128)
KSPLITS = (2, 3, 4, 6, 8)
TILES.update({v + 16 * (k - 1): TILES[v] for v in range(16) for k in KSPLITS})
# 4096 + i: the v2 tile kernel (conv_kernels.hip conv2_body): 32x32x16 MFMAs, 8-wave 256-row
# tiles (4-wave 128x128), two K steps in flight, epilogue through an fp32 LDS tile. Forward and
# backward-data (incl. the strided phases): plain, masked addend, BatchNorm statistics, BatchNorm-
# backward partials or sums (BNGradLink).
V2 = 4096
V2_TILES = {V2 + 0: (256, 128), V2 + 1: (256, 256), V2 + 2: (128, 128), V2 + 3: (256, 64),
            V2 + 4: (128, 256), V2 + 5: (128, 64), V2 + 6: (64, 64), V2 + 7: (64, 128),
            # serial single-buffer forms with wave-row epilogue bands: 4 waves per SIMD
            V2 + 8: (128, 128), V2 + 9: (128, 64), V2 + 10: (64, 128), V2 + 11: (64, 64)}
# 3x3 / stride 1 / pad 1 halo forms (width <= 63): the tile's input window is staged once per
# 64-channel chunk and the nine taps read it shifted (conv_kernels.hip Conv2Geo::HALO)
V2_HALO = {V2 + 12: (128, 128), V2 + 13: (128, 64),
           V2 + 14: (128, 64),   # 14: the window of <= 31-wide images (four blocks per CU)
           # 15: two groups of four waves split the 64-channel chunks (two waves per SIMD; even
           # chunk counts only)
           V2 + 15: (128, 128),
           # 16..18: eight waves, a 256-pixel or 256-channel tile per block (each weight tap
           # staged into LDS feeds twice the MFMAs of a 128x128 tile)
           V2 + 16: (256, 128), V2 + 17: (128, 256), V2 + 18: (256, 64)}
HALO_MAX_W = 63
HALO_SMALL = {V2 + v: 31 for v in (14, 15)}
HALO_SPLIT2 = {V2 + 15}
HALO_WIDE = {V2 + v for v in range(16, 19)}   # the 8-wave forms (set_halo_wide, for A/Bs)
_HALO_WIDE_ON = True
V2_TILES.update(V2_HALO)
TILES.update(V2_TILES)
_V2_ON = os.environ.get("ARENA_CONV_V2", "1") != "0"
_CUS = 256


def kvariant(v: int, ks: int) -> int:
    """Variant code of tile variant ``v`` (0..15) with its K steps split over ``ks`` blocks."""
    return v + 16 * (ks - 1)


def split_of(v: int) -> int:
    return 1 if v >= V2 else v // 16 + 1


def set_v2(on: bool) -> None:
    """A/B switch: offer the v2 tile kernel to the autotuner (part of the plan key)."""
    global _V2_ON
    _V2_ON = bool(on)


def v2_variants_for(cout: int):
    """v2 tile variants for ``cout`` output channels (forward / backward-data, incl. the strided
    phases); the halo forms come from ``halo_variants_for``."""
    return [v for v, (_, bn) in V2_TILES.items()
            if cout % bn == 0 and v not in V2_HALO] if _V2_ON else []


def set_halo_wide(on: bool) -> None:
    """A/B switch: offer the 8-wave halo forms to the autotuner (part of the plan key)."""
    global _HALO_WIDE_ON
    _HALO_WIDE_ON = bool(on)


def halo_variants_for(cout: int, k, stride: int, pad: int, width: int, cin: int | None = None):
    """The 3x3 halo forms, for a 3x3 / stride 1 / pad 1 convolution of a <= 63-wide image
    (``cin``: the input channels; the two-group forms need an even number of 64-channel chunks)."""
    if not _V2_ON or tuple(k) != (3, 3) or stride != 1 or pad != 1 or width > HALO_MAX_W:
        return []
    return [v for v, (_, bn) in V2_HALO.items()
            if cout % bn == 0 and width <= HALO_SMALL.get(v, HALO_MAX_W)
            and (v not in HALO_SPLIT2 or (cin is None or (cin // 64) % 2 == 0))
            and (_HALO_WIDE_ON or v not in HALO_WIDE)]


def out_hw(h: int, w: int, r: int, s: int, stride: int, pad: int) -> Tuple[int, int]:
    return (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1


def kernel_ok(x: Tensor, w: Tensor, stride: int, pad: int) -> bool:
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and w.shape[1] == x.shape[1] and stride >= 1 and pad >= 0
            # the stride-1 backward-data pass is a conv with padding R-1-pad: never negative
            and pad <= min(w.shape[2], w.shape[3]) - 1
            and x.shape[2] + 2 * pad >= w.shape[2] and x.shape[3] + 2 * pad >= w.shape[3])


def variants_for(cout: int):
    """Unsplit tile variants for ``cout`` output channels."""
    return [v for v, (_, bn) in TILES.items() if v < 16 and cout % bn == 0]


def split_variants_for(m: int, cout: int, ktot: int):
    """Split-K candidates for a GEMM of ``m`` rows, ``cout`` columns and ``ktot`` reduction: for
    tiles whose grid gives fewer than two blocks per CU, the splits that bring it to about 2 or 4
    blocks per CU with at least 4 K steps per slice."""
    out = []
    if os.environ.get("ARENA_CONV_KSPLIT", "1") == "0":
        return out
    steps = ktot // 64
    for v in variants_for(cout):
        if 4 <= v < 8 or v >= 14:
            continue   # the deep pipelines need long K loops: not split candidates
        bm, bn = TILES[v]
        tiles = -(-m // bm) * (cout // bn)
        if tiles >= 2 * _CUS or tiles > 65536:
            continue
        ks_set = set()
        for want in (2 * _CUS, 4 * _CUS):
            need = -(-want // tiles)
            ks = next((k for k in KSPLITS if k >= need), KSPLITS[-1])
            if steps // ks >= 4:
                ks_set.add(ks)
        out += [kvariant(v, k) for k in sorted(ks_set)]
    return out


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


def conv2d_fwd(x: Tensor, w: Tensor, stride: int = 1, pad: int = 0, variant: int = -1,
               with_stats: bool = False, addend: Tensor | None = None, bn=None,
               addmask: Tensor | None = None, final: bool = False,
               bn_acc: Tensor | None = None):
    """y = conv2d(x, w) (+ addend) for channels_last bf16 x [N,C,H,W] and w [Cout,C,R,S].

    with_stats: returns (y, (part, rpb)) where part holds per-tile BatchNorm partials of y
    (tile mean and sum of squared deviations per channel, ``rpb`` output pixels per tile), which
    ``BatchNormAct2d(..., stats=...)`` finalizes instead of re-reading y.
    addend: a bf16 tensor shaped like y, added to the fp32 sums before rounding (epilogue).
    addmask: uint8 bits (numel(y) / 8 bytes, bit i of byte v for element 8v + i, NHWC order):
    only the addend elements whose bit is set are added (a ReLU'd gradient, see GradJoin).
    bn: (bn_x, bn_mask or None, bn_mean) when y is the gradient of a BatchNorm layer's output:
    returns (y, (part, rpb)) with that BN's backward partials (sum g, sum g (bn_x - mean) per
    tile, g = y * mask) for its backward, which then skips its reduction pass; with ``bn_acc``
    (that BN's fp64 [2, C] backward sums) the epilogue adds them there instead and returns
    (y, None).
    final (with with_stats): the statistics come back finished, ``(y, FinishedStats)`` -- the
    epilogue's fp64 atomics + last-tile ticket replace the BN's finalize launch."""
    x = x.contiguous(memory_format=torch.channels_last)
    w = w.contiguous(memory_format=torch.channels_last)
    if variant < 0:
        ho, wo = out_hw(x.shape[2], x.shape[3], w.shape[2], w.shape[3], stride, pad)
        variant = pick_variant(x.shape[0] * ho * wo, w.shape[0])
    if addend is not None:
        addend = addend.contiguous(memory_format=torch.channels_last)
    bx = bm = bmu = None
    if bn is not None:
        bx, bm, bmu = bn
        with_stats = True
    fin = bool(final and with_stats and bn is None and addend is None)
    out = _ext.load().conv_fwd(x, w, int(stride), int(pad), int(variant), bool(with_stats),
                               addend, bx, bm, bmu, addmask if addend is not None else None,
                               stats_final=fin, bn_acc=bn_acc if bn is not None else None)
    if bn is not None and bn_acc is not None:
        return out[0], None          # the sums went into the caller's bn_acc
    if fin:
        from .batchnorm import FinishedStats
        return out[0], FinishedStats(out[1])
    if with_stats:
        return out[0], (out[1], TILES[variant][0])
    return out[0]


def flip_weight(w: Tensor) -> Tensor:
    """W' [Cin, Cout, R, S] (channels_last) with W'[ci, co, r, s] = W[co, ci, R-1-r, S-1-s]
    (one transpose kernel on the GPU; torch ops elsewhere)."""
    if (w.is_cuda and w.dtype == torch.bfloat16 and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0):
        return _ext.load().conv_flip_weight(w.contiguous(memory_format=torch.channels_last))
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


def conv2d_bwd_data(dy: Tensor, w: Tensor, pad: int, variant: int = -1,
                    addend: Tensor | None = None, bn=None, wflip: Tensor | None = None,
                    addmask: Tensor | None = None, bn_acc: Tensor | None = None):
    """dX (+ addend) of a stride-1 convolution (same spatial size when pad = (R-1)/2).
    With ``bn`` (see conv2d_fwd) returns (dX, (part, rpb)): the backward partials of the
    BatchNorm layer whose output is this convolution's input. ``wflip``: ``flip_weight(w)``
    computed ahead of time (``WeightFlipper``)."""
    r = w.shape[2]
    wf = wflip if wflip is not None else flip_weight(w)
    return conv2d_fwd(dy, wf, 1, r - 1 - pad, variant, addend=addend, bn=bn, addmask=addmask,
                      bn_acc=bn_acc)


# On by default since the v2 tiles carry the partials in their coalesced store loop and the plan
# times the linked backward-data form separately (ConvPlan.bwd_bn): ResNet-50 bs128 12.67 ->
# 12.22 / 12.32 ms per step (profiles/r4_bn_links_v2_tuned_ab.log). Round 3's v1-only form lost
# (15.69 vs 15.37 ms): its 128x128 EPI 2 kernel ran at one wave per SIMD.
_BN_LINKS = os.environ.get("ARENA_BN_LINKS", "1") == "1"


def set_bn_links(on: bool) -> None:
    """Enable/disable BNGradLink fusion (on by default; ARENA_BN_LINKS=0 turns it off)."""
    global _BN_LINKS
    _BN_LINKS = bool(on)


# BatchNorm statistics summed inside the conv kernel (fp64 fire-and-forget atomics into an
# [rep, 2, C] set the BN apply pass derives its coefficients from) instead of per-tile partials
# plus a finalize launch in the BN layer (on by default; ARENA_BN_FINAL=0 for A/Bs). Also switches
# the BN kernels' own statistics/backward reductions to the same acc mode.
_BN_FINAL = os.environ.get("ARENA_BN_FINAL", "1") == "1"
# Up to this many (tile, channel) pairs per layer the epilogue sums; above it, per-tile partials
# and the BN finalize launch. With one accumulator replica, the same-address atomics of the 56x56
# layers (3136 tiles per channel) serialized and 128 k was the best cap
# (profiles/r4_acc_threshold_ab.jsonl); with the row tiles spread over 4 replicas (csrc/ops/abi.h ARENA_ACC_REP) every layer
# takes the sums: 10,852 / 10,832 / 10,891 vs 10,678 / 10,664 / 10,706 images/s, alternating
# runs on one box (profiles/r5_acc_rep_ab.txt; 16 replicas cost the consumers more than they
# save, r5_accrep16_ab.jsonl).
_ACC_MAX_PAIRS = int(os.environ.get("ARENA_BN_ACC_MAX_PAIRS", str(4 << 20)))


# the same rule for the dgrad epilogue's BN-backward sums (BNGradLink acc form), separately
# switchable for A/Bs (ARENA_BN_LINK_ACC_MAX_PAIRS; 0: always per-tile partials + BN finalize)
_LINK_ACC_MAX_PAIRS = int(os.environ.get("ARENA_BN_LINK_ACC_MAX_PAIRS", str(_ACC_MAX_PAIRS)))


def set_link_acc_max_pairs(n: int) -> None:
    global _LINK_ACC_MAX_PAIRS
    _LINK_ACC_MAX_PAIRS = int(n)


def _use_link_acc(m: int, variant: int, c: int) -> bool:
    return -(-m // TILES[variant][0]) * c <= _LINK_ACC_MAX_PAIRS


def set_acc_max_pairs(n: int) -> None:
    """Epilogue-statistics threshold (see _ACC_MAX_PAIRS); decided per call, so a captured graph
    keeps the mode it was captured with."""
    global _ACC_MAX_PAIRS
    _ACC_MAX_PAIRS = int(n)


def _use_acc(m: int, variant: int, cout: int) -> bool:
    """Whether a forward of ``m`` output pixels on tile variant ``variant`` sums its BatchNorm
    statistics in the epilogue (fp64 atomics, one set per block) instead of per-tile partials."""
    return _BN_FINAL and -(-m // TILES[variant][0]) * cout <= _ACC_MAX_PAIRS


def _out_pixels(x: Tensor, w: Tensor, stride: int, pad: int) -> int:
    ho, wo = out_hw(x.shape[2], x.shape[3], w.shape[2], w.shape[3], stride, pad)
    return x.shape[0] * ho * wo


def set_bn_final(on: bool) -> None:
    global _BN_FINAL
    _BN_FINAL = bool(on)
    if torch.cuda.is_available() and _ext.available():
        _ext.load().bn_set_acc(bool(on))


def _stats_out(want: bool, part: Tensor, rpb: int):
    """What ``forward_stats`` hands the BN layer: finished statistics (the fp64 [rep, 2, C] sums
    of the conv epilogue) or the flat fp32 per-tile partials."""
    if not want:
        return None
    if part.dtype == torch.float64:
        from .batchnorm import FinishedStats
        return FinishedStats(part)
    return (part, rpb)


def conv2d_bwd_data_strided(dy: Tensor, w: Tensor, x_hw: Tuple[int, int], stride: int, pad: int,
                            variant: int = -1, addend: Tensor | None = None) -> Tensor:
    """dX of a stride-``stride`` convolution as ``stride**2`` phase convolutions on the kernel.

    Input pixel (i*s + a, j*s + b) only receives the filter taps r with (a + pad - r) % s == 0;
    over the phase grid (i, j) that is a stride-1 convolution of dY with the flipped sub-filter
    W[:, :, r0::s, c0::s], written straight into the (a, b) parity class of dX (the kernel's
    mapped output). All phase weights come from one ``conv_phase_weights`` launch. ``addend`` (the
    residual join's other gradient) is added in the epilogue. Phases without taps (1x1 stride 2:
    three of four) are the addend or zero: when phase (0, 0) is the only one with taps its
    epilogue writes them too (fill_sib), so dX is written in one pass. With a v2 tile variant
    the phases run as one launch (``conv_dgrad_phases``)."""
    N, Cout, Ho, Wo = dy.shape
    Cin, R, S = w.shape[1], w.shape[2], w.shape[3]
    H, W = x_hw
    dy = dy.contiguous(memory_format=torch.channels_last)
    if addend is not None:
        addend = addend.contiguous(memory_format=torch.channels_last)
    ext = _ext.load()
    phases = []
    for a in range(stride):
        r0 = (a + pad) % stride
        if r0 >= R:
            continue
        for b in range(stride):
            c0 = (b + pad) % stride
            if c0 >= S:
                continue
            phases.append((a, b, r0, c0))
    wps = ext.conv_phase_weights(w.contiguous(memory_format=torch.channels_last), stride, pad)
    full = len(phases) == stride * stride
    sib = len(phases) == 1 and phases[0][:2] == (0, 0)
    dx = torch.empty(N, Cin, H, W, device=dy.device, dtype=dy.dtype,
                     memory_format=torch.channels_last)
    if not (full or sib):          # uncovered pixels: addend or zero, then accumulate in place
        if addend is not None:
            dx.copy_(addend)
        else:
            dx.zero_()
        addend = dx
    geo = []
    for (a, b, r0, c0), wp in zip(phases, wps):
        Rp, Sp = wp.shape[2], wp.shape[3]
        ca, cb = (a + pad - r0) // stride, (b + pad - c0) // stride
        Hp, Wp = (H - a + stride - 1) // stride, (W - b + stride - 1) // stride
        if Hp > 0 and Wp > 0:
            geo.append((wp, [Rp - 1 - ca, Sp - 1 - cb, Hp, Wp, a, b]))
    if V2 <= variant and variant not in V2_HALO and len(geo) > 1:
        # v2 tiles: every phase in one launch (the phases' tiles fill the chip together)
        ext.conv_dgrad_phases(dy, [g[0] for g in geo], [g[1] for g in geo], dx, addend, stride,
                              int(variant))
        return dx
    for wp, (ph_, pw_, Hp, Wp, a, b) in geo:
        v = variant if variant >= 0 else pick_variant(N * Hp * Wp, Cin)
        ext.conv_fwd_ex(dy, wp, 1, ph_, pw_, Hp, Wp, int(v), False, addend, dx,
                        [stride, stride, a, b] + ([1] if sib else []), False)
    return dx


# ------------------------------------------------------------------------------------------------
# The 7x7/2 ResNet stem (3 input channels) as a space-to-depth 4x4/1 convolution over 16 channels
# (12 used), which the MFMA kernel runs in its c16 mode: K = 4*4*16 = 256 (147 useful), against
# 7*7*64 = 3136 if the 3 channels were padded to one 64-channel K step.
#   z[n][i][j][(dy*2+dx)*3 + c] = x[n][2i+dy][2j+dx][c]
#   W16[co][u][v][(dy*2+dx)*3 + c] = W[co][c][2u+dy-1][2v+dx-1]  (0 outside the 7x7 filter)
#   y[ho][wo] = sum_{u,v} z[ho-2+u][wo-2+v] . W16[u][v]
# ------------------------------------------------------------------------------------------------
def stem_weight(w: Tensor) -> Tensor:
    """W16 [Cout, 16, 4, 4] (channels_last) from a [Cout, C, 7, 7] stem weight, C <= 4 (torch
    ops, differentiable: dW comes back through them)."""
    co, c = w.shape[0], w.shape[1]
    wp = F.pad(w, (1, 0, 1, 0))                                   # [co, c, 8, 8]
    wp = wp.view(co, c, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1)     # co, u, v, dy, dx, c
    wp = wp.reshape(co, 4, 4, 4 * c)
    wp = F.pad(wp, (0, 16 - 4 * c))                                # [co, 4, 4, 16]
    return wp.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)


_STEM_FUSED = True


def set_stem_fused(on: bool) -> None:
    """Fused stem casts + one-kernel weight transform (default) or the torch-op form (A/Bs)."""
    global _STEM_FUSED
    _STEM_FUSED = bool(on)


class _StemWeightFn(torch.autograd.Function):
    """``stem_weight`` as one HIP kernel each way (instead of ~5 pad/permute/copy kernels per
    direction per step); the gradient comes back in the weight's dtype and memory layout."""

    @staticmethod
    def forward(ctx, w):
        ctx.save_for_backward(w)
        return _ext.load().stem_weight(w)

    @staticmethod
    def backward(ctx, dw16):
        (w,) = ctx.saved_tensors
        return _ext.load().stem_weight_grad(dw16.contiguous(memory_format=torch.channels_last), w)


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, w16, want_stats, fwd_variant, wgrad_cfg):
        Ho, Wo = z.shape[2], z.shape[3]
        fin = bool(want_stats and _use_acc(z.shape[0] * Ho * Wo, fwd_variant,
                                            w16.shape[0]))
        out = _ext.load().conv_fwd_ex(z, w16, 1, 2, 2, Ho, Wo, int(fwd_variant), bool(want_stats),
                                      None, None, [], True, stats_final=fin)
        ctx.save_for_backward(z)
        ctx.wgrad_cfg = wgrad_cfg
        ctx.set_materialize_grads(False)
        part = out[1] if want_stats else z.new_empty(0, dtype=torch.float32)
        ctx.mark_non_differentiable(part)
        return out[0], part

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None or not ctx.needs_input_grad[1]:
            return None, None, None, None, None
        (z,) = ctx.saved_tensors
        v, sp = ctx.wgrad_cfg
        dy = dy.contiguous(memory_format=torch.channels_last)
        dw = _ext.load().conv_wgrad_ex(z, dy, 4, 4, 1, 2, 2, int(v), int(sp), False, 1.0, True)
        return None, dw, None, None, None


def stem_ok(x: Tensor, w: Tensor, stride: int, pad: int) -> bool:
    return (x.is_cuda and x.dim() == 4 and tuple(w.shape[2:]) == (7, 7) and stride == 2
            and pad == 3 and x.shape[1] <= 4 and w.shape[0] % 64 == 0 and x.shape[2] % 2 == 0
            and x.shape[3] % 2 == 0 and not x.requires_grad)


class BNGradLink:
    """A BatchNorm layer whose output is the input of a convolution: the conv's backward-data
    pass produces exactly the gradient the BN's backward starts from, so its epilogue also
    computes the BN backward's per-channel partial sums (sum g, sum g * (x - mean), g = dY *
    ReLU mask) and the BN skips its reduction pass over dY and x. The BN's forward fills
    ``set_bn``; the conv's backward ``publish``es; the BN's backward ``take``s, which checks that
    it received the very tensor the partials describe (else it runs its own reduction).

    With the BN's own backward-sum set (``bacc``, batchnorm._BwdAcc) and few enough (tile,
    channel) pairs (``_use_acc``), the epilogue adds fp64 sums into that set instead of writing
    per-tile partials, and the BN's dx pass reads them directly: no reduction, no finalize."""
    __slots__ = ("x", "mask", "mean", "bacc", "part", "rpb", "acc", "dy_ptr")

    def __init__(self):
        self.x = self.mask = self.mean = self.bacc = self.part = self.acc = None
        self.rpb = 0
        self.dy_ptr = 0

    def set_bn(self, x: Tensor, mask: Tensor | None, mean: Tensor, bacc=None) -> None:
        if _BN_LINKS:
            self.x, self.mask, self.mean, self.bacc = x, mask, mean, bacc

    def ready(self) -> bool:
        return self.x is not None

    def publish(self, part: Tensor, rpb: int, dy: Tensor) -> None:
        self.part, self.rpb, self.dy_ptr = part, int(rpb), dy.data_ptr()

    def publish_acc(self, acc: Tensor, dy: Tensor) -> None:
        self.acc, self.dy_ptr = acc, dy.data_ptr()

    def take(self, dy: Tensor):
        """(part, rpb) or ("acc", sums) if the link's result describes ``dy``, else None.
        Releases the references."""
        out = None
        if dy.data_ptr() == self.dy_ptr and self.x is not None and dy.shape == self.x.shape:
            if self.acc is not None:
                out = ("acc", self.acc)
            elif self.part is not None:
                out = (self.part, self.rpb)
        self.x = self.mask = self.mean = self.bacc = self.part = self.acc = None
        self.dy_ptr = 0
        return out


_MASKED_JOIN = True


def set_masked_join(on: bool) -> None:
    """A block's last BN parks (dy, ReLU bits) in the residual join instead of writing dy * mask
    (default on; off for A/Bs)."""
    global _MASKED_JOIN
    _MASKED_JOIN = bool(on)


def masked_join() -> bool:
    return _MASKED_JOIN


class MaskedGrad:
    """A gradient given as (g, bits): the value is g where the bit is set, 0 elsewhere (a
    ReLU'd BatchNorm output's gradient, parked in a GradJoin without materializing g * mask)."""
    __slots__ = ("g", "bits")

    def __init__(self, g: Tensor, bits: Tensor):
        self.g, self.bits = g, bits

    def materialize(self) -> Tensor:
        """g * mask as a dense tensor (for consumers without a masked epilogue)."""
        return (self.g * _unpack_bits(self.bits, self.g)).contiguous(
            memory_format=torch.channels_last)


def _unpack_bits(bits: Tensor, like: Tensor) -> Tensor:
    """The 0/1 mask (dtype of ``like``, its NHWC layout) of a bit-packed mask."""
    shifts = torch.arange(8, device=bits.device, dtype=torch.uint8)
    m = ((bits.view(-1, 1) >> shifts) & 1).reshape(-1)
    n, c, h, w = like.shape
    return m.view(n, h, w, c).permute(0, 3, 1, 2).to(like.dtype)


class GradJoin:
    """One tensor, two consumers (a ResNet block input feeds conv1 and the shortcut): instead of
    letting autograd add the two gradients in a separate elementwise pass, the consumer whose
    backward runs first parks its gradient here and returns None for the input, and the second
    returns the sum -- fused into the backward-data kernel's epilogue when it runs on ours.
    Consumers ``register()`` in their forward; with fewer than two registered, both behave
    normally. The two backwards must both run (true inside one block), exactly once."""
    __slots__ = ("n", "arrived", "pending", "first_takes_masked")

    def __init__(self):
        self.n = 0
        self.arrived = 0
        self.pending = None
        self.first_takes_masked = False

    def register(self, takes_masked: bool = False) -> "GradJoin":
        """``takes_masked``: this consumer can fold a ``MaskedGrad`` into its own gradient (its
        backward-data kernel takes the addend's bit mask)."""
        self.n += 1
        if self.n == 1:
            self.first_takes_masked = bool(takes_masked)
        return self

    def peer_takes_masked(self) -> bool:
        """For the second registrant (a block's last BatchNorm; the conv consuming the block input
        registers first in forward order): the other consumer folds a MaskedGrad in, so this one
        may park (dy, ReLU bits) instead of writing dy * mask."""
        return self.n == 2 and self.first_takes_masked

    def active(self) -> bool:
        return self.n == 2

    def other(self) -> Tensor | None:
        """The first consumer's gradient when called from the second (else None)."""
        return self.pending if self.arrived == 1 else None

    def park_or_take(self, g: Tensor | None) -> bool:
        """Record this consumer's arrival with its gradient g. Returns True for the first one
        (g is parked: return None for the input), False for the second (g must already include
        ``other()``)."""
        self.arrived += 1
        if self.arrived == 1:
            self.pending = g
            return True
        self.arrived, self.pending = 0, None
        return False


WGRAD_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64)}   # Cout x R*S*C
WGRAD_TILES.update({v + 4: t for v, t in list(WGRAD_TILES.items())})   # + 4: serial
# 8..11: the v2 weight-gradient kernel (32x32x16 MFMAs, 128/256-wide tiles, two steps in flight)
WGRAD_V2 = {8: (128, 128), 9: (256, 128), 10: (128, 256), 11: (256, 256),
            12: (128, 128),   # 12: serial single-buffer, four waves per SIMD
            # 13 / 14: 12 with two / four wave groups per block splitting its pixel steps (the
            # same waves per CU in 1/2 / 1/4 of the blocks: that many fewer fp32 split slabs)
            13: (128, 128), 14: (128, 128)}
WGRAD_GROUPS = {13: 2, 14: 4}
WGRAD_TILES.update(WGRAD_V2)


def wgrad_variants_for(cin: int, cout: int):
    return [v for v, (bm, bn) in WGRAD_TILES.items() if cout % bm == 0 and cin % bn == 0
            and (v < 8 or _V2_ON)]


def conv2d_wgrad(x: Tensor, dy: Tensor, kernel: Tuple[int, int], stride: int = 1, pad: int = 0,
                 variant: int = -1, splits: int = 0, out_dtype=torch.bfloat16,
                 scale: float = 1.0) -> Tensor:
    """dW [Cout, C, R, S] (channels_last) of y = conv2d(x, w): split-K MFMA kernel + a
    fixed-order slab reduction (bit-reproducible)."""
    x = x.contiguous(memory_format=torch.channels_last)
    dy = dy.contiguous(memory_format=torch.channels_last)
    if variant < 0:
        variant = wgrad_variants_for(x.shape[1], dy.shape[1])[0]
    return _ext.load().conv_wgrad(x, dy, int(kernel[0]), int(kernel[1]), int(stride), int(pad),
                                  int(variant), int(splits), out_dtype == torch.float32,
                                  float(scale))


# ------------------------------------------------------------------------------------------------
# Per-shape plan: for each of forward / backward-data / backward-weight, the fastest of MIOpen and
# the kernel's tile variants (and split counts), timed once on the live device (like
# cudnn.benchmark, which this complements). ARENA_CONV=miopen forces the library everywhere,
# ARENA_CONV=ours forces the kernel wherever it applies (heuristic tiles, no timing).
# ------------------------------------------------------------------------------------------------
from dataclasses import dataclass, field  # noqa: E402
from typing import Dict, Optional  # noqa: E402

import torch.nn.functional as F  # noqa: E402
from torch import nn  # noqa: E402

MIOPEN = "miopen"


_MODE_OVERRIDE: Optional[str] = None


def set_mode(mode: Optional[str]) -> None:
    """Process-wide override of ARENA_CONV (auto | ours | miopen | off; None = use the env)."""
    global _MODE_OVERRIDE
    if mode not in (None, "auto", "ours", MIOPEN, "off"):
        raise ValueError(f"unknown conv mode {mode!r}")
    _MODE_OVERRIDE = mode


def _mode() -> str:
    return _MODE_OVERRIDE or os.environ.get("ARENA_CONV", "auto")


@dataclass
class ConvPlan:
    fwd: object = MIOPEN            # MIOPEN or a tile variant
    bwd: object = MIOPEN
    wgrad: object = MIOPEN          # MIOPEN or (variant, splits)
    # backward-data with the BN-backward partials in its epilogue (BNGradLink; stride 1): timed
    # in that form, since the extra epilogue reorders the tiles (v1's 128x128 form drops to one
    # wave per SIMD, 196 VGPRs + 72 AGPRs)
    bwd_bn: object = MIOPEN
    tuned: bool = False
    times: Dict[str, float] = field(default_factory=dict)


_PLANS: Dict[tuple, ConvPlan] = {}


def _time(fn, reps: int = 4, iters: int = 3) -> float:
    """GPU time of fn() in us: ``reps`` calls captured in a hipGraph, replayed ``iters`` times.
    (Eager timing would charge a library's host-side launch cost, which the training step's
    graph replay never pays: MIOpen's convolution_backward costs ~50 us of host time per call.)"""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if os.environ.get("ARENA_CONV_TIME_EAGER") == "1":
        s.record()
        for _ in range(reps * iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / (reps * iters)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        g.replay()
    e.record()
    e.synchronize()
    del g
    return s.elapsed_time(e) * 1e3 / (reps * iters)


def _miopen_bwd(dy, x, w, stride, pad, mask):
    return torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad],
                                               [1, 1], False, [0, 0], 1, mask)


# blocks per CU the weight-gradient split counts aim at (ARENA_WGRAD_BPC, for A/Bs)
_WGRAD_BPC = tuple(float(b) for b in os.environ.get("ARENA_WGRAD_BPC", "1,2,4").split(","))


def _wgrad_candidates(cin, cout, k):
    """(tile variant, split count) pairs: splits that give ~1, 2 or 4 blocks per CU."""
    out = []
    for v in wgrad_variants_for(cin, cout):
        bm, bn = WGRAD_TILES[v]
        tiles = (cout // bm) * (k[0] * k[1] * cin // bn)
        # wave-group forms: a block already holds GRP x 4 waves -- one or two blocks per CU
        bpcs = (1, 2) if v in WGRAD_GROUPS else _WGRAD_BPC
        for bpc in bpcs:
            blocks = int(bpc * _CUS)
            out.append((v, max(1, -(-blocks // tiles))))
    return sorted(set(out))


# what a forward whose statistics come as per-tile partials pays on top of its own time: the BN
# layer's partial-merge finalize launch (bn_stats_finalize, ~11 us per layer at batch 128,
# profiles/r3_finalize16_steady_kernels.csv)
_FIN_PENALTY_US = float(os.environ.get("ARENA_CONV_FIN_PENALTY_US", "11"))


def _best(t: dict, kind: str, n: int):
    """The n fastest variant codes timed so far for direction ``kind``."""
    return [c for (kd, c), _ in sorted(((k, v) for k, v in t.items() if k[0] == kind),
                                       key=lambda kv: kv[1])][:n]


def plan_for(x: Tensor, w: Tensor, stride: int, pad: int) -> ConvPlan:
    key = (tuple(x.shape), tuple(w.shape), stride, pad, x.device.index, _mode(), _V2_ON,
           _BN_LINKS, _HALO_WIDE_ON)
    plan = _PLANS.get(key)
    if plan is not None and (plan.tuned or torch.cuda.is_current_stream_capturing()):
        return plan
    mode = _mode()
    plan = plan or ConvPlan()
    cin, cout, k = w.shape[1], w.shape[0], (w.shape[2], w.shape[3])
    ok = kernel_ok(x, w, stride, pad)
    ho, wo = out_hw(x.shape[2], x.shape[3], k[0], k[1], stride, pad)
    wg = _wgrad_candidates(cin, cout, k) if ok else []
    if mode == MIOPEN or not ok:
        plan.tuned = True
    elif mode == "ours" or torch.cuda.is_current_stream_capturing():
        # ARENA_CONV_DIRS (debugging): the directions "ours" puts on the kernels
        dirs = os.environ.get("ARENA_CONV_DIRS", "fwd,bwd,wgrad").split(",")
        plan.fwd = pick_variant(x.shape[0] * ho * wo, cout) if "fwd" in dirs else MIOPEN
        plan.bwd = ((pick_variant(x.shape[0] * x.shape[2] * x.shape[3], cin) if stride == 1
                     else -1) if "bwd" in dirs else MIOPEN)
        plan.wgrad = wg[len(wg) // 2] if (wg and "wgrad" in dirs) else MIOPEN
        plan.bwd_bn = plan.bwd if stride == 1 else MIOPEN
        plan.tuned = mode == "ours"
    else:
        def tune() -> dict:
            # Only the MFMA kernels are candidates: a captured step with MIOpen convolutions in it
            # returned wrong gradients on replays that followed other GPU/host work, while the same
            # step on these kernels alone stayed bit-identical run to run (tools/graph_mem_*.py,
            # docs/perf.md "MIOpen inside a captured step"). ARENA_CONV=miopen keeps the library
            # path for comparisons.
            # (a random output gradient of the conv's output shape; no library call: F.conv2d here
            # ran MIOpen's Find -- its naive and CK kernels -- once per shape, ~0.5 s of startup)
            dy = torch.randn(x.shape[0], cout, ho, wo, device=x.device, dtype=x.dtype).contiguous(
                memory_format=torch.channels_last)
            t = {}
            m_out = x.shape[0] * ho * wo

            def fwd_time(v):
                # timed the way the step runs it: statistics summed in the epilogue where _use_acc
                # says so (into a scratch set), else per-tile partials plus the BN finalize launch
                # that consumes them (charged as _FIN_PENALTY_US)
                fin = _use_acc(m_out, v, cout)
                us = _time(lambda: conv2d_fwd(x, w, stride, pad, v, with_stats=True, final=fin))
                return us if fin else us + _FIN_PENALTY_US

            fns = {}
            halo = lambda c, kc: halo_variants_for(c, k, stride, pad, x.shape[3], kc)  # noqa: E731
            for v in (variants_for(cout) + v2_variants_for(cout) + halo(cout, cin)
                      + split_variants_for(m_out, cout, cin * k[0] * k[1])):
                fns[("fwd", v)] = (lambda v=v: fwd_time(v))
            if stride == 1:
                m_in = x.shape[0] * x.shape[2] * x.shape[3]
                for v in (variants_for(cin) + v2_variants_for(cin) + halo(cin, cout)
                          + split_variants_for(m_in, cin, cout * k[0] * k[1])):
                    fns[("bwd", v)] = (lambda v=v: _time(
                        lambda: conv2d_bwd_data(dy, w, pad, v)))
                if _BN_LINKS:   # the linked form: a BN input, ReLU bits and mean of x's shape
                    bnx = torch.randn_like(x)
                    bmask = torch.randint(0, 256, (m_in * cin // 8,), device=x.device,
                                          dtype=torch.uint8)
                    bmean = torch.zeros(cin, device=x.device)
                    from .batchnorm import acc_rep
                    bsums = torch.zeros(acc_rep() * 2 * cin, dtype=torch.float64,
                                        device=x.device)
                    for v in variants_for(cin) + v2_variants_for(cin) + halo(cin, cout):
                        # timed in the epilogue form the step will run: fp64 sums into the BN's
                        # backward set where _use_link_acc picks it, else per-tile partials
                        acc = bsums if _use_link_acc(m_in, v, cin) else None
                        fns[("bwdbn", v)] = (lambda v=v, acc=acc: _time(lambda: conv2d_bwd_data(
                            dy, w, pad, v, bn=(bnx, bmask, bmean), bn_acc=acc)))
            else:   # phase decomposition: per-phase heuristic (-1) or one tile for every phase
                hw = (x.shape[2], x.shape[3])
                for v in [-1] + variants_for(cin) + v2_variants_for(cin):
                    fns[("bwd", v)] = (lambda v=v: _time(
                        lambda: conv2d_bwd_data_strided(dy, w, hw, stride, pad, v)))
            for c in wg:
                fns[("wgrad", c)] = (lambda c=c: _time(
                    lambda: conv2d_wgrad(x, dy, k, stride, pad, c[0], c[1])))
            ext = _ext.load()
            ext.bn_acc_scratch(True)
            try:
                for key_, fn in fns.items():
                    t[key_] = fn()
                # One timing per candidate picks the lucky one among near-equal variants (the
                # choices moved run to run by ~1 % of the step): the 3 fastest of each direction are
                # timed twice more, interleaved, and ranked by their median.
                kinds = ("fwd", "bwd", "wgrad") + (("bwdbn",) if any(k_[0] == "bwdbn" for k_ in fns)
                                                   else ())
                finals = {kind: _best(t, kind, 3) for kind in kinds}
                reps = {(kind, c): [t[(kind, c)]] for kind, cs in finals.items() for c in cs}
                for _ in range(2):
                    for key_ in reps:
                        reps[key_].append(fns[key_]())
                for key_, vs in reps.items():
                    t[key_] = sorted(vs)[1]
            finally:
                ext.bn_acc_scratch(False)
            out = {}
            names = {"bwdbn": "bwd_bn"}
            for kind in kinds:
                best = min(t[(kind, c)] for c in finals[kind])
                choice = next(c for c in finals[kind] if t[(kind, c)] == best)
                out[names.get(kind, kind)] = choice
            out["times"] = {f"{kd}:{c}": round(v, 1) for (kd, c), v in t.items()}
            return out

        # one decision per job: rank 0 times, every rank adopts (or the ARENA_CONV_PLAN file)
        got = planstore.decide("conv", key[:4] + key[5:], x.device, tune)
        for f in ("fwd", "bwd", "wgrad", "bwd_bn"):
            if f in got:
                v = got[f]
                setattr(plan, f, tuple(v) if isinstance(v, list) else v)
        plan.times = dict(got.get("times", {}))
        plan.tuned = True
    _PLANS[key] = plan
    return plan


# ------------------------------------------------------------------------------------------------
# Weight gradients on a side stream. In a conv's backward, dX (-> the BatchNorm backward chain:
# reduce, finalize, dx) and dW are independent; most BN-backward and finalize launches are latency-
# or tail-bound and leave CUs idle, so running dW concurrently on a second HIP stream fills them
# (in a captured step the two streams become parallel graph branches). The caller must join the
# side stream before anything reads the weight gradients: ``sync_wgrad()`` (cnn_bench does it
# between backward and the optimizer step). Off by default; single-process use only (DP bucket
# hooks read gradients as soon as autograd hands them over).
#
# A side-stream dW is handed to autograd before it is complete, so it is only used when nothing
# on the main stream can read it before ``sync_wgrad()``: the conv's weight input must be the leaf
# parameter itself (bf16 master-weight training -- with fp32 weights under autocast, the cast's
# ToCopyBackward would read dW on the main stream) and its ``.grad`` must be unset (AccumulateGrad
# then stores the tensor; a ``+=`` into an existing gradient would read it). Otherwise the
# weight gradient runs on the main stream as usual.
# ------------------------------------------------------------------------------------------------
_ASYNC_WGRAD = False
_SIDE: Dict[int, "torch.cuda.Stream"] = {}


def set_async_wgrad(on: bool) -> None:
    global _ASYNC_WGRAD
    _ASYNC_WGRAD = bool(on)


def async_wgrad() -> bool:
    return _ASYNC_WGRAD


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = _SIDE[idx] = torch.cuda.Stream(device=idx)
    return s


def sync_wgrad() -> None:
    """Make the current stream wait for every weight gradient queued on the side stream."""
    if not _SIDE or not torch.cuda.is_available():
        return
    s = _SIDE.get(torch.cuda.current_device())
    if s is not None:
        torch.cuda.current_stream().wait_stream(s)


def plans() -> Dict[tuple, ConvPlan]:
    """The per-shape choices made so far (for logs and profiles)."""
    return dict(_PLANS)


# ------------------------------------------------------------------------------------------------
# Flipped weights for a whole model in one launch. Every stride-1 backward-data pass on the kernel
# runs on W' = flip_weight(W): one transpose launch per conv per step (49 in a ResNet-50 step,
# ~5 us each). ``WeightFlipper.scope()`` wraps a model's training forward: it flips every eligible
# weight in ONE conv_flip_multi launch into persistent buffers, and the convolutions that run
# inside the scope hand their flipped copy to their backward (ctx). The weights cannot change
# between that forward and its backward, and nothing outside the scope ever reads the buffers, so
# a copy is never stale. Under hipGraph capture the launch is part of the captured forward.
# ------------------------------------------------------------------------------------------------
_ACTIVE_FLIPS: Optional[Dict[int, Tensor]] = None


def _flip_eligible(w: Tensor) -> bool:
    return (w.is_cuda and w.dim() == 4 and w.dtype == torch.bfloat16
            and w.is_contiguous(memory_format=torch.channels_last) and w.shape[0] % 64 == 0
            and w.shape[1] % 64 == 0 and w.shape[2] * w.shape[3] <= 64)


class WeightFlipper:
    """Pre-flips the weights of a model's stride-1 ``Conv2dNHWC`` layers for their backward-data
    passes (see above). bf16 channels_last weights only (master-weight training); with fp32
    weights under autocast each conv casts and flips its own weight as before."""

    def __init__(self, modules):
        self.convs = [m for m in modules if type(m) is Conv2dNHWC and m.stride[0] == 1]
        self._key = None
        self._src: list = []
        self._dst: list = []
        self._retired: list = []   # old flip buffers a captured graph may still reference

    def scope(self):
        return _FlipScope(self)

    def _prepare(self):
        if _mode() in ("off", MIOPEN) or not torch.is_grad_enabled():
            return None
        ws = [m.weight for m in self.convs if m.training and _flip_eligible(m.weight)]
        if not ws:
            return None
        key = tuple((w.data_ptr(), tuple(w.shape)) for w in ws)
        if key != self._key:
            # A captured hipGraph keeps writing and reading the flip buffers it was captured
            # with, so they are never freed while the flipper lives: a destination whose shape
            # is unchanged is reused in place, and superseded buffers are retired (kept alive)
            # instead of being handed back to the allocator for other tensors.
            old = {}
            for d in self._dst:
                old.setdefault(tuple(d.shape), []).append(d)
            dst = []
            for w in ws:
                shp = (w.shape[1], w.shape[0], w.shape[2], w.shape[3])
                pool = old.get(shp)
                dst.append(pool.pop(0) if pool else
                           torch.empty(shp, device=w.device, dtype=w.dtype,
                                       memory_format=torch.channels_last))
            self._retired.extend(d for pool in old.values() for d in pool)
            self._src, self._dst = ws, dst
            self._key = key
        _ext.load().conv_flip_multi(self._src, self._dst)
        return {w.data_ptr(): d for w, d in zip(self._src, self._dst)}


class _FlipScope:
    def __init__(self, flipper: WeightFlipper):
        self.flipper = flipper
        self.prev = None

    def __enter__(self):
        global _ACTIVE_FLIPS
        self.prev = _ACTIVE_FLIPS
        flips = self.flipper._prepare()
        if flips is not None:
            _ACTIVE_FLIPS = flips
        return self

    def __exit__(self, *exc):
        global _ACTIVE_FLIPS
        _ACTIVE_FLIPS = self.prev
        return False


def _active_flip(w: Tensor) -> Optional[Tensor]:
    if _ACTIVE_FLIPS is None:
        return None
    wf = _ACTIVE_FLIPS.get(w.data_ptr())
    if wf is None or wf.shape[0] != w.shape[1] or wf.shape[1] != w.shape[0] \
            or wf.shape[2:] != w.shape[2:]:
        return None
    return wf


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, plan, want_stats, join=None, bn_link=None):
        part = x.new_empty(0, dtype=torch.float32)
        if plan.fwd == MIOPEN:
            y = F.conv2d(x, w, stride=stride, padding=pad)
        elif want_stats and _use_acc(_out_pixels(x, w, stride, pad), plan.fwd,
                                     w.shape[0]):
            y, st = conv2d_fwd(x, w, stride, pad, plan.fwd, with_stats=True, final=True)
            part = st.fin
        elif want_stats:
            y, (part, _) = conv2d_fwd(x, w, stride, pad, plan.fwd, with_stats=True)
        else:
            y = conv2d_fwd(x, w, stride, pad, plan.fwd)
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pad, plan)
        ctx.w_leaf = w.is_leaf
        # W' of a WeightFlipper scope (flipped this step, before this forward)
        ctx.wflip = _active_flip(w) if (stride == 1 and plan.bwd != MIOPEN) else None
        # the backward-data kernel can take a masked addend (a BN's (dy, ReLU bits), see GradJoin)
        ctx.join = join.register(takes_masked=(stride == 1 and plan.bwd != MIOPEN)) \
            if join is not None else None
        ctx.bn_link = bn_link if (bn_link is not None and bn_link.ready()) else None
        ctx.mark_non_differentiable(part)
        # no zero-filled gradient for the statistics output (one fill kernel per conv per step)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        if dy is None:
            return None, None, None, None, None, None, None, None
        x, w = ctx.saved_tensors
        stride, pad, plan = ctx.conf
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            join = ctx.join if (ctx.join is not None and ctx.join.active()) else None
            # the second consumer of a joined input folds the first one's gradient in
            other = join.other() if join is not None else None
            omask = None
            if isinstance(other, MaskedGrad):
                if stride == 1 and plan.bwd != MIOPEN:
                    other, omask = other.g.contiguous(memory_format=torch.channels_last), \
                        other.bits
                else:
                    other = other.materialize()
            lk = ctx.bn_link
            # the BN partials need the COMPLETE gradient of x: not from a join's first arriver
            use_bn = (lk is not None and plan.bwd != MIOPEN and stride == 1
                      and lk.x.shape == x.shape
                      and (join is None or other is not None))
            if plan.bwd == MIOPEN:
                dx = _miopen_bwd(dy, x, w, stride, pad, [True, False, False])[0]
                if other is not None:
                    dx.add_(other)
            elif stride != 1:
                dx = conv2d_bwd_data_strided(dy, w, (x.shape[2], x.shape[3]), stride, pad,
                                             plan.bwd, addend=other)
            elif use_bn:
                vb = plan.bwd if plan.bwd_bn == MIOPEN else plan.bwd_bn
                m_in = x.shape[0] * x.shape[2] * x.shape[3]
                if lk.bacc is not None and _use_link_acc(m_in, vb, x.shape[1]):
                    acc = lk.bacc.for_backward(x, x.shape[1])
                    dx, _ = conv2d_bwd_data(dy, w, pad, vb, addend=other,
                                            bn=(lk.x, lk.mask, lk.mean), wflip=ctx.wflip,
                                            addmask=omask, bn_acc=acc)
                    lk.publish_acc(acc, dx)
                else:
                    dx, (part, rpb) = conv2d_bwd_data(dy, w, pad, vb, addend=other,
                                                      bn=(lk.x, lk.mask, lk.mean),
                                                      wflip=ctx.wflip, addmask=omask)
                    lk.publish(part, rpb, dx)
            else:
                dx = conv2d_bwd_data(dy, w, pad, plan.bwd, addend=other, wflip=ctx.wflip,
                                     addmask=omask)
            if join is not None and join.park_or_take(dx):
                dx = None
        if ctx.needs_input_grad[1]:
            side = None
            if _ASYNC_WGRAD and dy.is_cuda and ctx.w_leaf and w.grad is None:
                main = torch.cuda.current_stream()
                side = _side_stream(dy.device)
                side.wait_stream(main)   # dy, x (and w) are complete on the main stream
            with torch.cuda.stream(side) if side is not None else _nullctx():
                if plan.wgrad == MIOPEN:
                    dw = _miopen_bwd(dy, x, w, stride, pad, [False, True, False])[1]
                else:
                    v, sp = plan.wgrad
                    dw = conv2d_wgrad(x, dy, (w.shape[2], w.shape[3]), stride, pad, v, sp,
                                      out_dtype=w.dtype)
            if side is not None:
                # allocator bookkeeping across the two streams
                x.record_stream(side)
                dy.record_stream(side)
                dw.record_stream(main)
        return dx, dw, None, None, None, None, None, None


class Conv2dNHWC(nn.Conv2d):
    """``nn.Conv2d`` (no bias, no groups/dilation) that runs channels_last bf16 convolutions on
    the MFMA implicit-GEMM kernels when they are faster than MIOpen for the shape (timed once
    per shape). Under bf16 autocast the weight/input casts happen here, as autocast would do
    them. Everything else (CPU, fp32, unsupported shapes) is plain ``nn.Conv2d``."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if isinstance(self.padding, str) or self.bias is not None or self.groups != 1 or \
                self.dilation != (1, 1) or self.stride[0] != self.stride[1] or \
                self.padding[0] != self.padding[1]:
            raise ValueError("Conv2dNHWC: square stride/padding, no bias, groups or dilation")

    def forward(self, x: Tensor) -> Tensor:
        return self.forward_stats(x, want_stats=False)[0]

    def forward_stats(self, x: Tensor, want_stats: bool = True, join: GradJoin | None = None,
                      bn_link: BNGradLink | None = None):
        """(y, stats): ``stats`` are the BatchNorm partials of y for ``BatchNormAct2d(y,
        stats=stats)`` when the kernel produced y (else None: the BN computes them itself).
        ``join``: x has a second consumer registered on the same GradJoin (see there).
        ``bn_link``: x is the output of the BatchNorm layer that filled this link."""
        if not x.is_cuda or _mode() == "off":
            return super().forward(x), None
        amp = torch.is_autocast_enabled("cuda") and \
            torch.get_autocast_dtype("cuda") == torch.bfloat16
        w = self.weight
        if amp:
            x = x.to(torch.bfloat16)
            w = w.to(torch.bfloat16)
        if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
            return super().forward(x), None
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
        s, p = self.stride[0], self.padding[0]
        plan = plan_for(x, w, s, p)
        want = want_stats and plan.fwd != MIOPEN and torch.is_grad_enabled() and self.training
        with torch.autocast("cuda", enabled=False):
            y, part = _ConvFn.apply(x, w, s, p, plan, want, join, bn_link)
        return y, _stats_out(want, part, TILES[plan.fwd][0] if want else 0)


class StemConv2d(Conv2dNHWC):
    """The 7x7/2 stem convolution (3 input channels) on the MFMA kernel through its space-to-depth
    form (see ``stem_weight``): one s2d kernel + one c16 convolution forward (with the BN
    statistics epilogue), one c16 split-K wgrad backward. Same parameters and state_dict as
    ``nn.Conv2d(C, Cout, 7, stride=2, padding=3, bias=False)``; anything else (CPU, fp32, an input
    that needs a gradient, ARENA_CONV=miopen/off) runs ``Conv2dNHWC``."""

    def forward_stats(self, x: Tensor, want_stats: bool = True, join: GradJoin | None = None,
                      bn_link: BNGradLink | None = None):
        s, p = self.stride[0], self.padding[0]
        if not x.is_cuda or _mode() in ("off", MIOPEN) or join is not None:
            return super().forward_stats(x, want_stats, join, bn_link)
        amp = torch.is_autocast_enabled("cuda") and \
            torch.get_autocast_dtype("cuda") == torch.bfloat16
        w = self.weight
        # under autocast both casts are fused: s2d_stem rounds an fp32 batch to bf16 as it
        # rearranges it, and the stem-weight kernel rounds an fp32 weight (its backward writes
        # the gradient in the parameter's own dtype and layout)
        fuse = _STEM_FUSED
        xin = x if (not amp or (fuse and x.dtype == torch.float32)) else x.to(torch.bfloat16)
        ok = (xin.dtype in (torch.bfloat16, torch.float32) and w.dtype in (torch.bfloat16,
                                                                          torch.float32)
              if amp else (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16))
        if not ok or not stem_ok(xin, w, s, p):
            return super().forward_stats(x, want_stats, join, bn_link)
        xin = xin.contiguous(memory_format=torch.channels_last)
        want = want_stats and torch.is_grad_enabled() and self.training
        with torch.autocast("cuda", enabled=False):
            z = _ext.load().s2d_stem(xin)
            w16 = _StemWeightFn.apply(w) if fuse else stem_weight(w.to(torch.bfloat16))
            fv, wcfg = _stem_plan(z, w16)
            y, part = _StemFn.apply(z, w16, want, fv, wcfg)
        return y, _stats_out(want, part, TILES[fv][0] if want else 0)


_STEM_PLANS: Dict[tuple, Tuple[int, Tuple[int, int]]] = {}


def _stem_plan(z: Tensor, w16: Tensor) -> Tuple[int, Tuple[int, int]]:
    """(forward tile variant, (wgrad variant, splits)) of the c16 stem convolution: the fastest
    of the 64-wide tiles (c16 needs BN = 64) and wgrad forms, timed once per shape like
    ``plan_for`` (heuristic under ARENA_CONV=ours or while a graph is being captured)."""
    key = (tuple(z.shape), tuple(w16.shape), z.device.index, _mode())
    plan = _STEM_PLANS.get(key)
    if plan is not None:
        return plan
    ext = _ext.load()
    ho, wo = z.shape[2], z.shape[3]
    fvs = [v for v in variants_for(w16.shape[0]) if TILES[v][1] == 64 and v < 12]   # c16: 4 waves
    wcs = [(3, 0), (7, 0)]
    if _mode() == "ours" or torch.cuda.is_current_stream_capturing():
        fv = pick_variant(z.shape[0] * ho * wo, w16.shape[0])
        plan = (fv if TILES[fv][1] == 64 else 1, wcs[0])
        if _mode() == "ours":
            _STEM_PLANS[key] = plan
        return plan

    def tune() -> dict:
        tf = {v: _time(lambda: ext.conv_fwd_ex(z, w16, 1, 2, 2, ho, wo, v, True, None, None, [],
                                                True)) for v in fvs}
        dy = torch.randn(z.shape[0], w16.shape[0], ho, wo, device=z.device,
                         dtype=z.dtype).contiguous(memory_format=torch.channels_last)
        tw = {c: _time(lambda: ext.conv_wgrad_ex(z, dy, 4, 4, 1, 2, 2, c[0], c[1], False, 1.0,
                                                 True)) for c in wcs}
        if os.environ.get("ARENA_CONV_LOG") == "1":
            print(f"stem {tuple(z.shape)}: {tf} {tw}", flush=True)
        return {"fwd": min(tf, key=tf.get), "wgrad": list(min(tw, key=tw.get))}

    got = planstore.decide("stem", (key[0], key[1], key[3]), z.device, tune)
    plan = (int(got["fwd"]), tuple(got["wgrad"]))
    _STEM_PLANS[key] = plan
    return plan
