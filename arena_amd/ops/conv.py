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

import os
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


def conv2d_fwd(x: Tensor, w: Tensor, stride: int = 1, pad: int = 0, variant: int = -1,
               with_stats: bool = False, addend: Tensor | None = None, bn=None):
    """y = conv2d(x, w) (+ addend) for channels_last bf16 x [N,C,H,W] and w [Cout,C,R,S].

    with_stats: returns (y, (part, rpb)) where part holds per-tile BatchNorm partials of y
    (tile mean and sum of squared deviations per channel, ``rpb`` output pixels per tile), which
    ``BatchNormAct2d(..., stats=...)`` finalizes instead of re-reading y.
    addend: a bf16 tensor shaped like y, added to the fp32 sums before rounding (epilogue).
    bn: (bn_x, bn_mask or None, bn_mean) when y is the gradient of a BatchNorm layer's output:
    returns (y, (part, rpb)) with that BN's backward partials (sum g, sum g (bn_x - mean) per
    tile, g = y * mask) for its backward, which then skips its reduction pass."""
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
    out = _ext.load().conv_fwd(x, w, int(stride), int(pad), int(variant), bool(with_stats),
                               addend, bx, bm, bmu)
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
                    addend: Tensor | None = None, bn=None):
    """dX (+ addend) of a stride-1 convolution (same spatial size when pad = (R-1)/2).
    With ``bn`` (see conv2d_fwd) returns (dX, (part, rpb)): the backward partials of the
    BatchNorm layer whose output is this convolution's input."""
    r = w.shape[2]
    return conv2d_fwd(dy, flip_weight(w), 1, r - 1 - pad, variant, addend=addend, bn=bn)


# Off by default: on ResNet-50 bs128 the heavier dgrad epilogue cost more than the reduction pass
# it saves (15.69 / 15.74 vs 15.37 / 15.53 ms per step, same-process A/B, docs/perf.md).
_BN_LINKS = os.environ.get("ARENA_BN_LINKS", "0") == "1"


def set_bn_links(on: bool) -> None:
    """Enable/disable BNGradLink fusion (off by default; ARENA_BN_LINKS=1)."""
    global _BN_LINKS
    _BN_LINKS = bool(on)


class BNGradLink:
    """A BatchNorm layer whose output is the input of a convolution: the conv's backward-data
    pass produces exactly the gradient the BN's backward starts from, so its epilogue also
    computes the BN backward's per-channel partial sums (sum g, sum g * (x - mean), g = dY *
    ReLU mask) and the BN skips its reduction pass over dY and x. The BN's forward fills
    ``set_bn``; the conv's backward ``publish``es; the BN's backward ``take``s, which checks that
    it received the very tensor the partials describe (else it runs its own reduction)."""
    __slots__ = ("x", "mask", "mean", "part", "rpb", "dy_ptr")

    def __init__(self):
        self.x = self.mask = self.mean = self.part = None
        self.rpb = 0
        self.dy_ptr = 0

    def set_bn(self, x: Tensor, mask: Tensor | None, mean: Tensor) -> None:
        if _BN_LINKS:
            self.x, self.mask, self.mean = x, mask, mean

    def ready(self) -> bool:
        return self.x is not None

    def publish(self, part: Tensor, rpb: int, dy: Tensor) -> None:
        self.part, self.rpb, self.dy_ptr = part, int(rpb), dy.data_ptr()

    def take(self, dy: Tensor):
        """(part, rpb) if the partials describe ``dy``, else None. Releases the references."""
        out = None
        if self.part is not None and dy.data_ptr() == self.dy_ptr and self.x is not None \
                and dy.shape == self.x.shape:
            out = (self.part, self.rpb)
        self.x = self.mask = self.mean = self.part = None
        self.dy_ptr = 0
        return out


class GradJoin:
    """One tensor, two consumers (a ResNet block input feeds conv1 and the shortcut): instead of
    letting autograd add the two gradients in a separate elementwise pass, the consumer whose
    backward runs first parks its gradient here and returns None for the input, and the second
    returns the sum -- fused into the backward-data kernel's epilogue when it runs on ours.
    Consumers ``register()`` in their forward; with fewer than two registered, both behave
    normally. The two backwards must both run (true inside one block), exactly once."""
    __slots__ = ("n", "arrived", "pending")

    def __init__(self):
        self.n = 0
        self.arrived = 0
        self.pending: Tensor | None = None

    def register(self) -> "GradJoin":
        self.n += 1
        return self

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


def wgrad_variants_for(cin: int, cout: int):
    return [v for v, (bm, bn) in WGRAD_TILES.items() if cout % bm == 0 and cin % bn == 0]


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
    tuned: bool = False
    times: Dict[str, float] = field(default_factory=dict)


_PLANS: Dict[tuple, ConvPlan] = {}


def _time(fn, reps: int = 4, iters: int = 3) -> float:
    """GPU time of fn() in us: ``reps`` calls captured in a hipGraph, replayed ``iters`` times.
    (Eager timing would charge a library's host-side launch cost, which the training step's
    graph replay never pays: MIOpen's convolution_backward costs ~50 us of host time per call.)"""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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


def _wgrad_candidates(cin, cout, k):
    """(tile variant, split count) pairs: splits that give ~1, 2 or 4 blocks per CU."""
    out = []
    for v in wgrad_variants_for(cin, cout):
        bm, bn = WGRAD_TILES[v]
        tiles = (cout // bm) * (k[0] * k[1] * cin // bn)
        for blocks in (_CUS, 2 * _CUS, 4 * _CUS):
            out.append((v, max(1, -(-blocks // tiles))))
    return sorted(set(out))


def plan_for(x: Tensor, w: Tensor, stride: int, pad: int) -> ConvPlan:
    key = (tuple(x.shape), tuple(w.shape), stride, pad, x.device.index, _mode())
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
        plan.fwd = pick_variant(x.shape[0] * ho * wo, cout)
        plan.bwd = pick_variant(x.shape[0] * x.shape[2] * x.shape[3], cin) if stride == 1 else MIOPEN
        plan.wgrad = wg[len(wg) // 2] if wg else MIOPEN
        plan.tuned = mode == "ours"
    else:
        y = F.conv2d(x, w, stride=stride, padding=pad)
        dy = torch.randn_like(y)
        t = {}
        # the kernel's forward also produces the BatchNorm statistics of y (every conv of the
        # model family feeds a BN), which saves the BN's statistics pass over y: charge MIOpen
        # for that pass (one HBM read of y at ~4.5 TB/s plus a launch)
        stats_pass = y.numel() * y.element_size() / 4.5e6 + 3.0
        t[("fwd", MIOPEN)] = _time(lambda: F.conv2d(x, w, stride=stride, padding=pad)) + \
            stats_pass
        for v in variants_for(cout):
            t[("fwd", v)] = _time(lambda: conv2d_fwd(x, w, stride, pad, v, with_stats=True))
        t[("bwd", MIOPEN)] = _time(lambda: _miopen_bwd(dy, x, w, stride, pad, [True, False, False]))
        if stride == 1:
            for v in variants_for(cin):
                t[("bwd", v)] = _time(lambda: conv2d_bwd_data(dy, w, pad, v))
        t[("wgrad", MIOPEN)] = _time(lambda: _miopen_bwd(dy, x, w, stride, pad,
                                                         [False, True, False]))
        for c in wg:
            t[("wgrad", c)] = _time(lambda: conv2d_wgrad(x, dy, k, stride, pad, c[0], c[1]))
        for kind in ("fwd", "bwd", "wgrad"):
            best = min((v for (kd, _), v in t.items() if kd == kind))
            choice = next(c for (kd, c), v in t.items() if kd == kind and v == best)
            setattr(plan, kind, choice)
        plan.times = {f"{kd}:{c}": round(v, 1) for (kd, c), v in t.items()}
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
        elif want_stats:
            y, (part, _) = conv2d_fwd(x, w, stride, pad, plan.fwd, with_stats=True)
        else:
            y = conv2d_fwd(x, w, stride, pad, plan.fwd)
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pad, plan)
        ctx.join = join.register() if join is not None else None
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
            lk = ctx.bn_link
            # the BN partials need the COMPLETE gradient of x: not from a join's first arriver
            use_bn = (lk is not None and plan.bwd != MIOPEN and lk.x.shape == x.shape
                      and (join is None or other is not None))
            if plan.bwd == MIOPEN:
                dx = _miopen_bwd(dy, x, w, stride, pad, [True, False, False])[0]
                if other is not None:
                    dx.add_(other)
            elif use_bn:
                dx, (part, rpb) = conv2d_bwd_data(dy, w, pad, plan.bwd, addend=other,
                                                  bn=(lk.x, lk.mask, lk.mean))
                lk.publish(part, rpb, dx)
            else:
                dx = conv2d_bwd_data(dy, w, pad, plan.bwd, addend=other)
            if join is not None and join.park_or_take(dx):
                dx = None
        if ctx.needs_input_grad[1]:
            side = None
            if _ASYNC_WGRAD and dy.is_cuda:
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
        return y, ((part, TILES[plan.fwd][0]) if want else None)
