"""Fused training BatchNorm (+ residual add) (+ ReLU) for NHWC activations.

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` whose forward can also add a residual tensor
and apply ReLU: ``y = relu(bn(x) + residual)``. That is the whole tail of a ResNet bottleneck in
one module. On an MI355X, with a channels_last bf16/fp32 input and a supported channel count,
it runs the HIP kernels in ``csrc/ops/bn_kernels.hip``:

* forward: 2 launches (statistics, then apply + ReLU mask bits); the statistics come from the
  producing convolution's epilogue when it ran on the MFMA kernel (then 1 launch).
  The statistics pass and the conv epilogue accumulate fp64 sums with fire-and-forget
  memory-side atomics, and the apply pass derives its coefficients from those sums itself: no
  finalize launch between them (it used to merge up to 3136 per-tile partials per channel);
* backward: 2 launches (reduction into this layer's own fp64 sums, then dx and the residual
  gradient, which derives its coefficients from the sums).

The sums are zeroed by a later kernel of the same layer instead of a launch of their own: the
forward's by the backward dx pass, the backward's (``_BwdAcc``, one set per module) by the
next forward's apply pass.

Otherwise it runs the same math as stock PyTorch ops. That includes CPU tensors, which serve as
the reference.

Semantics match ``nn.BatchNorm2d`` in training and eval mode:

* batch statistics with the biased variance for normalisation;
* running statistics updated with ``momentum`` and the unbiased variance;
* the ReLU mask is the saved output's sign (y > 0), stored as one bit per element.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from . import _ext, conv

SUPPORTED_C = {8, 16, 32, 64, 128, 256, 512, 1024, 2048}


def kernel_ok(x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> bool:
    """Shapes/layouts the HIP kernels take (everything else runs the PyTorch path)."""
    ok = (x.is_cuda and x.dim() == 4 and x.shape[1] in SUPPORTED_C and x.numel() > 0
          and x.dtype in (torch.bfloat16, torch.float32)
          and x.is_contiguous(memory_format=torch.channels_last))
    if ok and residual is not None:
        ok = (residual.shape == x.shape and residual.dtype == x.dtype
              and residual.is_contiguous(memory_format=torch.channels_last))
    return ok


def reference(x, residual, weight, bias, running_mean, running_var, training, momentum, eps,
              relu):
    """The PyTorch composition the kernels implement (CPU path and numerics reference)."""
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def acc_rep() -> int:
    """Replicas per fp64 accumulator set (csrc/ops/abi.h ARENA_ACC_REP): a set is [rep, 2, C];
    producers with many blocks (the conv epilogues) spread their same-address atomics over the
    replicas and every reader sums them."""
    return int(getattr(_ext.load(), "acc_rep", 1))


def acc_totals(t: torch.Tensor) -> torch.Tensor:
    """The [2, C] totals of an accumulator set (its replicas summed)."""
    return t.reshape(-1, 2, t.shape[-1]).sum(0)


class FinishedStats:
    """Batch statistics of a conv output accumulated inside the conv kernel: the fp64 [rep, 2, C]
    accumulator set (sum y, sum y^2, spread over ``acc_rep()`` replicas) its epilogue added into
    with memory-side atomics (``conv2d_fwd(..., with_stats=True, final=True)``). The BN layer
    consuming it skips its statistics pass; its apply pass derives the coefficients from the
    sums, and its backward dx pass zeroes the set, which returns to a rotating pool (a set whose
    backward never ran is zeroed on the stream before the pool hands it out again)."""
    __slots__ = ("fin",)

    def __init__(self, fin: torch.Tensor):
        self.fin = fin

    def sums(self) -> torch.Tensor:
        """[2, C]: (sum y, sum y^2)."""
        return acc_totals(self.fin)

    def discard(self) -> None:
        self.fin.zero_()


class ResidualMask:
    """The residual gradient of ``relu(bn3(x) + r)`` is dy * ReLU mask. When r is the output of
    another fused BN (a downsample block's ``down_bn``), bn3's backward returns dy itself for r and
    hands over the mask here, and down_bn's backward applies it as if it had a ReLU: its reduction
    and dx passes already read a mask, so dy * mask is never written. The gradient down_bn
    receives is the unmasked dy whenever bn3 published, so ``take`` always returns the mask then.
    bn3 only publishes when down_bn ran on the fused kernels (``armed`` by its forward), the only
    path whose backward takes the mask.

    down_bn's forward also leaves its input, batch mean and backward-sum set here (``x2``,
    ``mean2``, ``bacc2``): bn3's dx pass, which holds the masked dy anyway, then adds down_bn's
    backward sums as it streams (``bn_bwd(x2=...)``) and publishes them, and down_bn's backward
    skips its reduction pass (ARENA_RES_SUMS=0: down_bn reduces itself)."""
    __slots__ = ("armed", "mask", "x2", "mean2", "bacc2", "sums")

    def __init__(self):
        self.armed, self.mask = False, None
        self.x2 = self.mean2 = self.bacc2 = self.sums = None

    def publish(self, mask: torch.Tensor, sums: Optional[torch.Tensor] = None) -> None:
        self.mask, self.sums = mask, sums

    def take(self):
        m, self.mask = self.mask, None
        return m

    def take_sums(self):
        s, self.sums = self.sums, None
        self.x2 = self.mean2 = self.bacc2 = None
        return s


_RES_SUMS = os.environ.get("ARENA_RES_SUMS", "1") == "1"


def set_res_sums(on: bool) -> None:
    global _RES_SUMS
    _RES_SUMS = bool(on)


_FIN_BWD = True


def set_fin_bwd(on: bool) -> None:
    """A/B switch: backward sums in the layer's own set, coefficients derived in the dx pass (on,
    default) or a pool set and a finalize launch (off)."""
    global _FIN_BWD
    _FIN_BWD = bool(on)


class _BwdAcc:
    """A BN layer's own fp64 [rep, 2, C] backward sums (``bn_bwd(acc_b=...)``, ``acc_rep()``
    replicas). The backward's dx pass leaves them in place; the layer's next forward apply pass
    zeroes them (``bn_fwd(zero_b=...)``).
    ``dirty`` tracks that on the host: a backward that finds the set still dirty (no forward ran in
    between) zeroes it first. One set per module keeps captured graphs valid: every replay's
    forward zeroes the set its previous replay's backward filled."""
    __slots__ = ("t", "dirty")

    def __init__(self):
        self.t, self.dirty = None, False

    def take_zero(self):
        """The set for the forward apply pass to zero, or None."""
        if self.t is None or not self.dirty:
            return None
        self.dirty = False
        return self.t

    def for_backward(self, like: torch.Tensor, c: int) -> torch.Tensor:
        n = acc_rep() * 2 * c
        if self.t is None or self.t.device != like.device or self.t.numel() != n:
            self.t = torch.zeros(n, dtype=torch.float64, device=like.device)
        elif self.dirty:
            self.t.zero_()
        self.dirty = True
        return self.t


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, training, momentum,
                eps, relu, num_batches=None, stats=None, join=None, link=None, res_out=None,
                res_in=None, bacc=None):
        ext = _ext.load()
        part, rpb, fin = None, 0, None
        if stats is not None and training:
            if isinstance(stats, FinishedStats):
                fin = stats.fin       # summed by the conv epilogue: apply only
            else:
                part, rpb = stats
        y, mean, invstd, mask, facc = ext.bn_fwd(
            x, residual, weight, bias, running_mean, running_var, training, momentum, eps, relu,
            num_batches, part, rpb, fin, zero_b=bacc.take_zero() if bacc is not None else None)
        # the statistics sums stay in place until this layer's backward dx pass zeroes them
        ctx.facc = facc if (facc is not None and facc.numel() > 0) else None
        ctx.bacc = bacc
        # the ReLU mask is kept as bits (M*C/8 bytes), not as a reference to y
        ctx.save_for_backward(x, mask if relu and training else None, mean, invstd, weight)
        ctx.relu, ctx.has_res, ctx.training = relu, residual is not None, training
        ctx.affine = weight is not None
        # the residual is also another op's input: gradients meet in a GradJoin (ops/conv.py)
        ctx.join = join.register() if (join is not None and residual is not None) else None
        # the conv consuming y computes this layer's backward partials (ops/conv.py BNGradLink)
        ctx.link = None
        if link is not None and training and x.dtype == torch.bfloat16:
            link.set_bn(x, mask if relu else None, mean, bacc if _FIN_BWD else None)
            ctx.link = link
        # res_out: this BN's residual is another fused BN's output (see ResidualMask);
        # res_in: this BN's output is that residual
        ctx.res_out = res_out if (res_out is not None and res_out.armed and residual is not None
                                  and relu and training and conv.masked_join()) else None
        ctx.res_in = res_in if training else None
        if res_in is not None:
            res_in.armed = training
            if (training and _RES_SUMS and bacc is not None and _FIN_BWD
                    and x.dtype == torch.bfloat16):
                res_in.x2, res_in.mean2, res_in.bacc2 = x, mean, bacc
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, mean, invstd, weight = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("BatchNormAct2d backward in eval mode is not supported by the "
                               "fused kernels; use train() or the PyTorch path")
        dy = dy.contiguous(memory_format=torch.channels_last)
        ext = ctx.link.take(dy) if ctx.link is not None else None
        relu = ctx.relu
        sums2 = None
        if ctx.res_in is not None:   # the consumer BN handed over its ReLU mask for this dy
            m = ctx.res_in.take()
            if m is not None:
                relu, mask = True, m
                sums2 = ctx.res_in.take_sums()   # and maybe summed this layer's sums too
        # the residual gradient is dy * ReLU mask; when this BN reaches the residual join first
        # and the other consumer's dgrad epilogue takes a masked addend, park (dy, mask) instead
        # of writing that product (one full write of the block input's size saved)
        masked = (ctx.has_res and ctx.relu and mask is not None and conv.masked_join()
                  and ctx.join is not None and ctx.join.active() and ctx.needs_input_grad[1]
                  and ctx.join.other() is None and ctx.join.peer_takes_masked())
        to_res = (not masked and ctx.res_out is not None and ctx.has_res and mask is not None
                  and ctx.needs_input_grad[1] and ctx.join is None)
        ready = bool(ext) and isinstance(ext[0], str)   # ("acc", sums): the conv summed
        if ready:
            acc_b, ext = ext[1], None
        elif sums2 is not None:                         # bn3's dx pass summed them
            acc_b, ext, ready = sums2, None, True
        else:
            acc_b = ctx.bacc.for_backward(x, x.shape[1]) \
                if (ctx.bacc is not None and not ext and _FIN_BWD) else None
        # to_res: the residual BN's backward sums ride along in this dx pass where they can
        ro = ctx.res_out if to_res else None
        s2 = (ro is not None and ro.x2 is not None and acc_b is not None and relu
              and ro.x2.shape == x.shape and ro.x2.dtype == x.dtype)
        acc2 = ro.bacc2.for_backward(ro.x2, x.shape[1]) if s2 else None
        dx, dres, dgamma, dbeta, sums2_out = _ext.load().bn_bwd(
            dy, mask, x, mean, invstd, weight, relu, ctx.has_res and not masked and not to_res,
            ctx.affine, ext[0] if ext else None, ext[1] if ext else 0, acc_b=acc_b,
            zero_f=ctx.facc, acc_ready=ready, x2=ro.x2 if s2 else None,
            mean2=ro.mean2 if s2 else None, acc2=acc2)
        if to_res:
            # sums2_out: the set filled for the residual BN (None: it reduces itself; its set,
            # marked dirty above, is zeroed again by its own backward's for_backward)
            ctx.res_out.publish(mask, sums2_out)
            dres = dy
        elif masked:
            parked = ctx.join.park_or_take(conv.MaskedGrad(dy, mask))
            assert parked, "masked residual gradient must be the join's first arrival"
            dres = None
        elif not ctx.has_res:
            dres = None
        elif ctx.join is not None and ctx.join.active() and ctx.needs_input_grad[1]:
            other = ctx.join.other()
            if other is not None:   # second consumer (the conv usually comes second and fuses)
                dres = dres + other
            if ctx.join.park_or_take(dres):
                dres = None
        return (dx, dres, dgamma if ctx.affine else None,
                dbeta if ctx.affine else None, None, None, None, None, None, None, None, None,
                None, None, None, None, None)


def bn_act(x, residual=None, weight=None, bias=None, running_mean=None, running_var=None,
           training=True, momentum=0.1, eps=1e-5, relu=True):
    """Functional form of :class:`BatchNormAct2d`."""
    if not kernel_ok(x, residual):
        return reference(x, residual, weight, bias, running_mean, running_var, training,
                         momentum, eps, relu)
    return _BNActFn.apply(x, residual, weight, bias, running_mean, running_var, training,
                          momentum, eps, relu)


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` + optional residual add + optional ReLU, fused on MI355X."""

    def __init__(self, num_features: int, act: str = "relu", **kw):
        super().__init__(num_features, **kw)
        if act not in ("relu", "none"):
            raise ValueError(f"act must be 'relu' or 'none', got {act!r}")
        self.relu = act == "relu"
        self._bacc = _BwdAcc()

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                stats=None, join=None, link=None, res_out=None, res_in=None) -> torch.Tensor:
        """``stats``: BatchNorm partials of ``x`` from the producing ``Conv2dNHWC.forward_stats``
        (skips the statistics pass over x; training mode on the fused kernels only).
        ``join``: a ``GradJoin`` the residual's other consumer is registered on.
        ``link``: a ``BNGradLink`` handed to the conv that consumes the output.
        ``res_out`` / ``res_in``: a ``ResidualMask`` shared by the BN whose residual is this
        other BN's output (res_out) and that other BN (res_in)."""
        training = self.training or not self.track_running_stats
        tracking = self.training and self.track_running_stats
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        fused = kernel_ok(x, residual) and not (not training and torch.is_grad_enabled()
                                                and x.requires_grad)
        if fused and training and self.momentum is not None:
            # num_batches_tracked += 1 happens inside the statistics finalize kernel
            return _BNActFn.apply(x, residual, self.weight, self.bias, rm, rv, True,
                                  self.momentum, self.eps, self.relu,
                                  self.num_batches_tracked if tracking else None, stats, join,
                                  link, res_out, res_in, self._bacc)
        if tracking:
            self.num_batches_tracked.add_(1)
        mom = self.momentum if self.momentum is not None else \
            1.0 / float(self.num_batches_tracked)
        if not fused:
            # layouts the kernels do not take, or eval with autograd on: the PyTorch path
            return reference(x, residual, self.weight, self.bias, rm, rv, training, mom,
                             self.eps, self.relu)
        return _BNActFn.apply(x, residual, self.weight, self.bias, rm, rv, training, mom,
                              self.eps, self.relu, None, None, join, link, res_out, res_in,
                              self._bacc)


# ------------------------------------------------------------------------------------------------
# Fused stem: BatchNorm + ReLU + max pool (bn_kernels.hip arena_bn_pool_fwd / _bwd). The pool
# normalises its window reads on the fly, so the BN output and its mask bits are never written;
# its backward gathers the pooled gradient inside the BN passes instead of writing the pool's dx.
# ------------------------------------------------------------------------------------------------
_STEM_POOL_FUSED = True


def set_stem_pool_fused(on: bool) -> None:
    """A/B switch for ``bn_relu_maxpool`` (off: BN apply + max pool kernels)."""
    global _STEM_POOL_FUSED
    _STEM_POOL_FUSED = bool(on)


# The forward also saves x at each window's argmax (pooled size): the backward's sums then come
# from (dy, xsel), two pooled-size streams, instead of x (4x larger) plus the argmax gather
# (ARENA_STEM_XSEL=0: the per-pixel reduction over x).
_STEM_XSEL = os.environ.get("ARENA_STEM_XSEL", "1") == "1"


def set_stem_xsel(on: bool) -> None:
    global _STEM_XSEL
    _STEM_XSEL = bool(on)


class _BNPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, num_batches,
                fin, part, rpb, bacc, k, s, p):
        y, pos, mean, invstd, scale, shift, xsel = _ext.load().bn_pool_fwd(
            x, weight, bias, running_mean, running_var, momentum, eps, num_batches, fin, part,
            rpb, k, s, p, bacc.take_zero(), _STEM_XSEL)
        ctx.save_for_backward(x, pos, mean, invstd, scale, shift, weight, xsel)
        ctx.fin, ctx.bacc, ctx.geom = fin, bacc, (k, s, p)
        ctx.affine = weight is not None
        ctx.mark_non_differentiable(pos)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, pos, mean, invstd, scale, shift, weight, xsel = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx, dgamma, dbeta = _ext.load().bn_pool_bwd(
            dy, pos, x, mean, invstd, scale, shift, weight, ctx.affine, *ctx.geom,
            ctx.bacc.for_backward(x, x.shape[1]), ctx.fin, xsel)
        return (dx, dgamma if ctx.affine else None, dbeta if ctx.affine else None, None, None,
                None, None, None, None, None, None, None, None, None, None)


def bn_relu_maxpool(bn: BatchNormAct2d, pool: nn.Module, x: torch.Tensor, stats=None):
    """``pool(bn(x, stats=stats))`` for a ReLU ``BatchNormAct2d`` followed by a max pool
    (``MaxPool2dNHWC``: kernel_size / stride / padding), fused on MI355X in training mode when the
    statistics come from the producing conv (``FinishedStats`` sums or per-tile partials); the
    two modules otherwise."""
    k, s, p = pool.kernel_size, pool.stride, pool.padding
    fused = (_STEM_POOL_FUSED and bn.training and bn.relu and bn.track_running_stats
             and bn.momentum is not None and stats is not None
             and kernel_ok(x) and x.shape[1] <= 256 and isinstance(k, int) and isinstance(s, int)
             and isinstance(p, int) and (k + s - 1) // s == 2 and 2 * p <= k
             and x.shape[2] + 2 * p >= k and x.shape[3] + 2 * p >= k)
    if not fused:
        return pool(bn(x, stats=stats))
    fin, part, rpb = (stats.fin, None, 0) if isinstance(stats, FinishedStats) else \
        (None, stats[0], int(stats[1]))
    return _BNPoolFn.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.momentum,
                           bn.eps, bn.num_batches_tracked, fin, part, rpb, bn._bacc, k, s, p)
