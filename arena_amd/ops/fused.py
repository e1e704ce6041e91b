"""Functional API over the native kernels with device dispatch.

GPU tensors -> HIP kernels in ``arena_amd._C`` (raises if the extension is missing: no silent
fallback); CPU tensors -> the bit-compatible PyTorch reference in :mod:`arena_amd.ops.reference`.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import _ext, reference

Tensor = torch.Tensor


def _impl(t: Tensor):
    return _ext.load() if t.is_cuda else reference


def linear_fwd(x: Tensor, W: Tensor, Y: Tensor, bias: Optional[Tensor] = None, *,
               x_scale: float = 1.0, idx: Optional[Tensor] = None,
               cursor: Optional[Tensor] = None, batch: int = 0, act: int = 1,
               keep_prob: float = 1.0, seed: int = 0, step: Optional[Tensor] = None) -> Tensor:
    """Y = dropout(act(gather(x)·scale @ W + bias)). ``act``: 0 identity, 1 ReLU."""
    _impl(W).linear_fwd(x, float(x_scale), idx, cursor, int(batch), W, bias, Y, int(act),
                        float(keep_prob), int(seed), step)
    return Y


def xent_head(H: Tensor, W2: Tensor, b2: Optional[Tensor], labels: Tensor, *,
              loss_acc: Tensor, correct_acc: Tensor, idx: Optional[Tensor] = None,
              cursor: Optional[Tensor] = None, batch: int = 0,
              dlogits: Optional[Tensor] = None, dZ: Optional[Tensor] = None,
              keep_prob: float = 1.0, relu_mask: bool = True, loss_scale: float = 1.0,
              hist_step: Optional[Tensor] = None, ctr_dst: Optional[Tensor] = None,
              ctr_src: Optional[Tensor] = None, ctr_add: int = 0) -> None:
    _impl(H).xent_head(H, W2, b2, labels, idx, cursor, int(batch), dlogits, dZ, float(keep_prob),
                       bool(relu_mask), float(loss_scale), loss_acc, correct_acc, hist_step,
                       ctr_dst, ctr_src, int(ctr_add))


def mlp_fwd_logits(x: Tensor, W1: Tensor, b1: Tensor, H: Tensor, W2: Tensor, logits2: Tensor, *,
                   W2_copy: Optional[Tensor] = None, xb: Optional[Tensor] = None,
                   labels: Optional[Tensor] = None, yb: Optional[Tensor] = None,
                   x_scale: float = 1.0,
                   idx: Optional[Tensor] = None, cursor: Optional[Tensor] = None, batch: int = 0,
                   keep_prob: float = 1.0, seed: int = 0, step: Optional[Tensor] = None,
                   ctr_dst: Optional[Tensor] = None, ctr_src: Optional[Tensor] = None,
                   ctr_add: int = 0, rows: Optional[Tensor] = None) -> None:
    """H = dropout(relu(x·W1ᵀ+b1)) and logits2[step & 1] += H·W2ᵀ in ONE launch.

    ``logits2`` is [2, M, C]; the consuming wgrad (head mode) zeroes the other buffer each step.
    With ``xb``/``labels``/``yb`` the gathered u8 batch rows and their labels are published for the
    backward kernel (so it skips the cursor -> permutation -> row dependency chain).
    ``rows`` (optional): this step's dataset rows, as the previous ``wgrad_grouped`` wrote them
    with ``next_rows`` -- must equal ``idx[(cursor * batch + r) % len]``.
    """
    _impl(H).mlp_fwd_logits(x, float(x_scale), idx, cursor, int(batch), W1, b1, H,
                            float(keep_prob), int(seed), step, W2, W2_copy, logits2, xb, labels, yb,
                            ctr_dst, ctr_src, int(ctr_add), rows)


def wgrad_grouped(xs: Sequence[Tensor], dzs: Sequence[Optional[Tensor]], outW: Sequence[Tensor],
                  outB: Sequence[Optional[Tensor]], *, x_scales: Sequence[float],
                  gather: Sequence[bool], idx: Optional[Tensor] = None,
                  cursor: Optional[Tensor] = None, cursor_off: int = 0, batch: int = 0,
                  head_modes: Optional[Sequence[int]] = None, head_w2=None, head_h=None,
                  head_keep_prob: float = 1.0, head_logits2: Optional[Tensor] = None,
                  head_step: Optional[Tensor] = None, head_step_off: int = 0,
                  head_b2: Optional[Tensor] = None, head_labels: Optional[Tensor] = None,
                  head_loss_scale: float = 1.0, head_loss_acc: Optional[Tensor] = None,
                  head_correct_acc: Optional[Tensor] = None,
                  mode: int = 0, mW=None, vW=None, mB=None, vB=None, lr: float = 1e-3,
                  lr_t: Optional[Tensor] = None, betas=(0.9, 0.999), eps: float = 1e-8,
                  weight_decay: float = 0.0, t_step: Optional[Tensor] = None,
                  grad_scale: float = 1.0, tf_style: bool = False,
                  ctr_dst: Optional[Tensor] = None, ctr_src: Optional[Tensor] = None,
                  ctr_add: int = 0, next_rows: Optional[Tensor] = None,
                  next_rows_perm: Optional[Tensor] = None, head_parity: int = -1) -> None:
    """dW_i = dz_iᵀ·gather(x_i), db_i = Σ_rows dz_i for up to 2 layers in one launch.

    Head modes (fused MLP step): every workgroup recomputes softmax-xent from ``head_logits2``
    (+ ``head_b2``, ``head_labels``); ``head_modes[i]`` 1 -> dz = dlogits (output layer),
    2 -> dz = (dlogits·head_w2[i]) ⊙ (head_h[i] > 0) / head_keep_prob (hidden layer).
    ``head_parity`` 0/1 names this step's logits buffer at launch (it must equal the counter's
    parity); -1 derives it from ``head_step`` in-kernel.
    mode 0 writes ``grad_scale * dW`` into ``outW`` (e.g. views of the flat all-reduce bucket);
    mode 1 applies Adam in place to parameters ``outW``/``outB`` with state ``mW,vW,mB,vB``.
    """
    n = len(xs)
    none = [None] * n
    hm = list(head_modes) if head_modes is not None else [0] * n
    _impl(outW[0]).wgrad_grouped(
        list(xs), [float(s) for s in x_scales], [bool(g) for g in gather], idx, cursor,
        int(cursor_off), int(batch), list(dzs), [int(m) for m in hm], list(head_w2 or none),
        list(head_h or none), float(head_keep_prob), head_logits2, head_step, int(head_step_off),
        head_b2, head_labels, float(head_loss_scale), head_loss_acc, head_correct_acc, int(mode),
        list(outW), list(outB), list(mW or none), list(vW or none), list(mB or none),
        list(vB or none), float(lr), lr_t, float(betas[0]), float(betas[1]), float(eps),
        float(weight_decay), t_step, float(grad_scale), bool(tf_style), ctr_dst, ctr_src,
        int(ctr_add), next_rows, next_rows_perm, int(head_parity))


def adam_flat(P: Tensor, M: Tensor, V: Tensor, G: Tensor, *, lr: float = 1e-3,
              lr_t: Optional[Tensor] = None, betas=(0.9, 0.999), eps: float = 1e-8,
              weight_decay: float = 0.0, t_step: Optional[Tensor] = None,
              grad_scale: float = 1.0, tf_style: bool = False,
              ctr_dst: Optional[Tensor] = None, ctr_src: Optional[Tensor] = None,
              ctr_add: int = 0) -> None:
    _impl(P).adam_flat(P, M, V, G, float(lr), lr_t, float(betas[0]), float(betas[1]), float(eps),
                       float(weight_decay), t_step, float(grad_scale), bool(tf_style), ctr_dst,
                       ctr_src, int(ctr_add))


def sgd_flat(P: Tensor, G: Tensor, *, lr: float, lr_t: Optional[Tensor] = None,
             grad_scale: float = 1.0) -> None:
    _impl(P).sgd_flat(P, G, float(lr), lr_t, float(grad_scale))


def softmax_xent(logits: Tensor, labels: Tensor, grad_scale: float = 1.0,
                 need_grad: bool = True):
    """Per-row cross-entropy loss and (optionally) dlogits = (softmax - onehot) * grad_scale."""
    out = _impl(logits).softmax_xent(logits, labels, float(grad_scale), bool(need_grad))
    return tuple(out)


def flatten_into(tensors: Sequence[Tensor], offsets: Sequence[int], flat: Tensor,
                 scale: float = 1.0) -> None:
    """flat[off_i : off_i+n_i] = t_i * scale (one multi-tensor launch per 48 tensors)."""
    _impl(flat).mt_copy_scale(list(tensors), [int(o) for o in offsets], flat, float(scale), 0)


def unflatten_from(tensors: Sequence[Tensor], offsets: Sequence[int], flat: Tensor,
                   scale: float = 1.0) -> None:
    """t_i = flat[off_i : off_i+n_i] * scale."""
    _impl(flat).mt_copy_scale(list(tensors), [int(o) for o in offsets], flat, float(scale), 1)


def mt_sgd_master(grads: Sequence[Tensor], offsets: Sequence[int], master: Tensor, mom: Tensor,
                  wbf: Tensor, *, lr: float, momentum: float, weight_decay: float) -> None:
    """One launch (per 48 tensors) of momentum SGD over bf16 grads with fp32 master weights;
    also writes the rounded bf16 weights into ``wbf`` (see ``mt_sgd_master_kernel``)."""
    _impl(master).mt_sgd_master(list(grads), [int(o) for o in offsets], master, mom, wbf,
                                float(lr), float(momentum), float(weight_decay))


def shard_sgd(grad: Tensor, w32: Tensor, mom: Tensor, wbf: Optional[Tensor] = None, *, lr: float,
              momentum: float, weight_decay: float, scale: float) -> None:
    """Momentum SGD over one flat range (a rank's shard of a reduce-scattered bucket):
    d = grad * scale + wd * w32; mom = momentum * mom + d; w32 -= lr * mom; with bf16 ``grad``
    the fp32 ``w32`` are masters and ``wbf`` receives the rounded bf16 weights."""
    _impl(w32).shard_sgd(grad, w32, mom, wbf, float(lr), float(momentum), float(weight_decay),
                         float(scale))
