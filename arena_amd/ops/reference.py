"""Plain-PyTorch fp32 reference implementations of every arena_amd HIP kernel.

Used (a) as the numerics oracle in tests and (b) as the implementation for CPU tensors (the
multi-process gloo paths that run without a GPU). Semantics match csrc/ops/mlp_kernels.hip
exactly, including the counter-hash dropout mask, the device step counters and the gather.
"""
from __future__ import annotations

import math

import torch

_M32 = 0xFFFFFFFF


def _mul32(h: torch.Tensor, c: int) -> torch.Tensor:
    """(h * c) mod 2**32 for int64 tensors holding uint32 values, without int64 overflow."""
    lo = h & 0xFFFF
    hi = h >> 16
    return ((lo * c) + (((hi * c) & 0xFFFF) << 16)) & _M32


def _mix32(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = _mul32(h, 0x7FEB352D)
    h = h ^ (h >> 15)
    h = _mul32(h, 0x846CA68B)
    h = h ^ (h >> 16)
    return h


def hash4(seed: int, step: int, rows: torch.Tensor, cols: torch.Tensor) -> torch.Tensor:
    """uint32 hash of (seed, step, row, col) -- bit-identical to arena::hash4 (common.h)."""
    h = torch.full_like(rows, (seed & _M32) ^ 0x9E3779B9, dtype=torch.int64)
    h = _mix32(h)
    h = _mix32(h ^ _mul32(torch.full_like(h, step & _M32), 0x85EBCA77))
    h = _mix32(h ^ _mul32(rows.to(torch.int64) & _M32, 0xC2B2AE3D))
    h = _mix32(h ^ _mul32(cols.to(torch.int64) & _M32, 0x27D4EB2F))
    return h


def keep_threshold(keep_prob: float) -> int:
    return 0xFFFFFFFF if keep_prob >= 1.0 else int(keep_prob * 4294967296.0)


def dropout_keep_mask(M: int, N: int, keep_prob: float, seed: int, step: int,
                      device=None) -> torch.Tensor:
    """Boolean [M, N] keep-mask used by linear_fwd's fused dropout."""
    if keep_prob >= 1.0:
        return torch.ones(M, N, dtype=torch.bool, device=device)
    rows = torch.arange(M, device=device, dtype=torch.int64).unsqueeze(1).expand(M, N)
    cols = torch.arange(N, device=device, dtype=torch.int64).unsqueeze(0).expand(M, N)
    return hash4(seed, step, rows, cols) < keep_threshold(keep_prob)


def _cursor_val(cursor: torch.Tensor | None, off: int) -> int:
    return (int(cursor.reshape(-1)[0].item()) if cursor is not None else 0) + off


def gather_rows(x: torch.Tensor, idx: torch.Tensor | None, cursor: torch.Tensor | None,
                batch: int, M: int, cursor_off: int = 0) -> torch.Tensor:
    if idx is None:
        return x[:M]
    cur = _cursor_val(cursor, cursor_off)
    pos = (cur * batch + torch.arange(M, dtype=torch.int64, device=x.device)) % idx.numel()
    return x[idx.to(torch.int64)[pos]]


def linear_fwd(x, x_scale, idx, cursor, batch, W, bias, Y, act, keep_prob, seed, step):
    M = Y.shape[0]
    xr = gather_rows(x, idx, cursor, batch, M).to(torch.float32) * x_scale
    z = xr @ W.t()  # W is [out, in]
    if bias is not None:
        z = z + bias
    if act == 1:
        z = torch.relu(z)
    if keep_prob < 1.0:
        st = int(step.reshape(-1)[0].item()) & _M32 if step is not None else 0
        mask = dropout_keep_mask(M, W.shape[0], keep_prob, seed, st, device=z.device)
        z = torch.where(mask, z * (1.0 / keep_prob), torch.zeros_like(z))
    Y.copy_(z)


def xent_head(H, W2, b2, labels, idx, cursor, batch, dlogits, dZ, keep_prob, relu_mask,
              loss_scale, loss_acc, correct_acc, hist_step, ctr_dst, ctr_src, ctr_add):
    M = H.shape[0]
    hs = int(hist_step.reshape(-1)[0].item()) if hist_step is not None else 0
    L = loss_acc.numel()
    slot = hs % L if L > 1 else 0
    if L > 1:
        loss_acc[(hs + 1) % L] = 0.0
        correct_acc[(hs + 1) % L] = 0
    logits = H @ W2.t()  # W2 is [classes, hidden]
    if b2 is not None:
        logits = logits + b2
    y = gather_rows(labels, idx, cursor, batch, M).to(torch.int64)
    lse = torch.logsumexp(logits, dim=1)
    loss = lse - logits.gather(1, y.unsqueeze(1)).squeeze(1)
    loss_acc[slot] += (loss * loss_scale).sum()
    correct_acc[slot] += (logits.argmax(dim=1) == y).sum().to(correct_acc.dtype)
    if ctr_dst is not None:
        src = int(ctr_src.reshape(-1)[0].item()) if ctr_src is not None else 0
        ctr_dst.fill_(src + ctr_add)
    if dlogits is None:
        return
    g = (torch.softmax(logits, dim=1) - torch.nn.functional.one_hot(y, W2.shape[0]).to(H.dtype))
    g = g * loss_scale
    dlogits.view(M, -1).copy_(g)
    if dZ is None:
        return
    dz = g @ W2
    if relu_mask:
        inv_keep = 1.0 / keep_prob if keep_prob < 1.0 else 1.0
        dz = torch.where(H > 0, dz * inv_keep, torch.zeros_like(dz))
    dZ.view(M, -1).copy_(dz)


def adam_update(p, m, v, g, lr, b1, b2, eps, wd, t, grad_scale, tf_style):
    """In-place Adam on tensors (fp32), same formula as adam_apply in mlp_kernels.hip."""
    g = g * grad_scale + wd * p
    m.mul_(b1).add_(g, alpha=1.0 - b1)
    v.mul_(b2).addcmul_(g, g, value=1.0 - b2)
    bc1 = 1.0 - b1 ** t
    bc2 = 1.0 - b2 ** t
    if tf_style:
        step_size = lr * math.sqrt(bc2) / bc1
        p.sub_(step_size * m / (v.sqrt() + eps))
    else:
        p.sub_((lr / bc1) * m / (v.sqrt() / math.sqrt(bc2) + eps))


def head_dz(dl, w2, h, keep_prob):
    """dz = (dlogits · W2) ⊙ (h > 0) / keep -- ReLU + dropout backward through the head."""
    dz = dl @ w2
    inv_keep = 1.0 / keep_prob
    return torch.where(h > 0, dz * inv_keep, torch.zeros_like(dz))


def mlp_fwd_logits(x, x_scale, idx, cursor, batch, W1, b1, H, keep_prob, seed, step, W2, W2_copy,
                   logits2, xb, labels, yb, ctr_dst, ctr_src, ctr_add, rows=None):
    """Reference for the logits-emitting forward: H and logits2[step & 1] += H·W2ᵀ.
    ``rows`` (the kernel's precomputed gather) must equal the idx/cursor gather; checked here."""
    if rows is not None:
        want = gather_rows(torch.arange(x.shape[0], dtype=torch.int32), idx, cursor, batch,
                           H.shape[0])
        if not torch.equal(rows.to(torch.int32).cpu(), want.cpu()):
            raise AssertionError("precomputed rows disagree with the cursor/permutation gather")
    if ctr_dst is not None:
        src = int(ctr_src.reshape(-1)[0].item()) if ctr_src is not None else 0
        ctr_new = src + ctr_add
    linear_fwd(x, x_scale, idx, cursor, batch, W1, b1, H, 1, keep_prob, seed, step)
    if xb is not None:
        M = H.shape[0]
        xb.copy_(gather_rows(x, idx, cursor, batch, M))
        yb.copy_(gather_rows(labels, idx, cursor, batch, M).to(yb.dtype))
    if W2_copy is not None:
        W2_copy.view_as(W2).copy_(W2)
    st = int(step.reshape(-1)[0].item()) if step is not None else 0
    logits2[st & 1] += H @ W2.t()
    if ctr_dst is not None:
        ctr_dst.fill_(ctr_new)


def _head_dlogits(logits2, hd_step, hd_step_off, b2, labels, idx, cursor, cursor_off, batch,
                  gather_any, loss_scale, loss_acc, correct_acc):
    hstep = int(hd_step.reshape(-1)[0].item()) + hd_step_off
    lg = logits2[hstep & 1].clone()
    M, C = lg.shape
    if b2 is not None:
        lg = lg + b2
    y = (gather_rows(labels, idx, cursor, batch, M, cursor_off) if gather_any
         else labels[:M]).to(torch.int64)
    lse = torch.logsumexp(lg, dim=1)
    loss = lse - lg.gather(1, y.unsqueeze(1)).squeeze(1)
    L = loss_acc.numel()
    loss_acc[(hstep + 1) & (L - 1)] = 0.0
    correct_acc[(hstep + 1) & (L - 1)] = 0
    loss_acc[hstep & (L - 1)] += (loss * loss_scale).sum()
    correct_acc[hstep & (L - 1)] += (lg.argmax(dim=1) == y).sum().to(correct_acc.dtype)
    dl = (torch.softmax(lg, dim=1) - torch.nn.functional.one_hot(y, C).to(lg.dtype)) * loss_scale
    logits2[(hstep + 1) & 1].zero_()
    return dl


def wgrad_grouped(xs, x_scales, gather, idx, cursor, cursor_off, batch, dzs, hd_modes, hd_w2, hd_h,
                  hd_keep_prob, hd_logits2, hd_step, hd_step_off, hd_b2, hd_labels, hd_loss_scale,
                  hd_loss_acc, hd_correct_acc, mode, outW, outB, mW, vW, mB, vB, lr, lr_t, b1, b2,
                  eps, wd, t_step, grad_scale, tf_style, ctr_dst, ctr_src, ctr_add,
                  next_rows=None, next_rows_perm=None, hd_parity=-1):
    if hd_parity >= 0:  # the launch-time parity must name the counter's buffer (kernel contract)
        hs = int(hd_step.reshape(-1)[0].item()) + hd_step_off
        if (hs & 1) != hd_parity:
            raise AssertionError(f"head parity {hd_parity} does not match step {hs}")
    t = int(t_step.reshape(-1)[0].item()) if t_step is not None else 1
    lr_v = float(lr_t.reshape(-1)[0].item()) if lr_t is not None else lr
    dl = None
    if next_rows is not None:  # the next step's dataset rows (cursor = this step + 1)
        st = int(hd_step.reshape(-1)[0].item()) + hd_step_off + 1
        n, L = next_rows.numel(), next_rows_perm.numel()
        pos = (st * n + torch.arange(n)) % L
        next_rows.copy_(next_rows_perm.reshape(-1).cpu()[pos].to(next_rows.device))
    if any(m != 0 for m in hd_modes):
        dl = _head_dlogits(hd_logits2, hd_step, hd_step_off, hd_b2, hd_labels, idx, cursor,
                           cursor_off, batch, any(gather), hd_loss_scale, hd_loss_acc,
                           hd_correct_acc)
    pending = []
    for i in range(len(xs)):
        if hd_modes[i] == 0:
            dz = dzs[i]
        elif hd_modes[i] == 1:
            dz = dl
        else:
            dz = head_dz(dl, hd_w2[i], hd_h[i], hd_keep_prob)
        M = dz.shape[0]
        if gather[i]:
            xr = gather_rows(xs[i], idx, cursor, batch, M, cursor_off)
        else:
            xr = xs[i][:M]
        xr = xr.to(torch.float32) * x_scales[i]
        gw = dz.t() @ xr  # [N, K] = [out, in]
        gb = dz.sum(dim=0)
        pending.append((i, gw, gb))
    for i, gw, gb in pending:
        if mode == 0:
            outW[i].view_as(gw).copy_(gw * grad_scale)
            if outB[i] is not None:
                outB[i].copy_(gb * grad_scale)
        else:
            adam_update(outW[i].view_as(gw), mW[i].view_as(gw), vW[i].view_as(gw), gw, lr_v, b1,
                        b2, eps, wd, t, grad_scale, tf_style)
            if outB[i] is not None:
                adam_update(outB[i], mB[i], vB[i], gb, lr_v, b1, b2, eps, wd, t, grad_scale,
                            tf_style)
    if ctr_dst is not None:
        src = int(ctr_src.reshape(-1)[0].item()) if ctr_src is not None else 0
        ctr_dst.fill_(src + ctr_add)


def adam_flat(P, M, V, G, lr, lr_t, b1, b2, eps, wd, t_step, grad_scale, tf_style, ctr_dst,
              ctr_src, ctr_add):
    t = int(t_step.reshape(-1)[0].item()) if t_step is not None else 1
    lr_v = float(lr_t.reshape(-1)[0].item()) if lr_t is not None else lr
    adam_update(P, M, V, G, lr_v, b1, b2, eps, wd, t, grad_scale, tf_style)
    if ctr_dst is not None:
        src = int(ctr_src.reshape(-1)[0].item()) if ctr_src is not None else 0
        ctr_dst.fill_(src + ctr_add)


def sgd_flat(P, G, lr, lr_t, grad_scale):
    lr_v = float(lr_t.reshape(-1)[0].item()) if lr_t is not None else lr
    P.sub_(G * (lr_v * grad_scale))


def softmax_xent(logits, labels, grad_scale, need_grad):
    lse = torch.logsumexp(logits, dim=1)
    loss = lse - logits.gather(1, labels.unsqueeze(1)).squeeze(1)
    if not need_grad:
        return [loss]
    d = torch.softmax(logits, dim=1)
    d[torch.arange(labels.numel()), labels] -= 1.0
    return [loss, d * grad_scale]


def mt_copy_scale(tensors, offsets, flat, scale, direction):
    for t, off in zip(tensors, offsets):
        n = t.numel()
        if direction == 0:
            flat[off:off + n].copy_(t.reshape(-1) * scale)
        else:
            t.view(-1).copy_(flat[off:off + n] * scale)


def _storage_flat(t):
    """A dense tensor's elements in memory order (channels_last weights included)."""
    return t.as_strided((t.numel(),), (1,), t.storage_offset())


def mt_sgd_master(grads, offsets, master, mom, wbf, lr, momentum, weight_decay):
    for g, off in zip(grads, offsets):
        n = g.numel()
        w, m = master[off:off + n], mom[off:off + n]
        m.mul_(momentum).add_(_storage_flat(g).float() + weight_decay * w)
        w.sub_(lr * m)
        wbf[off:off + n].copy_(w)


def shard_sgd(grad, w32, mom, wbf, lr, momentum, weight_decay, scale):
    """CPU reference of the HIP ``shard_sgd`` kernel (same operation order)."""
    d = grad.float() * scale + weight_decay * w32
    mom.mul_(momentum).add_(d)
    w32.sub_(lr * mom)
    if wbf is not None:
        wbf.copy_(w32)
