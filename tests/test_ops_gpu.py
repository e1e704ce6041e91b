"""Numerics of the native HIP kernels vs the plain-PyTorch fp32 reference (runs on an MI355X)."""
import pytest
import torch

from arena_amd import ops
from arena_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-4, atol=1e-5):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), rtol=rtol, atol=atol)


@pytest.mark.parametrize("M,K,N", [(100, 784, 500), (37, 68, 21), (1, 4, 1), (130, 512, 10),
                                   (256, 1024, 256)])
@pytest.mark.parametrize("act", [0, 1])
def test_linear_fwd_f32(cuda, M, K, N, act):
    g = torch.Generator().manual_seed(M * 7 + K)
    x = torch.randn(M, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) * 0.1).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    Y = torch.empty(M, N, device=cuda)
    ops.linear_fwd(x, W, Y, b, act=act)
    Yr = torch.empty_like(Y)
    ref.linear_fwd(x, 1.0, None, None, 0, W, b, Yr, act, 1.0, 0, None)
    _close(Y, Yr)


def test_linear_fwd_u8_gather_dropout(cuda):
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (1000, 784), generator=g, dtype=torch.uint8).to(cuda)
    idx = torch.randperm(1000, generator=g).to(torch.int32).to(cuda)
    cursor = torch.tensor([7], dtype=torch.int64, device=cuda)
    W = (torch.randn(500, 784, generator=g) * 0.05).to(cuda)
    b = torch.randn(500, generator=g).to(cuda)
    Y = torch.empty(100, 500, device=cuda)
    ops.linear_fwd(data, W, Y, b, x_scale=1 / 255.0, idx=idx, cursor=cursor, batch=100, act=1,
                   keep_prob=0.9, seed=1234, step=cursor)
    Yr = torch.empty_like(Y)
    ref.linear_fwd(data, 1 / 255.0, idx, cursor, 100, W, b, Yr, 1, 0.9, 1234, cursor)
    _close(Y, Yr)
    # the mask really drops ~10 % of the positive activations
    frac = ((Yr == 0) & (torch.relu(Yr) == 0)).float().mean().item()
    assert 0.05 < frac < 0.95


def test_dropout_hash_matches_reference(cuda):
    # x = identity rows, W = I -> Y = dropout(relu(1)) exposes the raw keep-mask
    N = 64
    x = torch.eye(N, device=cuda)
    W = torch.eye(N, device=cuda)
    Y = torch.empty(N, N, device=cuda)
    step = torch.tensor([3], dtype=torch.int64, device=cuda)
    ops.linear_fwd(x, W, Y, torch.ones(N, device=cuda), act=1, keep_prob=0.5, seed=99, step=step)
    mask = ref.dropout_keep_mask(N, N, 0.5, 99, 3)
    assert torch.equal((Y.cpu() > 0), mask)


@pytest.mark.parametrize("M,D,C", [(100, 500, 10), (33, 100, 10), (8, 1024, 16), (5, 64, 3)])
def test_xent_head(cuda, M, D, C):
    g = torch.Generator().manual_seed(D)
    H = torch.relu(torch.randn(M, D, generator=g)).to(cuda)
    W2 = (torch.randn(C, D, generator=g) * 0.1).to(cuda)
    b2 = torch.randn(C, generator=g).to(cuda)
    y = torch.randint(0, C, (M,), generator=g, dtype=torch.uint8).to(cuda)
    outs = {}
    for impl in ("hip", "ref"):
        la = torch.zeros(8, device=cuda)
        ca = torch.zeros(8, dtype=torch.int32, device=cuda)
        dl = torch.empty(M, C, device=cuda)
        dz = torch.empty(M, D, device=cuda)
        A = torch.tensor([5], dtype=torch.int64, device=cuda)
        Bc = torch.zeros(1, dtype=torch.int64, device=cuda)
        args = (H, W2, b2, y, None, None, 0, dl, dz, 0.9, True, 1.0 / M, la, ca, A, Bc, A, 1)
        if impl == "hip":
            from arena_amd.ops import _ext
            _ext.load().xent_head(*args)
        else:
            ref.xent_head(*args)
        torch.cuda.synchronize()
        outs[impl] = (la, ca, dl, dz, Bc)
    h, r = outs["hip"], outs["ref"]
    _close(h[0], r[0], rtol=1e-4, atol=1e-5)
    assert torch.equal(h[1].cpu(), r[1].cpu())
    _close(h[2], r[2])
    _close(h[3], r[3])
    assert int(h[4].item()) == 6


@pytest.mark.parametrize("mode", [0, 1])
def test_wgrad_grouped(cuda, mode):
    g = torch.Generator().manual_seed(mode)
    data = torch.randint(0, 256, (500, 784), generator=g, dtype=torch.uint8).to(cuda)
    idx = torch.randperm(500, generator=g).to(torch.int32).to(cuda)
    cur = torch.tensor([3], dtype=torch.int64, device=cuda)
    Hh = torch.relu(torch.randn(100, 500, generator=g)).to(cuda)
    dz1 = torch.randn(100, 500, generator=g).to(cuda)
    dz2 = torch.randn(100, 10, generator=g).to(cuda)
    res = {}
    for impl in ("hip", "ref"):
        W1 = (torch.randn(500, 784, generator=torch.Generator().manual_seed(1))).to(cuda)
        W2 = (torch.randn(10, 500, generator=torch.Generator().manual_seed(2))).to(cuda)
        b1 = torch.zeros(500, device=cuda)
        b2 = torch.zeros(10, device=cuda)
        st = [torch.full_like(t, 0.01) for t in (W1, W2, b1, b2)] + \
             [torch.full_like(t, 0.02) for t in (W1, W2, b1, b2)]
        t = torch.tensor([4], dtype=torch.int64, device=cuda)
        A = torch.zeros(1, dtype=torch.int64, device=cuda)
        args = ([data, Hh], [1 / 255.0, 1.0], [True, False], idx, cur, -1, 100, [dz1, dz2],
                [0, 0], [None, None], [None, None], 1.0, None, None, 0, None, None, 1.0, None,
                None, mode,
                [W1, W2], [b1, b2], [st[0], st[1]], [st[4], st[5]], [st[2], st[3]],
                [st[6], st[7]], 1e-3, None, 0.9, 0.999, 1e-8, 0.0, t, 0.5, False, A, t, 0)
        if impl == "hip":
            from arena_amd.ops import _ext
            _ext.load().wgrad_grouped(*args, None, None, -1)
        else:
            ref.wgrad_grouped(*args)
        torch.cuda.synchronize()
        res[impl] = (W1, W2, b1, b2, st, A)
    for a, b in zip(res["hip"][:4], res["ref"][:4]):
        _close(a, b, rtol=2e-4, atol=2e-5)
    if mode == 1:
        for a, b in zip(res["hip"][4], res["ref"][4]):
            _close(a, b, rtol=2e-4, atol=2e-6)
    assert int(res["hip"][5].item()) == 4


def test_adam_flat_matches_torch_optim(cuda):
    g = torch.Generator().manual_seed(0)
    n = 4096 + 12
    p0 = torch.randn(n, generator=g)
    P = p0.clone().to(cuda)
    M = torch.zeros(n, device=cuda)
    V = torch.zeros(n, device=cuda)
    tp = torch.nn.Parameter(p0.clone().to(cuda))
    opt = torch.optim.Adam([tp], lr=1e-2, betas=(0.9, 0.99), eps=1e-6)
    t = torch.zeros(1, dtype=torch.int64, device=cuda)
    for step in range(1, 6):
        grad = torch.randn(n, generator=g).to(cuda)
        t.fill_(step)
        ops.adam_flat(P, M, V, grad, lr=1e-2, betas=(0.9, 0.99), eps=1e-6, t_step=t)
        tp.grad = grad.clone()
        opt.step()
    _close(P, tp.detach(), rtol=1e-5, atol=1e-6)


def test_softmax_xent(cuda):
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(257, 1000, generator=g).to(cuda)
    y = torch.randint(0, 1000, (257,), generator=g).to(cuda)
    loss, dl = ops.softmax_xent(logits, y, 1.0 / 257)
    lt = logits.clone().requires_grad_(True)
    l = torch.nn.functional.cross_entropy(lt, y)
    l.backward()
    _close(loss.mean(), l.detach())
    _close(dl, lt.grad)


def test_multi_tensor_flatten_roundtrip(cuda):
    ts = [torch.randn(s, device=cuda) for s in (1, 5, 4096, 1025, 3, 70000)]
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += (t.numel() + 3) // 4 * 4
    flat = torch.zeros(o, device=cuda)
    ops.flatten_into(ts, offs, flat, 2.0)
    for t, off in zip(ts, offs):
        _close(flat[off:off + t.numel()], t * 2)
    outs = [torch.empty_like(t) for t in ts]
    ops.unflatten_from(outs, offs, flat, 0.5)
    for a, b in zip(outs, ts):
        _close(a, b)


def test_fused_linear_autograd(cuda):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(64, 128, generator=g).to(cuda).requires_grad_(True)
    W = (torch.randn(32, 128, generator=g) * 0.1).to(cuda).requires_grad_(True)
    b = torch.randn(32, generator=g).to(cuda).requires_grad_(True)
    y = ops.fused_linear(x, W, b, act=1)
    (y * torch.arange(32, device=cuda)).sum().backward()
    x2, W2, b2 = (t.detach().clone().requires_grad_(True) for t in (x, W, b))
    y2 = torch.relu(x2 @ W2.t() + b2)
    (y2 * torch.arange(32, device=cuda)).sum().backward()
    _close(y, y2)
    _close(x.grad, x2.grad)
    _close(W.grad, W2.grad)
    _close(b.grad, b2.grad)


@pytest.mark.parametrize("M,N,C", [(100, 500, 10), (37, 100, 10), (16, 64, 3)])
def test_mlp_fwd_logits_matches_reference(cuda, M, N, C):
    g = torch.Generator().manual_seed(N + C)
    data = torch.randint(0, 256, (400, 784), generator=g, dtype=torch.uint8).to(cuda)
    idx = torch.randperm(400, generator=g).to(torch.int32).to(cuda)
    W1 = (torch.randn(N, 784, generator=g) * 0.05).to(cuda)
    b1 = (torch.randn(N, generator=g) * 0.1).to(cuda)
    W2 = (torch.randn(C, N, generator=g) * 0.1).to(cuda)
    out = {}
    for impl in ("hip", "ref"):
        A = torch.tensor([3], dtype=torch.int64, device=cuda)
        Bc = torch.zeros(1, dtype=torch.int64, device=cuda)
        H = torch.empty(M, N, device=cuda)
        w2c = torch.empty(C, N, device=cuda)
        lg2 = torch.zeros(2, M, C, device=cuda)
        labels = torch.randint(0, C, (400,), generator=torch.Generator().manual_seed(5),
                               dtype=torch.uint8).to(cuda)
        xb = torch.zeros(M, 784, dtype=torch.uint8, device=cuda)
        yb = torch.zeros(M, dtype=torch.int32, device=cuda)
        args = (data, 1 / 255.0, idx, A, M, W1, b1, H, 0.9, 77, A, W2, w2c, lg2, xb, labels, yb,
                Bc, A, 1)
        if impl == "hip":
            from arena_amd.ops import _ext
            _ext.load().mlp_fwd_logits(*args, None)
        else:
            ref.mlp_fwd_logits(*args)
        torch.cuda.synchronize()
        out[impl] = (H, lg2, Bc, w2c, xb, yb)
    h, r = out["hip"], out["ref"]
    assert torch.equal(h[4].cpu(), r[4].cpu())
    assert torch.equal(h[5].cpu(), r[5].cpu())
    _close(h[0], r[0])
    _close(h[1], r[1], rtol=1e-4, atol=1e-4)
    assert float(h[1][0].abs().sum()) == 0.0  # step 3 -> buffer 1 only
    assert int(h[2].item()) == 4
    _close(h[3], W2)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("parity", [-1, 1])  # from the counter / known at launch (step 5)
def test_wgrad_head_modes(cuda, mode, parity):
    """Both layers' grads from raw logits (softmax recomputed per workgroup) vs the reference."""
    g = torch.Generator().manual_seed(10 + mode)
    M, N, K, C = 100, 500, 784, 10
    data = torch.randint(0, 256, (300, K), generator=g, dtype=torch.uint8).to(cuda)
    labels = torch.randint(0, C, (300,), generator=g, dtype=torch.uint8).to(cuda)
    idx = torch.randperm(300, generator=g).to(torch.int32).to(cuda)
    Hh = torch.relu(torch.randn(M, N, generator=g)).to(cuda)
    Hh[Hh < 0.3] = 0.0
    W2c = (torch.randn(C, N, generator=g) * 0.1).to(cuda)
    lg0 = torch.randn(M, C, generator=g).to(cuda)
    b2v = torch.randn(C, generator=g).to(cuda)
    res = {}
    for impl in ("hip", "ref"):
        cur = torch.tensor([6], dtype=torch.int64, device=cuda)  # B counter: step index 5
        lg2 = torch.zeros(2, M, C, device=cuda)
        lg2[1] = lg0
        lg2[0] = 7.0  # must be zeroed by the launch
        W1 = torch.randn(N, K, generator=torch.Generator().manual_seed(1)).to(cuda) * 0.01
        W2 = torch.randn(C, N, generator=torch.Generator().manual_seed(2)).to(cuda) * 0.01
        b1 = torch.zeros(N, device=cuda)
        b2 = b2v.clone()
        st = [torch.full_like(t, 1e-3) for t in (W1, W2, b1, b2)] + \
             [torch.full_like(t, 1e-4) for t in (W1, W2, b1, b2)]
        la = torch.zeros(8, device=cuda)
        ca = torch.zeros(8, dtype=torch.int32, device=cuda)
        la[6] = 5.0
        args = ([data, Hh], [1 / 255.0, 1.0], [True, False], idx, cur, -1, M, [None, None],
                [2, 1], [W2c, None], [Hh, None], 0.9, lg2, cur, -1, b2v, labels, 1.0 / M, la,
                ca, mode, [W1, W2], [b1, b2], [st[0], st[1]], [st[4], st[5]], [st[2], st[3]],
                [st[6], st[7]], 1e-3, None, 0.9, 0.999, 1e-8, 0.0, cur, 1.0, False, None, None,
                0)
        if impl == "hip":
            from arena_amd.ops import _ext
            _ext.load().wgrad_grouped(*args, None, None, parity)
        else:
            ref.wgrad_grouped(*args, None, None, parity)
        torch.cuda.synchronize()
        res[impl] = (W1, W2, b1, b2, la, ca, lg2)
    h, r = res["hip"], res["ref"]
    for a, b in zip(h[:4], r[:4]):
        _close(a, b, rtol=2e-4, atol=1e-6)
    _close(h[4], r[4], rtol=1e-4, atol=1e-5)
    assert float(h[4][6]) == 0.0  # next slot zeroed
    assert torch.equal(h[5].cpu(), r[5].cpu())
    assert float(h[6][0].abs().sum()) == 0.0  # next logits buffer zeroed
