"""Fused BatchNorm(+residual)(+ReLU) HIP kernels vs an fp32 PyTorch reference (F.batch_norm).

Checks forward output, batch statistics / running-stat updates, eval mode, and the backward
gradients (dx, residual grad, dgamma, dbeta) for fp32 and bf16 NHWC tensors. Reference = the same
composition in fp32 on the (bf16-rounded) inputs, through autograd.
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(4, 64, 14, 14), (2, 256, 7, 7), (8, 32, 9, 11), (3, 2048, 3, 3), (2, 8, 5, 5),
          (16, 64, 56, 56)]


def _ref(x, res, w, b, rm, rv, relu, training=True, mom=0.1, eps=1e-5):
    y = F.batch_norm(x, rm, rv, w, b, training, mom, eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


def _nhwc(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["relu", "relu_res", "plain"])
def test_bn_act_fwd_bwd(shape, dtype, mode):
    from arena_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(0)
    N, C, H, W = shape
    relu, with_res = mode != "plain", mode == "relu_res"
    x = _nhwc((torch.randn(shape, device="cuda") * 2 + 0.5).to(dtype))
    res = _nhwc(torch.randn(shape, device="cuda").to(dtype)) if with_res else None
    m = BatchNormAct2d(C, act="relu" if relu else "none").cuda()
    with torch.no_grad():
        m.weight.copy_(torch.rand(C, device="cuda") + 0.5)
        m.bias.copy_(torch.randn(C, device="cuda") * 0.1)
    rm0, rv0 = m.running_mean.clone(), m.running_var.clone()
    xk = x.detach().clone().requires_grad_(True)
    rk = res.detach().clone().requires_grad_(True) if with_res else None
    y = m(xk, rk)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    # reference in fp32 from the same (rounded) inputs
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True) if with_res else None
    wr = m.weight.detach().clone().requires_grad_(True)
    br = m.bias.detach().clone().requires_grad_(True)
    rmr, rvr = rm0.clone(), rv0.clone()
    yr = _ref(xr, rr, wr, br, rmr, rvr, relu)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(m.running_mean, rmr, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, rvr, rtol=1e-4, atol=1e-5)
    assert int(m.num_batches_tracked) == 1          # incremented by the finalize kernel
    # backward
    g = _nhwc(torch.randn(shape, device="cuda").to(dtype))
    y.backward(g)
    yr.backward(g.float())
    gtol = dict(rtol=2e-3, atol=2e-3) if dtype == torch.float32 else dict(rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(xk.grad.float(), xr.grad, **gtol)
    if with_res:
        torch.testing.assert_close(rk.grad.float(), rr.grad, **gtol)
    scale = max(1.0, float(wr.grad.abs().max()))
    torch.testing.assert_close(m.weight.grad / scale, wr.grad / scale, **gtol)
    scale = max(1.0, float(br.grad.abs().max()))
    torch.testing.assert_close(m.bias.grad / scale, br.grad / scale, **gtol)


def test_bn_statistics_robust_to_large_mean():
    """Welford + Chan merges: a large common offset must not destroy the variance."""
    from arena_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(1)
    # E[x^2] - E[x]^2 in fp32 would lose the unit variance under the 1e6 mean square
    x = _nhwc(torch.randn(32, 64, 28, 28, device="cuda") + 1000.0)
    m = BatchNormAct2d(64, act="none").cuda()
    y = m(x)
    yr = F.batch_norm(x.double(), None, None, m.weight.double(), m.bias.double(), True, 0.1, 1e-5)
    torch.testing.assert_close(y.double(), yr, rtol=1e-3, atol=1e-3)


def test_bn_eval_mode_uses_running_stats():
    from arena_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(2)
    m = BatchNormAct2d(128, act="relu").cuda()
    with torch.no_grad():
        m.running_mean.copy_(torch.randn(128, device="cuda"))
        m.running_var.copy_(torch.rand(128, device="cuda") + 0.5)
    m.eval()
    x = _nhwc(torch.randn(4, 128, 8, 8, device="cuda"))
    with torch.no_grad():
        y = m(x)
    yr = _ref(x, None, m.weight, m.bias, m.running_mean, m.running_var, True, training=False)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)


def test_resnet_tiny_bf16_step_uses_fused_bn():
    """The model's BN layers take the kernel path under autocast + channels_last."""
    from arena_amd.models.resnet import resnet
    from arena_amd.ops import batchnorm
    calls = {"n": 0}
    orig = batchnorm._BNActFn.apply

    def counting(*a):
        calls["n"] += 1
        return orig(*a)

    batchnorm._BNActFn.apply = counting
    try:
        m = resnet("resnet_tiny", num_classes=10, width=16).cuda().to(
            memory_format=torch.channels_last)
        x = _nhwc(torch.randn(4, 3, 64, 64, device="cuda"))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x), torch.randint(0, 10, (4,), device="cuda"))
        loss.backward()
    finally:
        batchnorm._BNActFn.apply = orig
    n_bn = sum(1 for mod in m.modules() if isinstance(mod, batchnorm.BatchNormAct2d))
    assert calls["n"] == n_bn and torch.isfinite(loss)
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def test_cnn_bench_example_runs_with_graph_capture(tmp_path):
    """The ResNet benchmark example end to end on the GPU (tiny ResNet): fused BN under bf16
    autocast, whole-step hipGraph capture, tf_cnn_benchmarks-style output."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, MIOPEN_FIND_MODE="FAST", ARENA_HEARTBEAT_FILE=str(tmp_path / "hb"))
    r = subprocess.run([sys.executable, "-m", "arena_amd.examples.cnn_bench", "--model",
                        "resnet_tiny", "--width", "16", "--image_size", "64", "--num_classes",
                        "10", "--batch_size", "16", "--num_batches", "6",
                        "--num_warmup_batches", "2", "--display_every", "3", "--json"],
                       capture_output=True, text=True, timeout=240, env=env,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "total images/sec:" in r.stdout
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["exec"] == "hipgraph" and res["images_per_s"] > 0
    assert (tmp_path / "hb").exists()          # progress heartbeats were written


@pytest.mark.parametrize("shape", [(4, 128, 14, 14), (2, 256, 7, 7), (8, 64, 28, 28)])
def test_conv_finished_stats_feed_bn(shape):
    """Statistics accumulated by the conv epilogue (fp64 memory-side atomics) and finished by the
    BN layer's per-channel finalize give the same BN forward/backward and running statistics as
    the fp32 reference; the pool of accumulator sets wraps around correctly."""
    from arena_amd.ops import conv
    from arena_amd.ops.batchnorm import BatchNormAct2d, FinishedStats
    torch.manual_seed(1)
    N, C, H, W = shape
    x = _nhwc(torch.randn(N, 64, H, W, device="cuda").to(torch.bfloat16))
    w = _nhwc((torch.randn(C, 64, 3, 3, device="cuda") * 0.05).to(torch.bfloat16))
    for rep in range(130):   # more uses than the pool has sets (128)
        y, st = conv.conv2d_fwd(x, w, 1, 1, with_stats=True, final=True)
        assert isinstance(st, FinishedStats) and st.fin.shape[-2:] == (2, C)
        assert st.fin.dtype == torch.float64
        yf = y.double()
        Mrows = N * H * W
        tot = st.sums()
        assert torch.allclose(tot[0] / Mrows, yf.mean(dim=(0, 2, 3)), rtol=1e-5, atol=1e-6)
        assert torch.allclose(tot[1] / Mrows, (yf * yf).mean(dim=(0, 2, 3)), rtol=1e-5,
                              atol=1e-6)
        if rep < 129:
            st.discard()      # what a BN layer's finalize does: the set is zero again
    m = BatchNormAct2d(C).cuda()
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(m.state_dict())
    y.requires_grad_()
    yr = y.detach().float().requires_grad_()
    out = m(y, stats=st)
    outr = F.relu(ref(yr))
    assert (out.float() - outr).abs().max() < 3e-2
    assert torch.allclose(m.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(m.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
    assert int(m.num_batches_tracked) == 1
    g = torch.randn_like(outr)
    out.backward(g.to(out.dtype))
    outr.backward(g)
    assert (y.grad.float() - yr.grad).abs().max() / yr.grad.abs().max() < 3e-2
    # (bf16 output gradient in, fp32 reference: compare at the scale of the largest entry)
    for a, b in ((m.weight.grad, ref.weight.grad), (m.bias.grad, ref.bias.grad)):
        assert (a - b).abs().max() / b.abs().max() < 1e-2


def test_resnet_step_finished_stats_match_partials():
    """A ResNet training step with the finished-statistics path (default) against the per-tile
    partials + finalize path: same loss, gradients and running statistics to rounding, and a
    captured hipGraph replays it consistently."""
    from arena_amd.models import resnet as R
    from arena_amd.ops import conv
    torch.manual_seed(0)
    out = {}
    try:
        for final in (False, True):
            conv.set_bn_final(final)
            torch.manual_seed(0)
            net = R.resnet("resnet_tiny", num_classes=10, width=64).cuda().to(
                memory_format=torch.channels_last)
            x = _nhwc(torch.randn(8, 3, 64, 64, device="cuda"))
            y = torch.randint(0, 10, (8,), device="cuda")
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(net(x), y)
            loss.backward()
            out[final] = (float(loss), {n: p.grad.float().clone() for n, p in net.named_parameters()},
                          {n: b.clone() for n, b in net.named_buffers()})
    finally:
        conv.set_bn_final(True)
    la, ga, ba = out[False]
    lb, gb, bb = out[True]
    assert abs(la - lb) < 1e-3 * max(1.0, abs(la))
    for n in ga:
        d = float((ga[n] - gb[n]).abs().max())
        assert d <= 2e-2 * max(1e-3, float(ga[n].abs().max())), (n, d)
    for n in ba:
        if ba[n].dtype.is_floating_point:
            assert torch.allclose(ba[n], bb[n], rtol=1e-3, atol=1e-4), n
        else:
            assert torch.equal(ba[n], bb[n]), n


@pytest.mark.parametrize("C", [64, 512, 2048])
def test_bn_accumulators_rezeroed_across_steps(C):
    """The statistics sums are zeroed by later kernels of the same layer (forward sums by the
    backward dx pass, backward sums by the next forward apply pass), not by a finalize launch:
    repeated training steps, training-mode forwards with no backward in between, and a graph
    replay must all see clean sums (checked against nn.BatchNorm2d at every step)."""
    from arena_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(3)
    shape = (4, C, 7, 7)
    m = BatchNormAct2d(C).cuda()
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(m.state_dict())

    def step(i):
        x = _nhwc(torch.randn(shape, device="cuda") * (1 + i) + i)
        g = _nhwc(torch.randn(shape, device="cuda"))
        xk = x.clone().requires_grad_(True)
        xr = x.clone().requires_grad_(True)
        y = m(xk)
        yr = F.relu(ref(xr))
        torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
        y.backward(g)
        yr.backward(g)
        torch.testing.assert_close(xk.grad, xr.grad, rtol=2e-3, atol=2e-3)
        torch.testing.assert_close(m.weight.grad, ref.weight.grad, rtol=2e-3, atol=2e-3)
        m.weight.grad = m.bias.grad = ref.weight.grad = ref.bias.grad = None

    for i in range(3):
        step(i)
    with torch.no_grad():   # training-mode forwards whose backward never runs
        for i in range(2):
            x = _nhwc(torch.randn(shape, device="cuda"))
            torch.testing.assert_close(m(x), F.relu(ref(x)), rtol=1e-4, atol=1e-4)
    step(5)
    torch.testing.assert_close(m.running_mean, ref.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
    assert int(m.num_batches_tracked) == int(ref.num_batches_tracked)


@pytest.mark.parametrize("dtype,partials,pad", [(torch.bfloat16, False, 1), (torch.float32, False, 1),
                                                (torch.bfloat16, True, 1), (torch.bfloat16, False, 0)])
@pytest.mark.parametrize("xsel", [True, False])
def test_bn_relu_maxpool_fused_matches_modules(dtype, partials, pad, xsel):
    """The fused stem (BN + ReLU + 3x3/2 max pool, statistics summed by the conv epilogue):
    pooled output bit-identical to BatchNormAct2d + MaxPool2dNHWC, same running statistics,
    gradients equal to rounding (the fused backward does not round the pooled gradient to the
    activation dtype before the BN reduction), over repeated steps (accumulator re-zeroing).
    xsel: the backward's sums from the forward's saved argmax inputs (default) or per pixel."""
    from arena_amd.ops import batchnorm, conv
    from arena_amd.ops.pool import MaxPool2dNHWC
    batchnorm.set_stem_xsel(xsel)
    torch.manual_seed(4)
    N, Cin, C, H, W = 4, 64, 64, 18, 17
    mods = []
    for _ in range(2):
        bn = batchnorm.BatchNormAct2d(C).cuda()
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.5, 1.5, C))
            bn.bias.copy_(torch.linspace(-0.2, 0.3, C))
        mods.append((bn, MaxPool2dNHWC(3, 2, pad)))   # pad 1: the 2x2-quad backward kernels
    wt = _nhwc((torch.randn(C, Cin, 3, 3, device="cuda") * 0.05).to(torch.bfloat16))
    try:
        for step in range(3):
            xin = _nhwc(torch.randn(N, Cin, H, W, device="cuda").to(torch.bfloat16))
            g = None
            outs = []
            for fused, (bn, pool) in zip((True, False), mods):
                batchnorm.set_stem_pool_fused(fused)
                y, st = conv.conv2d_fwd(xin, wt, 1, 1, with_stats=True, final=not partials)
                y = y.to(dtype).detach().requires_grad_(True) if dtype != torch.bfloat16 else \
                    y.detach().requires_grad_(True)
                if dtype != torch.bfloat16:     # fp32 BN input: a statistics pass, not the sums
                    st.discard()
                    st = batchnorm.FinishedStats(st.fin)
                    with torch.no_grad():   # replica 0 holds the sums, the others stay zero
                        yf = y.double()
                        f = st.fin.view(-1, 2, C)
                        f[0, 0].copy_(yf.sum(dim=(0, 2, 3)))
                        f[0, 1].copy_((yf * yf).sum(dim=(0, 2, 3)))
                out = batchnorm.bn_relu_maxpool(bn, pool, y, st)
                if g is None:
                    g = _nhwc(torch.randn(out.shape, device="cuda").to(out.dtype))
                out.backward(g)
                outs.append((out.detach(), y.grad, bn.weight.grad.clone(), bn.bias.grad.clone()))
                bn.weight.grad = bn.bias.grad = None
            (o1, dx1, dw1, db1), (o2, dx2, dw2, db2) = outs
            assert torch.equal(o1, o2), step
            tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4,
                                                                                   atol=1e-5)
            torch.testing.assert_close(dx1.float(), dx2.float(), **tol)
            # per-channel sums over bf16-rounded vs fp32 pool gradients: compare at the scale of
            # the largest entry
            lim = 1e-2 if dtype == torch.bfloat16 else 1e-4
            for a, b in ((dw1, dw2), (db1, db2)):
                assert float((a - b).abs().max()) <= lim * float(b.abs().max()), (step, a, b)
            torch.testing.assert_close(mods[0][0].running_var, mods[1][0].running_var)
            assert int(mods[0][0].num_batches_tracked) == step + 1
    finally:
        batchnorm.set_stem_pool_fused(True)
        batchnorm.set_stem_xsel(True)
