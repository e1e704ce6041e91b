"""BatchNorm-apply fold: a ReLU BN whose output feeds one convolution is never
written -- the conv stages the BN's input and applies relu(fma(x - mean, scale, shift)) to each
staged chunk in LDS (forward A operand, weight-gradient X operand), and the linked dgrad epilogue
and the BN backward recompute the ReLU bits from x.

The folded operand is bn_apply's arithmetic and rounding, so against the unfused path on the SAME
tile variant every result is bit-identical: forward output and its BN statistics, weight gradient
(fixed-order split reduction), the linked dgrad's dX and BN-backward sums, the BN backward's dx.
Shapes cover the 1x1 generic tiles (tail tile, C = 512) and the 3x3 halo tiles (padded taps,
windows spanning several images, the 31- and 63-wide limits of the two window sizes). Each is
also checked against an fp32 F.conv2d of relu(bn(x)). A whole bottleneck block, fold on vs off,
gives the same outputs and gradients.
"""
import pytest
import torch
import torch.nn.functional as F

from arena_amd.ops import conv

pytestmark = pytest.mark.gpu

FOLD_SHAPES = [  # n, cin, h, w, cout, k
    (3, 128, 7, 7, 256, 1),      # 1x1, 147 rows: one partial tile
    (2, 64, 9, 11, 128, 1),      # 1x1, M = 198: tail rows
    (2, 512, 7, 7, 256, 1),      # the widest folded BN (C = 512)
    (2, 64, 9, 11, 64, 3),       # 3x3 halo, padded taps
    (4, 128, 7, 7, 128, 3),      # halo windows spanning several images
    (2, 128, 9, 31, 128, 3),     # the small window's widest image (31)
    (1, 128, 5, 63, 128, 3),     # the big window's widest image (63)
]


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


def _bn_parts(y1, seed):
    """A BN layer's unfused forward of y1 (statistics from the producing conv's fp64 sums): the
    stored output, its ReLU bits, mean, invstd; and the folded forward's [3, C] table + invstd
    from the SAME sums. Returns (out, mask, mean, invstd, coef, coef_invstd, gamma)."""
    from arena_amd.ops import _ext
    ext = _ext.load()
    c = y1.shape[1]
    g = torch.Generator(device="cuda").manual_seed(seed)
    gamma = torch.rand(c, device="cuda", generator=g) * 1.5 - 0.5    # some negative scales
    beta = torch.randn(c, device="cuda", generator=g) * 0.5
    m = y1.shape[0] * y1.shape[2] * y1.shape[3]
    yf = y1.permute(0, 2, 3, 1).reshape(m, c).double()
    # what the conv epilogue sums, in replica 0 of a [rep, 2, C] set
    from arena_amd.ops.batchnorm import acc_rep
    fin = torch.zeros(acc_rep(), 2, c, dtype=torch.float64, device="cuda")
    fin[0] = torch.stack([yf.sum(0), (yf * yf).sum(0)])
    rm0, rv0 = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    out, mean, invstd, mask, _ = ext.bn_fwd(y1, None, gamma, beta, rm0.clone(), rv0.clone(), True,
                                            0.1, 1e-5, True, None, None, 0, fin)
    rm1, rv1 = rm0.clone(), rv0.clone()
    coef, inv2 = ext.bn_fold_fwd(y1, gamma, beta, rm1, rv1, 0.1, 1e-5, None, stats_fin=fin)
    return out, mask, mean, invstd, coef, inv2, gamma, (rm1, rv1)


@pytest.mark.parametrize("shape", FOLD_SHAPES)
def test_fold_kernels_bit_identical_to_unfused(shape):
    from arena_amd.ops import _ext
    ext = _ext.load()
    n, cin, h, w, cout, k = shape
    pad = k // 2
    g = torch.Generator(device="cuda").manual_seed(cin + k)
    y1 = (torch.randn(n, cin, h, w, device="cuda", generator=g) * 2 + 0.3).to(
        torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, k, k, device="cuda", generator=g) * 0.1).to(
        torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out, mask, mean, invstd, coef, inv2, gamma, _ = _bn_parts(y1, seed=k)
    # the fold's coefficients are the apply pass's: mean, scale, shift, invstd
    assert torch.equal(coef[0], mean) and torch.equal(inv2, invstd)
    # fp32 reference of the consumer: conv of relu(bn(y1)) with the layer's own coefficients
    a32 = torch.relu((y1.float() - coef[0].view(1, -1, 1, 1)) * coef[1].view(1, -1, 1, 1)
                     + coef[2].view(1, -1, 1, 1))
    ref = F.conv2d(a32, wt.float(), padding=pad)
    fvs = conv._fold_fwd_variants(cout, (k, k), 1, pad, w)
    assert fvs, shape
    for v in fvs:
        for fin in (False, True):
            yu = conv.conv2d_fwd(out, wt, 1, pad, v, with_stats=True, final=fin)
            yp = conv.conv2d_fwd(y1, wt, 1, pad, v, with_stats=True, final=fin, pre=coef)
            assert torch.equal(yp[0], yu[0]), (v, fin)
            su = yu[1].sums() if fin else yu[1][0]
            sp = yp[1].sums() if fin else yp[1][0]
            if fin:
                torch.testing.assert_close(sp, su, rtol=1e-9, atol=1e-6)   # fp64 atomics order
            else:
                assert torch.equal(sp, su), v
        assert _rel(yp[0], ref) < 1e-2, (v, _rel(yp[0], ref))
    # weight gradient: the X operand normalised in LDS (padded taps stay zero)
    dy = torch.randn(ref.shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    _, dw_ref, _ = torch.ops.aten.convolution_backward(
        dy.float(), a32.to(torch.bfloat16).float(), wt.float(), None, [1, 1], [pad, pad], [1, 1],
        False, [0, 0], 1, [False, True, False])
    for v in conv.wgrad_variants_for(cin, cout):
        for sp in (1, 3, 0):
            dwu = conv.conv2d_wgrad(out, dy, (k, k), 1, pad, v, sp, out_dtype=torch.float32)
            dwp = conv.conv2d_wgrad(y1, dy, (k, k), 1, pad, v, sp, out_dtype=torch.float32,
                                    pre=coef)
            assert torch.equal(dwp, dwu), (v, sp)
        assert _rel(dwp, dw_ref) < 1e-2, (v, _rel(dwp, dw_ref))
    # the linked dgrad of the consumer: the BN's ReLU bits recomputed from y1 (v2 / halo tiles)
    bvs = conv.v2_variants_for(cin) + conv.halo_variants_for(cin, (k, k), 1, pad, w)
    for v in bvs:
        dxu, (pu, _) = conv.conv2d_bwd_data(dy, wt, pad, v, bn=(y1, mask, mean))
        dxp, (pp, _) = conv.conv2d_bwd_data(dy, wt, pad, v, bn=(y1, None, mean), pre=coef)
        assert torch.equal(dxp, dxu) and torch.equal(pp, pu), v
    # the BN backward with the bits recomputed from x
    d_out = torch.randn(y1.shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    ru = ext.bn_bwd(d_out, mask, y1, mean, invstd, gamma, True, False, True)
    rp = ext.bn_bwd(d_out, None, y1, mean, invstd, gamma, True, False, True, coef=coef)
    # (the reduction's fp64 atomics may order differently: a mismatched ReLU bit would show as
    # a whole element off, so allow only last-bit differences)
    assert _rel(rp[0], ru[0]) < 1e-2
    assert int((rp[0] != ru[0]).sum()) <= max(1, rp[0].numel() // 1000)
    torch.testing.assert_close(rp[2], ru[2], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rp[3], ru[3], rtol=1e-5, atol=1e-5)


def test_fold_coefficients_update_running_stats_from_partials():
    """The partials form (per-tile statistics of the producing conv -> finalize): same table and
    running statistics as the unfused forward."""
    from arena_amd.ops import _ext
    ext = _ext.load()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.randn(4, 128, 14, 14, device="cuda", generator=g)).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wt = (torch.randn(256, 128, 1, 1, device="cuda", generator=g) * 0.1).to(
        torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y, (part, rpb) = conv.conv2d_fwd(x, wt, 1, 0, conv.V2 + 8, with_stats=True)
    gamma = torch.rand(256, device="cuda", generator=g) + 0.5
    beta = torch.randn(256, device="cuda", generator=g)
    rm_a, rv_a = torch.zeros(256, device="cuda"), torch.ones(256, device="cuda")
    rm_b, rv_b = rm_a.clone(), rv_a.clone()
    nb_a = torch.zeros((), dtype=torch.int64, device="cuda")
    nb_b = nb_a.clone()
    _, mean, invstd, _, _ = ext.bn_fwd(y, None, gamma, beta, rm_a, rv_a, True, 0.1, 1e-5, True,
                                       nb_a, part, rpb)
    coef, inv2 = ext.bn_fold_fwd(y, gamma, beta, rm_b, rv_b, 0.1, 1e-5, nb_b, stats_part=part,
                                 stats_rpb=rpb)
    assert torch.equal(coef[0], mean) and torch.equal(inv2, invstd)
    assert torch.equal(coef[1], gamma * invstd) and torch.equal(coef[2], beta)
    assert torch.equal(rm_b, rm_a) and torch.equal(rv_b, rv_a)
    assert int(nb_a) == int(nb_b) == 1


@pytest.mark.parametrize("stride", [1, 2])
def test_bottleneck_fold_matches_unfolded(stride, monkeypatch):
    """Two bottleneck blocks with bn1 / bn2 folded into conv2 / conv3 against the same blocks
    unfolded ON THE SAME TILE VARIANTS (the unfolded convs are given the fold forms' variants):
    forward output, input gradient, every parameter gradient, running statistics."""
    from arena_amd.models import resnet as R
    from arena_amd.ops import batchnorm as B
    conv.set_mode("ours")
    fold0 = conv.bn_fold_enabled()
    conv.set_bn_fold(True)
    try:
        torch.manual_seed(0)
        net = torch.nn.ModuleList([R.Bottleneck(256, 64, stride), R.Bottleneck(256, 64, 1)]).cuda()
        net = net.to(memory_format=torch.channels_last)
        with torch.no_grad():
            for b in net:
                b.bn3.weight.uniform_(0.5, 1.5)
        x0 = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        gg = torch.Generator(device="cuda").manual_seed(7)
        calls = {"n": 0}
        orig = B._BNFoldFn.apply

        def counting(*a):
            calls["n"] += 1
            return orig(*a)

        monkeypatch.setattr(B._BNFoldFn, "apply", counting)
        fold_fn = B.BatchNormAct2d.forward_fold

        def run():
            net.zero_grad(set_to_none=True)
            st = {k: v.clone() for k, v in net.state_dict().items()}
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = net[1](net[0](x))
            # a random output gradient (a uniform one cancels in every BN backward)
            g = torch.randn(y.shape, device="cuda", generator=gg.manual_seed(7)).to(
                y.dtype).contiguous(memory_format=torch.channels_last)
            y.backward(g)
            res = (y.detach().float(), x.grad.float(),
                   {n: p.grad.float().clone() for n, p in net.named_parameters()},
                   {k: v.clone() for k, v in net.state_dict().items()})
            net.load_state_dict(st)
            return res

        out = {"fold": run()}
        # folded: bn1 + bn2 of both blocks, except bn1 of a stride-2 block (3x3 / 2 consumer)
        assert calls["n"] == (4 if stride == 1 else 3), calls
        # the unfolded run on the fold forms' variants: the convs' plans are the same objects
        for plan in conv.plans().values():
            if plan.fwd_fold != conv.MIOPEN:
                plan.fwd, plan.bwd_bn, plan.wgrad = plan.fwd_fold, plan.bwd_bn_fold, \
                    plan.wgrad_fold
        monkeypatch.setattr(B.BatchNormAct2d, "forward_fold",
                            lambda self, x, consumer, stats=None, link=None:
                            (self(x, stats=stats, link=link), None))
        out["plain"] = run()
        monkeypatch.setattr(B.BatchNormAct2d, "forward_fold", fold_fn)
        yf, xf, gf, sf = out["fold"]
        yp, xp, gp, sp = out["plain"]
        bad = {n: _rel(gf[n], v) for n, v in gp.items() if _rel(gf[n], v) > 1e-2}
        assert not bad, bad
        assert _rel(yf, yp) < 1e-2
        assert _rel(xf, xp) < 1e-2
        for k, v in sp.items():   # running statistics, batch counters
            if v.is_floating_point():
                torch.testing.assert_close(sf[k], v, rtol=1e-3, atol=1e-4)
            else:
                assert torch.equal(sf[k], v), k
    finally:
        conv.set_bn_fold(fold0)
        conv.set_mode(None)
