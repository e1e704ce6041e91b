"""NHWC bf16 implicit-GEMM convolution kernels (csrc/ops/conv_kernels.hip) vs fp32 PyTorch.

GPU: forward, backward-data (flipped weight) and backward-weight (split-K slabs) of every tile
variant on shapes with padding, stride 2, 1x1/3x3 taps and output-pixel counts that are not a
multiple of the tile (tail rows); the autotuned ``Conv2dNHWC`` module under bf16 autocast; a
ResNet training step with the kernels equal to the MIOpen one. CPU: the module is nn.Conv2d.
"""
import pytest
import torch
import torch.nn.functional as F

from arena_amd.ops import conv

SHAPES = [  # n, cin, h, w, cout, k, stride
    (2, 64, 9, 11, 64, 3, 1),
    (3, 128, 7, 7, 128, 1, 1),
    (2, 64, 10, 10, 128, 3, 2),
    (1, 128, 15, 13, 64, 1, 2),
    (2, 192, 6, 5, 256, 3, 1),
    (8, 64, 28, 28, 64, 3, 1),   # 98 pixel steps: the split reduce's unrolled path, 49 BN tiles
    (8, 64, 28, 28, 64, 1, 1),   # 98 splits of a 64x64 weight: the 8 x 32 split-reduce shape
]


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def _data(n, cin, h, w, cout, k, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(n, cin, h, w, device=dev, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wt = (torch.randn(cout, cin, k, k, device=dev, generator=g) * 0.1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    return x, wt


def test_conv2d_nhwc_module_is_nn_conv2d_on_cpu():
    torch.manual_seed(0)
    m = conv.Conv2dNHWC(8, 16, 3, stride=2, padding=1, bias=False)
    ref = torch.nn.Conv2d(8, 16, 3, stride=2, padding=1, bias=False)
    ref.weight.data.copy_(m.weight.data)
    x = torch.randn(2, 8, 9, 9, requires_grad=True)
    x2 = x.detach().clone().requires_grad_()
    y, y2 = m(x), ref(x2)
    torch.testing.assert_close(y, y2)
    y.sum().backward()
    y2.sum().backward()
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad)
    with pytest.raises(ValueError):
        conv.Conv2dNHWC(8, 16, 3, bias=True)


def test_pick_variant_fills_the_chip():
    assert conv.pick_variant(128 * 56 * 56, 256) == 0
    assert conv.pick_variant(128 * 7 * 7, 512) in (2, 3)   # 49 m-tiles: smaller tiles
    assert conv.pick_variant(1000, 64) in (1, 3)           # Cout 64 needs a 64-wide tile


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_bwd_wgrad_match_fp32(shape):
    from arena_amd.ops import _ext
    _ext.load()
    n, cin, h, w, cout, k, st = shape
    pad = k // 2
    x, wt = _data(n, cin, h, w, cout, k, "cuda")
    ref = F.conv2d(x.float(), wt.float(), stride=st, padding=pad)
    for v in conv.variants_for(cout):
        y = conv.conv2d_fwd(x, wt, st, pad, v)
        assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
        assert _rel(y, ref) < 1e-2, (v, _rel(y, ref))
    dy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dx_ref, dw_ref, _ = torch.ops.aten.convolution_backward(
        dy.float(), x.float(), wt.float(), None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
        [True, True, False])
    if st == 1:
        # the flip/transpose kernel is an exact permutation of the torch ops
        ref_flip = wt.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        wf = conv.flip_weight(wt)
        assert wf.shape == ref_flip.shape and torch.equal(wf, ref_flip)
        assert wf.is_contiguous(memory_format=torch.channels_last)
        addend = torch.randn(x.shape, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        for v in conv.variants_for(cin):
            dx = conv.conv2d_bwd_data(dy, wt, pad, v)
            assert dx.shape == x.shape
            assert _rel(dx, dx_ref) < 1e-2, (v, _rel(dx, dx_ref))
            # epilogue addend (the residual-gradient join): fp32 sum rounded once
            dxa = conv.conv2d_bwd_data(dy, wt, pad, v, addend=addend)
            assert _rel(dxa, dx_ref + addend.float()) < 1e-2, (v, _rel(dxa, dx_ref + addend.float()))
    for v in conv.wgrad_variants_for(cin, cout):
        for sp in (1, 3, 17, 0):
            dw = conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, sp, out_dtype=torch.float32)
            assert dw.shape == wt.shape
            assert _rel(dw, dw_ref) < 5e-3, (v, sp, _rel(dw, dw_ref))
            # fixed-order slab reduction: bit-reproducible
            dw2 = conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, sp, out_dtype=torch.float32)
            assert torch.equal(dw, dw2)
        dwb = conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, 0)
        assert dwb.dtype == torch.bfloat16 and dwb.is_contiguous(memory_format=torch.channels_last)


V2_SHAPES = [  # n, cin, h, w, cout, k, stride
    (2, 64, 9, 11, 64, 3, 1),       # M = 198 < one 256-row tile
    (3, 128, 7, 7, 128, 1, 1),
    (2, 64, 10, 10, 128, 3, 2),
    (2, 192, 6, 5, 256, 3, 1),
    (8, 64, 28, 28, 64, 3, 1),      # 6272 rows: tail tile of 128 rows
    (2, 256, 14, 14, 512, 1, 1),    # BN = 256 tiles, two row bands in the 256x256 epilogue
    (2, 64, 56, 56, 128, 3, 1),     # halo window of 242 rows
    (4, 128, 7, 7, 128, 3, 1),      # halo windows spanning several images
    (1, 64, 5, 63, 64, 3, 1),       # the widest halo image
    (2, 128, 9, 31, 128, 3, 1),     # the small window's widest image (V2+14 at its limit)
    (1, 128, 5, 63, 128, 3, 1),     # the big window at W = 63 with the 128-wide tile (V2+12)
    (2, 320, 7, 9, 128, 3, 1),      # five channel chunks: the ring and the double window wrap
]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", V2_SHAPES)
def test_conv_v2_matches_fp32(shape):
    """v2 tile kernel (32x32x16 MFMA, LDS epilogue): forward, stride-1 backward-data with the
    residual-join addend (dense and bit-masked), against fp32 F.conv2d; its BatchNorm statistics
    (per-tile partials and acc-mode sums) against the BN layer's own statistics pass."""
    from arena_amd.ops import _ext
    from arena_amd.ops.batchnorm import BatchNormAct2d
    _ext.load()
    n, cin, h, w, cout, k, st = shape
    pad = k // 2
    x, wt = _data(n, cin, h, w, cout, k, "cuda", seed=5)
    ref = F.conv2d(x.float(), wt.float(), stride=st, padding=pad)
    halo = conv.halo_variants_for(cout, (k, k), st, pad, w, cin)
    assert bool(halo) == (k == 3 and st == 1)
    vs = conv.v2_variants_for(cout) + halo
    assert vs
    for v in vs:
        y = conv.conv2d_fwd(x, wt, st, pad, v)
        assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
        assert _rel(y, ref) < 1e-2, (v, _rel(y, ref))
        y1 = conv.conv2d_fwd(x, wt, st, pad, 0 if cout % 128 == 0 else 1)
        # same products, same K order per output: equal to v1 to rounding (fp32 sum order of
        # the MFMA shapes differs)
        assert _rel(y, y1) < 1e-2
        yp, (part, rpb) = conv.conv2d_fwd(x, wt, st, pad, v, with_stats=True)
        assert torch.equal(yp, y) and rpb == conv.TILES[v][0]
        m = y.shape[0] * y.shape[2] * y.shape[3]
        assert part.numel() == -(-m // rpb) * 2 * cout
        yf, fin = conv.conv2d_fwd(x, wt, st, pad, v, with_stats=True, final=True)
        assert torch.equal(yf, y)
        for stats in ((part, rpb), fin):
            bns = [BatchNormAct2d(cout).cuda() for _ in range(2)]
            for b in bns:
                b.weight.data.uniform_(0.5, 1.5)
                b.bias.data.uniform_(-0.5, 0.5)
            bns[1].load_state_dict(bns[0].state_dict())
            out_ref = bns[0](y)
            out = bns[1](y, stats=stats)
            assert _rel(out, out_ref) < 1e-2, v
            torch.testing.assert_close(bns[1].running_mean, bns[0].running_mean, rtol=1e-4,
                                       atol=1e-5)
            torch.testing.assert_close(bns[1].running_var, bns[0].running_var, rtol=1e-3,
                                       atol=1e-5)
    if st != 1:
        return
    dy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dx_ref, _, _ = torch.ops.aten.convolution_backward(
        dy.float(), x.float(), wt.float(), None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1,
        [True, False, False])
    addend = torch.randn(x.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    bits = torch.randint(0, 256, (addend.numel() // 8,), device="cuda", dtype=torch.uint8)
    dense = conv.MaskedGrad(addend, bits).materialize()
    for v in conv.v2_variants_for(cin) + conv.halo_variants_for(cin, (k, k), 1, pad, w, cout):
        dx = conv.conv2d_bwd_data(dy, wt, pad, v)
        assert _rel(dx, dx_ref) < 1e-2, (v, _rel(dx, dx_ref))
        dxa = conv.conv2d_bwd_data(dy, wt, pad, v, addend=addend)
        assert _rel(dxa, dx_ref + addend.float()) < 1e-2, v
        a = conv.conv2d_bwd_data(dy, wt, pad, v, addend=addend, addmask=bits)
        b = conv.conv2d_bwd_data(dy, wt, pad, v, addend=dense)
        assert torch.equal(a, b), v
    # the linked (BN-backward partials) form at these shapes -- incl. the halo windows at their
    # widest images -- against fp32 sums of the stored dX
    bnx = torch.randn(x.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    m = x.shape[0] * x.shape[2] * x.shape[3]
    mean = torch.randn(cin, device="cuda") * 0.3
    xc = bnx.permute(0, 2, 3, 1).reshape(m, cin).float() - mean
    for v in conv.v2_variants_for(cin) + conv.halo_variants_for(cin, (k, k), 1, pad, w, cout):
        dx0 = conv.conv2d_bwd_data(dy, wt, pad, v)
        dx, (part, rpb) = conv.conv2d_bwd_data(dy, wt, pad, v, bn=(bnx, bits, mean))
        assert torch.equal(dx, dx0), v
        assert _rel(dx, dx_ref) < 1e-2, (v, _rel(dx, dx_ref))
        g = dx.permute(0, 2, 3, 1).reshape(m, cin).float() * \
            conv._unpack_bits(bits, dx).permute(0, 2, 3, 1).reshape(m, cin).float()
        p = part.view(-1, 2, cin)
        torch.testing.assert_close(p[:, 0].sum(0), g.sum(0), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(p[:, 1].sum(0), (g * xc).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(3, 128, 7, 7, 128, 1, 1), (2, 256, 7, 7, 256, 3, 1),
                                   (4, 128, 14, 14, 256, 3, 2), (2, 256, 9, 9, 512, 1, 1),
                                   (3, 256, 5, 7, 128, 3, 1)])
def test_conv_wgrad_v2_matches_fp32(shape):
    """v2 weight-gradient kernel (32x32x16 MFMA, transposed fragment reads of the granule-permuted
    pixel-major images): fp32-close to torch, bit-reproducible, every split count."""
    from arena_amd.ops import _ext
    _ext.load()
    n, cin, h, w, cout, k, st = shape
    pad = k // 2
    x, wt = _data(n, cin, h, w, cout, k, "cuda", seed=11)
    ho, wo = conv.out_hw(h, w, k, k, st, pad)
    dy = torch.randn(n, cout, ho, wo, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    _, dw_ref, _ = torch.ops.aten.convolution_backward(
        dy.float(), x.float(), wt.float(), None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
        [False, True, False])
    vs = [v for v in conv.wgrad_variants_for(cin, cout) if v in conv.WGRAD_V2]
    assert vs
    for v in vs:
        for sp in (1, 2, 5, 0):
            dw = conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, sp, out_dtype=torch.float32)
            assert _rel(dw, dw_ref) < 5e-3, (v, sp, _rel(dw, dw_ref))
            assert torch.equal(dw, conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, sp,
                                                     out_dtype=torch.float32))
        dwb = conv.conv2d_wgrad(x, dy, (k, k), st, pad, v, 0)
        assert dwb.dtype == torch.bfloat16 and _rel(dwb, dw_ref) < 1e-2


def test_v2_variants_are_forward_and_dgrad_only():
    assert set(conv.v2_variants_for(64)) == {conv.V2 + v for v in (3, 5, 6, 9, 11)}
    assert set(conv.v2_variants_for(256)) == set(conv.V2_TILES) - set(conv.V2_HALO)
    assert set(conv.halo_variants_for(256, (3, 3), 1, 1, 14)) == set(conv.V2_HALO)
    # no small window at 56 wide
    assert conv.halo_variants_for(64, (3, 3), 1, 1, 56) == [conv.V2 + 13, conv.V2 + 18]
    # the two-group forms need an even number of 64-channel chunks
    assert not set(conv.halo_variants_for(256, (3, 3), 1, 1, 14, 192)) & conv.HALO_SPLIT2
    assert conv.HALO_SPLIT2 <= set(conv.halo_variants_for(256, (3, 3), 1, 1, 14, 256))
    assert conv.V2 + 14 in conv.halo_variants_for(64, (3, 3), 1, 1, 31)
    assert conv.V2 + 14 not in conv.halo_variants_for(64, (3, 3), 1, 1, 32)
    assert not conv.halo_variants_for(256, (3, 3), 2, 1, 14)
    assert not conv.halo_variants_for(256, (3, 3), 1, 1, 64)
    assert not conv.halo_variants_for(256, (1, 1), 1, 0, 14)
    assert conv.HALO_WIDE <= set(conv.halo_variants_for(256, (3, 3), 1, 1, 14))
    conv.set_halo_wide(False)
    try:
        assert not set(conv.halo_variants_for(256, (3, 3), 1, 1, 14)) & conv.HALO_WIDE
    finally:
        conv.set_halo_wide(True)
    assert not set(conv.variants_for(256)) & set(conv.V2_TILES)   # disjoint code ranges
    # v2 weight gradients need >= 128-channel tiles on both sides
    assert not set(conv.wgrad_variants_for(64, 256)) & set(conv.WGRAD_V2)
    assert set(conv.wgrad_variants_for(256, 256)) >= set(conv.WGRAD_V2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 256, 7, 7, 128, 3, 1), (3, 128, 6, 5, 256, 1, 1),
                                   (2, 64, 9, 11, 64, 3, 1), (4, 128, 7, 7, 128, 3, 2)])
def test_conv_split_k_matches_unsplit(shape):
    """Split-K variants (in-kernel ticket reduction): fp32-close to the reference, bit-identical
    run to run (slices summed in slice order whichever block arrives last), the same BatchNorm
    partials / finished statistics and epilogue addend as the unsplit kernel."""
    from arena_amd.ops.batchnorm import BatchNormAct2d
    n, cin, h, w, cout, k, st = shape
    pad = k // 2
    x, wt = _data(n, cin, h, w, cout, k, "cuda", seed=5)
    ref = F.conv2d(x.float(), wt.float(), stride=st, padding=pad)
    steps = cin * k * k // 64
    for v in conv.variants_for(cout):
        for ks in [s for s in conv.KSPLITS if s <= steps][:3]:
            kv = conv.kvariant(v, ks)
            assert conv.split_of(kv) == ks and conv.TILES[kv] == conv.TILES[v]
            y = conv.conv2d_fwd(x, wt, st, pad, kv)
            assert _rel(y, ref) < 1e-2, (v, ks, _rel(y, ref))
            for _ in range(2):
                assert torch.equal(conv.conv2d_fwd(x, wt, st, pad, kv), y)
            # statistics epilogue on the summed tile: partials and finished (acc) statistics
            y2, stats = conv.conv2d_fwd(x, wt, st, pad, kv, with_stats=True)
            assert torch.equal(y2, y)
            y3, fin = conv.conv2d_fwd(x, wt, st, pad, kv, with_stats=True, final=True)
            assert torch.equal(y3, y)
            bns = [BatchNormAct2d(cout).cuda() for _ in range(3)]
            r = bns[0](y)
            assert _rel(bns[1](y, stats=stats), r) < 1e-2
            assert _rel(bns[2](y, stats=fin), r) < 1e-2
            torch.testing.assert_close(bns[2].running_var, bns[0].running_var, rtol=1e-3,
                                       atol=1e-5)
    if st == 1:
        dy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dx_ref = torch.ops.aten.convolution_backward(
            dy.float(), x.float(), wt.float(), None, [1, 1], [pad, pad], [1, 1], False, [0, 0], 1,
            [True, False, False])[0]
        addend = torch.randn(x.shape, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        for v in conv.variants_for(cin):
            kv = conv.kvariant(v, 2)
            dxa = conv.conv2d_bwd_data(dy, wt, pad, kv, addend=addend)
            assert _rel(dxa, dx_ref + addend.float()) < 1e-2, (v, _rel(dxa, dx_ref + addend.float()))


def test_wgrad_candidates_aim_at_blocks_per_cu():
    # 3x3 512 -> 512 (K = 4608): every candidate's grid (tiles x splits) reaches its target
    cands = conv._wgrad_candidates(512, 512, (3, 3))
    assert cands == sorted(set(cands)) and cands
    for v, splits in cands:
        bm, bn = conv.WGRAD_TILES[v]
        tiles = (512 // bm) * (9 * 512 // bn)
        assert any(tiles * splits >= b * conv._CUS and tiles * (splits - 1) < b * conv._CUS
                   for b in conv._WGRAD_BPC)


def test_split_variants_for_only_underfilled_grids():
    # 56x56 at batch 128: thousands of tiles, no split; 7x7 x 512 with K = 4608: splits offered
    assert conv.split_variants_for(128 * 56 * 56, 64, 576) == []
    sv = conv.split_variants_for(128 * 7 * 7, 512, 4608)
    assert sv and all(conv.split_of(v) > 1 and v % 16 in conv.variants_for(512) for v in sv)
    # every slice keeps at least 4 K steps
    assert all(4608 // 64 // conv.split_of(v) >= 4 for v in sv)
    assert conv.split_variants_for(128 * 7 * 7, 512, 256) == []


@pytest.mark.gpu
def test_conv_kernel_rejects_bad_shapes():
    from arena_amd.ops import _ext
    x, wt = _data(1, 32, 8, 8, 64, 3, "cuda")
    with pytest.raises(RuntimeError, match="multiples of 64"):
        _ext.load().conv_fwd(x, wt, 1, 1, 1, False)
    x, wt = _data(1, 64, 8, 8, 64, 3, "cuda")
    with pytest.raises(RuntimeError, match="Cout % 128"):
        _ext.load().conv_fwd(x, wt, 1, 1, 0, False)
    # pad > R-1 would need a negative backward-data padding: not a kernel shape (MIOpen runs it)
    x, wt = _data(2, 64, 8, 8, 128, 1, "cuda")
    assert conv.kernel_ok(x, wt, 1, 0) and not conv.kernel_ok(x, wt, 1, 1)
    x3, w3 = _data(2, 64, 8, 8, 128, 3, "cuda")
    assert conv.kernel_ok(x3, w3, 1, 2) and not conv.kernel_ok(x3, w3, 1, 3)


@pytest.mark.gpu
def test_conv_module_oversized_padding_falls_back(monkeypatch):
    """A 1x1 conv with padding=1 is a legal nn.Conv2d: it trains (through MIOpen) instead of
    failing in the kernel's autotuning or backward."""
    monkeypatch.setenv("ARENA_CONV", "auto")
    torch.manual_seed(0)
    m = conv.Conv2dNHWC(64, 128, 1, stride=1, padding=1, bias=False).cuda().to(
        memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(64, 128, 1, stride=1, padding=1, bias=False).cuda()
    ref.weight.data.copy_(m.weight.data)
    x = torch.randn(2, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    xr = x.detach().clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
        yr = ref(xr)
    assert y.shape == (2, 128, 10, 10)
    y.float().square().sum().backward()
    yr.float().square().sum().backward()
    assert _rel(y, yr) < 2e-2 and _rel(x.grad, xr.grad) < 2e-2
    assert _rel(m.weight.grad, ref.weight.grad) < 2e-2


@pytest.mark.gpu
def test_async_wgrad_with_fp32_weights_under_autocast(monkeypatch):
    """with fp32 parameters under bf16 autocast the cast's backward reads dW on the main
    stream, and a second backward accumulates into .grad: async wgrad must give exactly the
    gradients of the synchronous path (it falls back to the main stream there)."""
    from arena_amd.models import resnet as R
    monkeypatch.setenv("ARENA_CONV", "ours")
    torch.manual_seed(0)
    net = R.resnet("resnet_tiny", num_classes=10).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    grads = {}
    try:
        for mode in (False, True):
            conv.set_async_wgrad(mode)
            net.zero_grad(set_to_none=True)
            for _ in range(2):        # the second pass accumulates into existing .grad
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = net(x)
                out.float().square().mean().backward()
            conv.sync_wgrad()
            torch.cuda.synchronize()
            grads[mode] = {n: p.grad.clone() for n, p in net.named_parameters()}
    finally:
        conv.set_async_wgrad(False)
    for n, g in grads[False].items():
        assert torch.equal(grads[True][n], g), n


@pytest.mark.gpu
def test_weight_flipper_keeps_buffers_for_captured_graphs():
    """a key change (weights re-bound, train/eval toggled) must not free the flip
    buffers a captured graph still uses: same-shape buffers are reused in place and the rest are
    retired, not released."""
    from arena_amd.models import resnet as R
    conv.set_mode("ours")
    try:
        torch.manual_seed(0)
        net = R.resnet("resnet_tiny", num_classes=10).cuda().to(memory_format=torch.channels_last)
        for m in net.modules():
            if isinstance(m, torch.nn.Conv2d):
                m.weight.data = m.weight.data.to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
        fl = net._flipper
        with torch.enable_grad():
            assert fl._prepare() is not None
        before = [d.data_ptr() for d in fl._dst]
        assert before
        first = fl.convs[0]
        first.weight.data = first.weight.data.clone()      # re-bound: the key changes
        with torch.enable_grad():
            flips = fl._prepare()
        after = [d.data_ptr() for d in fl._dst]
        assert sorted(after) == sorted(before)              # same buffers, no new allocation
        assert flips[first.weight.data_ptr()].data_ptr() in before
        first.train(False)                                   # fewer convs: one buffer retired
        with torch.enable_grad():
            fl._prepare()
        live = {d.data_ptr() for d in fl._dst} | {d.data_ptr() for d in fl._retired}
        assert set(before) <= live
    finally:
        conv.set_mode(None)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["auto", "ours"])
def test_conv2d_nhwc_module_autocast(mode, monkeypatch):
    monkeypatch.setenv("ARENA_CONV", mode)
    torch.manual_seed(0)
    m = conv.Conv2dNHWC(64, 128, 3, stride=1, padding=1, bias=False).cuda().to(
        memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(64, 128, 3, stride=1, padding=1, bias=False).cuda()
    ref.weight.data.copy_(m.weight.data)
    x = torch.randn(4, 64, 14, 14, device="cuda").contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    xr = x.detach().clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    assert y.dtype == torch.bfloat16
    yr = ref(xr)
    assert _rel(y, yr) < 1e-2
    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16))
    yr.backward(gy)
    assert m.weight.grad.dtype == torch.float32
    assert _rel(m.weight.grad, ref.weight.grad) < 2e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    if mode == "ours":
        plan = conv.plan_for(x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last),
                             m.weight.to(torch.bfloat16).contiguous(
                                 memory_format=torch.channels_last), 1, 1)
        assert plan.fwd != conv.MIOPEN and plan.bwd != conv.MIOPEN and plan.wgrad != conv.MIOPEN


@pytest.mark.gpu
def test_resnet_step_kernels_match_miopen(monkeypatch):
    """One bf16 training step of a small ResNet with the MFMA conv kernels is as close to fp32
    math as the same step on MIOpen: each mode's gradients are measured against an fp32 run of the
    same weights/inputs (bf16-vs-bf16 comparisons are dominated by rounding noise that max-pool
    ties and BN cancellations amplify, so they cannot tell a bug from noise)."""
    from arena_amd.models.resnet import ResNet

    def run(mode, bf16):
        monkeypatch.setenv("ARENA_CONV", mode)
        torch.manual_seed(0)
        model = ResNet([1, 1], num_classes=10, width=64).cuda().to(
            memory_format=torch.channels_last)
        x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
        y = torch.arange(8, device="cuda") % 10
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        return loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters()}

    ref_loss, ref = run("off", False)
    err = {}
    for mode in ("miopen", "ours"):
        loss, grads = run(mode, True)
        assert abs(loss - ref_loss) < 2e-2, (mode, loss, ref_loss)
        err[mode] = {n: _rel(g, ref[n]) for n, g in grads.items()}
    for n, e in err["ours"].items():
        assert e < max(1.5 * err["miopen"][n], 0.05), (n, e, err["miopen"][n])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES[:4] + SHAPES[-1:])
def test_conv_fused_bn_statistics(shape):
    """The conv epilogue's BatchNorm partials give the same BN output, batch statistics and
    running statistics as the BN's own statistics pass (tail tiles included)."""
    from arena_amd.ops import _ext
    from arena_amd.ops.batchnorm import BatchNormAct2d
    n, cin, h, w, cout, k, st = shape
    pad = k // 2
    x, wt = _data(n, cin, h, w, cout, k, "cuda", seed=3)
    for v, one_pass in [(v, p) for v in conv.variants_for(cout) for p in (False, True)]:
        # one_pass: sums and sums of squares in one exchange (ConvArgs::st1p)
        _ext.load().conv_set_stats_one_pass(one_pass)
        y0 = conv.conv2d_fwd(x, wt, st, pad, v)
        y, stats = conv.conv2d_fwd(x, wt, st, pad, v, with_stats=True)
        assert torch.equal(y, y0)
        part, rpb = stats
        m = y.shape[0] * y.shape[2] * y.shape[3]
        assert rpb == conv.TILES[v][0] and part.numel() == -(-m // rpb) * 2 * cout
        bns = [BatchNormAct2d(cout).cuda() for _ in range(2)]
        for b in bns:
            b.weight.data.uniform_(0.5, 1.5)
            b.bias.data.uniform_(-0.5, 0.5)
        bns[1].load_state_dict(bns[0].state_dict())
        ref = bns[0](y)
        out = bns[1](y, stats=stats)
        assert _rel(out, ref) < 1e-2
        torch.testing.assert_close(bns[1].running_mean, bns[0].running_mean, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(bns[1].running_var, bns[0].running_var, rtol=1e-3, atol=1e-5)
        assert int(bns[1].num_batches_tracked) == 1
    _ext.load().conv_set_stats_one_pass(False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["ours", "miopen"])
def test_grad_join_matches_autograd_sum(mode, monkeypatch):
    """The block-input gradient summed through GradJoin (first consumer parks, second fuses) equals
    autograd's own summation, for an identity block and a downsample block."""
    from arena_amd.models import resnet as R
    conv.set_mode(mode)
    # MIOpen's default solvers for some of these shapes accumulate split results in a run-order
    # dependent way (run-to-run spread up to ~10 % max-relative on the block-input gradient):
    # ask for its deterministic solvers so the comparison is about the join
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)

    class NoJoin(conv.GradJoin):
        def register(self, takes_masked=False):
            return self   # never reaches two consumers: both behave as plain autograd

    try:
        for cin, mid, stride in ((256, 64, 1), (128, 64, 2)):
            torch.manual_seed(0)
            blk = R.Bottleneck(cin, mid, stride).cuda().to(memory_format=torch.channels_last)
            with torch.no_grad():
                blk.bn3.weight.uniform_(0.5, 1.5)   # zero-init would hide the main branch
            x0 = torch.randn(4, cin, 14, 14, device="cuda").to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            g = torch.randn(4, mid * 4, 14 // stride, 14 // stride, device="cuda").to(
                torch.bfloat16).contiguous(memory_format=torch.channels_last)
            out = {}
            for name, cls in (("join", conv.GradJoin), ("plain", NoJoin), ("plain2", NoJoin)):
                monkeypatch.setattr(R, "GradJoin", cls)
                blk.zero_grad(set_to_none=True)
                x = x0.clone().requires_grad_(True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    y = blk(x)
                y.backward(g)
                out[name] = (x.grad.float(), {n: p.grad.float().clone()
                                              for n, p in blk.named_parameters()})
            # MIOpen's backward-data is not run-to-run reproducible for some shapes (split
            # accumulation): measure its own spread and allow that much
            spread = _rel(out["plain2"][0], out["plain"][0])
            assert _rel(out["join"][0], out["plain"][0]) < max(2e-2, 2 * spread), (cin, stride,
                                                                                  spread)
            # parameter gradients do not depend on the join: identical with the (deterministic)
            # kernels, within MIOpen's run-to-run spread otherwise
            ptol = 1e-6 if mode == "ours" else 2e-2
            for n, gp in out["plain"][1].items():
                assert _rel(out["join"][1][n], gp) < ptol, n
    finally:
        conv.set_mode(None)


@pytest.mark.gpu
def test_dgrad_epilogue_bn_backward_partials():
    """conv2d_bwd_data(..., bn=(x, mask, mean)): per-tile sum g and sum g (x - mean) of the
    stored dX (g = dX * mask bit), the bn_bwd_reduce partial format, tail tile included, on every
    v1 and v2 tile, with and without an addend."""
    n, cin, h, w, cout, k = 3, 256, 9, 11, 64, 3   # 256 dX channels: every halo tile width
    x, wt = _data(n, cin, h, w, cout, k, "cuda", seed=5)
    dy = torch.randn(n, cout, h, w, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    bnx = torch.randn(n, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    m = n * h * w
    mask = torch.randint(0, 256, (m * cin // 8,), device="cuda", dtype=torch.uint8)
    mean = torch.randn(cin, device="cuda") * 0.3
    bits = ((mask.view(m, cin // 8, 1).int() >> torch.arange(8, device="cuda").view(1, 1, 8)) & 1)
    bits = bits.view(m, cin).float()
    addend = torch.randn(n, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    vs2 = conv.v2_variants_for(cin) + conv.halo_variants_for(cin, (k, k), 1, 1, w, cout)
    assert vs2 and set(conv.V2_HALO) - conv.HALO_SPLIT2 <= set(vs2)
    xc = bnx.permute(0, 2, 3, 1).reshape(m, cin).float() - mean
    for v in conv.variants_for(cin) + vs2:   # v1 tiles and the v2 coalesced-epilogue form
        dx0 = conv.conv2d_bwd_data(dy, wt, 1, v)
        dx, (part, rpb) = conv.conv2d_bwd_data(dy, wt, 1, v, bn=(bnx, mask, mean))
        assert torch.equal(dx, dx0), v
        assert rpb == conv.TILES[v][0]
        for add in (None, addend):   # with an addend, g is the stored dX + addend
            if add is not None:
                dx, (part, rpb) = conv.conv2d_bwd_data(dy, wt, 1, v, addend=add,
                                                       bn=(bnx, mask, mean))
                assert torch.equal(dx, conv.conv2d_bwd_data(dy, wt, 1, v, addend=add)), v
            g = dx.permute(0, 2, 3, 1).reshape(m, cin).float() * bits
            nt = -(-m // rpb)
            assert part.numel() == nt * 2 * cin
            p = part.view(nt, 2, cin)
            for t in range(nt):
                sl = slice(t * rpb, min(m, (t + 1) * rpb))
                torch.testing.assert_close(p[t, 0], g[sl].sum(0), rtol=1e-4, atol=1e-3)
                torch.testing.assert_close(p[t, 1], (g[sl] * xc[sl]).sum(0), rtol=1e-4,
                                           atol=1e-3)
        # acc form: the same sums added into an fp64 [rep, 2, C] set (twice: it accumulates)
        from arena_amd.ops.batchnorm import acc_rep, acc_totals
        acc_set = torch.zeros(acc_rep() * 2 * cin, dtype=torch.float64, device="cuda")
        for rep_ in range(2):
            dxs, none = conv.conv2d_bwd_data(dy, wt, 1, v, bn=(bnx, mask, mean), bn_acc=acc_set)
            assert none is None and torch.equal(dxs, dx0), v
        acc = acc_totals(acc_set.view(-1, 2, cin)).reshape(-1)
        g0 = dx0.permute(0, 2, 3, 1).reshape(m, cin).float() * bits
        torch.testing.assert_close(acc[:cin].float(), 2 * g0.sum(0), rtol=1e-4, atol=2e-3)
        torch.testing.assert_close(acc[cin:].float(), 2 * (g0 * xc).sum(0), rtol=1e-4, atol=2e-3)
        # no ReLU: every bit set
        _, (part1, _) = conv.conv2d_bwd_data(dy, wt, 1, v, bn=(bnx, None, mean))
        torch.testing.assert_close(part1.view(nt, 2, cin)[:, 0].sum(0),
                                   dx0.permute(0, 2, 3, 1).reshape(m, cin).float().sum(0),
                                   rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["partials", "acc"])
def test_bn_grad_links_match_plain_backward(monkeypatch, form):
    """Two ResNet blocks with the BN backward partials computed in the convs' backward-data
    epilogues (BNGradLink) give the gradients of the plain BN reduction path -- as per-tile
    partials (BN finalize + dx) and as fp64 sums in the BN's own set (dx only)."""
    from arena_amd.models import resnet as R
    conv.set_mode("ours")
    links0, pairs0 = conv._BN_LINKS, conv._LINK_ACC_MAX_PAIRS
    conv.set_bn_links(True)
    conv.set_link_acc_max_pairs(1 << 30 if form == "acc" else 0)

    class NoLink(conv.BNGradLink):
        def set_bn(self, *a, **k):
            pass   # never ready: every BN runs its own reduction

    class Counting(conv.BNGradLink):
        hits = 0
        kinds = set()

        def take(self, dy):
            r = super().take(dy)
            Counting.hits += r is not None
            if r is not None:
                Counting.kinds.add("acc" if isinstance(r[0], str) else "partials")
            return r

    try:
        torch.manual_seed(0)
        # channel counts the kernels take (multiples of 64)
        net = torch.nn.ModuleList([R.Bottleneck(256, 64, 1), R.Bottleneck(256, 64, 1)]).cuda()
        net = net.to(memory_format=torch.channels_last)
        with torch.no_grad():
            for b in net:
                b.bn3.weight.uniform_(0.5, 1.5)
        x0 = torch.randn(4, 256, 12, 12, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        g = torch.randn(4, 256, 12, 12, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        out = {}
        for name, cls in (("link", Counting), ("plain", NoLink)):
            monkeypatch.setattr(R, "BNGradLink", cls)
            net.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                link = cls()
                y = net[0](x, link_out=link)
                y = net[1](y, link=link)
            y.backward(g)
            out[name] = (x.grad.float(), {n: p.grad.float().clone()
                                          for n, p in net.named_parameters()})
        # bn1, bn2 of both blocks and block 0's bn3 (joined through block 1's conv1)
        assert Counting.hits == 5, Counting.hits
        assert Counting.kinds == {form}, Counting.kinds
        assert _rel(out["link"][0], out["plain"][0]) < 2e-2
        for n, gp in out["plain"][1].items():
            assert _rel(out["link"][1][n], gp) < 2e-2, n
    finally:
        conv.set_mode(None)
        conv.set_bn_links(links0)
        conv.set_link_acc_max_pairs(pairs0)


@pytest.mark.gpu
@pytest.mark.parametrize("k,pad,h,st", [(3, 1, 10, 2), (1, 0, 10, 2), (3, 1, 11, 2), (1, 0, 7, 2),
                                        (1, 0, 10, 3), (2, 0, 11, 3)])
def test_strided_dgrad_phases_match_fp32(k, pad, h, st):
    """Backward-data of a strided convolution as parity-class phase convolutions (mapped kernel
    output), with and without the addend, odd sizes included; covers the three ways dX gets
    written: every phase tapped, phase (0, 0) alone (sibling fill), and a zero/addend pre-pass
    (k=2, stride 3: a phase row without taps)."""
    n, cin, cout = 2, 64, 128
    x, wt = _data(n, cin, h, h, cout, k, "cuda", seed=7)
    ref = F.conv2d(x.float(), wt.float(), stride=st, padding=pad)
    dy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dx_ref = torch.ops.aten.convolution_backward(
        dy.float(), x.float(), wt.float(), None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
        [True, False, False])[0]
    dx = conv.conv2d_bwd_data_strided(dy, wt, (h, h), st, pad)
    assert dx.shape == x.shape and dx.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dx, dx_ref) < 1e-2, _rel(dx, dx_ref)
    addend = torch.randn(x.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dxa = conv.conv2d_bwd_data_strided(dy, wt, (h, h), st, pad, addend=addend)
    assert _rel(dxa, dx_ref + addend.float()) < 1e-2
    for v in conv.variants_for(cin):   # every tile variant of the phases
        assert _rel(conv.conv2d_bwd_data_strided(dy, wt, (h, h), st, pad, v), dx_ref) < 1e-2
    vs2 = conv.v2_variants_for(cin)
    assert vs2
    for v in vs2:                      # v2 tiles: the mapped store in their plain epilogue
        assert _rel(conv.conv2d_bwd_data_strided(dy, wt, (h, h), st, pad, v), dx_ref) < 1e-2, v
        got = conv.conv2d_bwd_data_strided(dy, wt, (h, h), st, pad, v, addend=addend)
        assert _rel(got, dx_ref + addend.float()) < 1e-2, v


@pytest.mark.gpu
@pytest.mark.parametrize("k,st,pad", [(3, 2, 1), (1, 2, 0), (3, 1, 1), (5, 3, 2)])
def test_phase_weights_match_torch_slicing(k, st, pad):
    """conv_phase_weights (one launch) == W[:, :, r0::s, c0::s].flip(2, 3).transpose(0, 1) per
    phase, bit for bit."""
    _, wt = _data(1, 64, 4, 4, 128, k, "cuda", seed=3)
    got = conv._ext.load().conv_phase_weights(wt, st, pad)
    want = []
    for a in range(st):
        r0 = (a + pad) % st
        for b in range(st):
            c0 = (b + pad) % st
            if r0 < k and c0 < k:
                want.append(wt[:, :, r0::st, c0::st].flip(2, 3).transpose(0, 1))
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.shape == w.shape and g.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(g, w)


@pytest.mark.gpu
def test_stem_conv_space_to_depth_matches_fp32():
    """StemConv2d (space-to-depth 4x4 c16 kernel) forward, BN statistics epilogue and weight
    gradient against fp32 PyTorch for the 7x7/2 3-channel stem."""
    from arena_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(0)
    m = conv.StemConv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().to(
        memory_format=torch.channels_last)
    x = torch.randn(4, 3, 38, 30, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, st = m.forward_stats(x)
    wb = m.weight.detach().to(torch.bfloat16).float()
    ref = F.conv2d(x.float(), wb, stride=2, padding=3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 1e-2, _rel(y, ref)
    assert st is not None
    bns = [BatchNormAct2d(64).cuda() for _ in range(2)]
    out = bns[1](y, stats=st)
    torch.testing.assert_close(out.float(), bns[0](y.detach()).float(), rtol=2e-2, atol=2e-2)
    g = torch.randn(y.shape, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y.backward(g)
    dw_ref = torch.ops.aten.convolution_backward(
        g.float(), x.float(), wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
        [False, True, False])[1]
    assert _rel(m.weight.grad, dw_ref) < 1e-2, _rel(m.weight.grad, dw_ref)


@pytest.mark.gpu
def test_conv_flip_multi_matches_flip_weight():
    """One conv_flip_multi launch over mixed shapes (1x1, 3x3, Cout != C) writes exactly what
    flip_weight writes per tensor."""
    from arena_amd.ops import _ext
    shapes = [(64, 64, 1, 1), (128, 64, 3, 3), (64, 256, 1, 1), (256, 128, 3, 3), (512, 2048, 1, 1)]
    ws = [(torch.randn(*s, device="cuda") * 0.1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last) for s in shapes]
    dst = [torch.full((w.shape[1], w.shape[0], w.shape[2], w.shape[3]), float("nan"),
                      device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last) for w in ws]
    _ext.load().conv_flip_multi(ws, dst)
    for w, d in zip(ws, dst):
        ref = w.flip(2, 3).transpose(0, 1)
        assert torch.equal(d, ref)
        assert torch.equal(d, conv.flip_weight(w))


@pytest.mark.gpu
def test_weight_flipper_scope_matches_per_conv_flips():
    """A bf16 channels_last ResNet trained through the WeightFlipper scope (one flip launch per
    step) gives bit-identical gradients to per-conv flips, and the scope's flipped copies are the
    ones the backward-data passes use."""
    from arena_amd.models import resnet as R
    conv.set_mode("ours")
    try:
        torch.manual_seed(0)
        net = R.resnet("resnet_tiny", num_classes=10).cuda().to(memory_format=torch.channels_last)
        for m in net.modules():   # bf16 conv weights, as under MasterSGD
            if isinstance(m, torch.nn.Conv2d):
                m.weight.data = m.weight.data.to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
        x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
        used = []
        orig = conv.conv2d_bwd_data

        def spy(*a, **k):
            used.append(k.get("wflip") is not None)
            return orig(*a, **k)

        grads = {}
        for name in ("flipper", "per_conv"):
            if name == "per_conv":
                net._flipper.convs = []
            net.zero_grad(set_to_none=True)
            conv.conv2d_bwd_data = spy
            try:
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = net(x)
                out.float().square().mean().backward()
            finally:
                conv.conv2d_bwd_data = orig
            grads[name] = {n: p.grad.clone() for n, p in net.named_parameters()}
            if name == "flipper":
                assert used and all(used), used
            else:
                assert used and not any(used)
            used.clear()
        for n, g in grads["per_conv"].items():
            assert torch.equal(grads["flipper"][n], g), n
        assert conv._ACTIVE_FLIPS is None   # the scope does not leak past forward
    finally:
        conv.set_mode(None)


@pytest.mark.gpu
@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [True, False])
def test_stem_weight_kernels_match_torch(wdtype, cl):
    """The one-kernel stem weight transform equals the torch-op form (stem_weight) on the
    bf16-rounded weight, and its backward equals autograd through that form, written in the
    weight's own dtype and memory layout."""
    from arena_amd.ops import _ext
    torch.manual_seed(0)
    w = torch.randn(64, 3, 7, 7, device="cuda").to(wdtype)
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    w16 = _ext.load().stem_weight(w)
    ref = conv.stem_weight(w.to(torch.bfloat16))
    assert w16.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(w16, ref)
    g16 = torch.randn(64, 16, 4, 4, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    wr = w.detach().to(torch.bfloat16).requires_grad_(True)
    conv.stem_weight(wr).backward(g16)
    dw = _ext.load().stem_weight_grad(g16, w)
    assert dw.dtype == w.dtype and dw.stride() == w.stride()
    assert torch.equal(dw.float(), wr.grad.float())


@pytest.mark.gpu
def test_s2d_stem_fp32_input_rounds_like_the_cast():
    """s2d_stem on an fp32 batch equals s2d_stem on the same batch cast to bf16 first."""
    from arena_amd.ops import _ext
    x = torch.randn(3, 3, 22, 18, device="cuda").contiguous(memory_format=torch.channels_last)
    a = _ext.load().s2d_stem(x)
    b = _ext.load().s2d_stem(x.to(torch.bfloat16))
    assert a.dtype == torch.bfloat16 and torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("c", [1, 2, 3, 4])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_s2d_stem_layout_matches_torch(c, dtype):
    """z[n, (dy*2 + dx)*C + c, i, j] = x[n, c, 2i + dy, 2j + dx], channels 4C..15 zero; also from
    a view whose storage offset breaks the kernel's word alignment."""
    from arena_amd.ops import _ext
    base = torch.randn(2 * 10 * 14 * c + 1, device="cuda").to(dtype)
    for x in (base[:-1].view(2, 10, 14, c).permute(0, 3, 1, 2),
              base[1:].view(2, 10, 14, c).permute(0, 3, 1, 2)):
        assert x.is_contiguous(memory_format=torch.channels_last)
        z = _ext.load().s2d_stem(x)
        xb = x.to(torch.bfloat16)
        ref = torch.zeros(2, 16, 5, 7, dtype=torch.bfloat16, device="cuda")
        for dy in range(2):
            for dx in range(2):
                d = dy * 2 + dx
                ref[:, d * c:(d + 1) * c] = xb[:, :, dy::2, dx::2]
        assert torch.equal(z, ref)


@pytest.mark.gpu
def test_masked_residual_join_matches_materialized():
    """Identity blocks whose last BN parks (dy, ReLU bits) in the residual join (the conv's
    backward-data epilogue adds dy where the bit is set) give the same gradients, bit for bit,
    as the BN writing dy * mask; and the masked path is the one taken."""
    from arena_amd.models import resnet as R
    conv.set_mode("ours")
    made = []
    orig = conv.MaskedGrad.__init__

    def spy(self, g, bits):
        made.append(1)
        orig(self, g, bits)

    try:
        torch.manual_seed(0)
        net = torch.nn.ModuleList([R.Bottleneck(256, 64, 1), R.Bottleneck(256, 64, 1)]).cuda()
        net = net.to(memory_format=torch.channels_last)
        with torch.no_grad():
            for b in net:
                b.bn3.weight.uniform_(0.5, 1.5)
        x0 = torch.randn(4, 256, 12, 12, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        g = torch.randn(4, 256, 12, 12, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        out = {}
        conv.MaskedGrad.__init__ = spy
        for on in (True, False):
            conv.set_masked_join(on)
            made.clear()
            net.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = net[1](net[0](x))
            y.backward(g)
            out[on] = (x.grad.clone(), {n: p.grad.clone() for n, p in net.named_parameters()},
                       len(made))
        assert out[True][2] == 2 and out[False][2] == 0, (out[True][2], out[False][2])
        assert torch.equal(out[True][0], out[False][0])
        for n, gp in out[False][1].items():
            assert torch.equal(out[True][1][n], gp), n
    finally:
        conv.MaskedGrad.__init__ = orig
        conv.set_masked_join(True)
        conv.set_mode(None)


@pytest.mark.gpu
def test_conv_masked_addend_matches_torch():
    """conv2d_bwd_data with a bit-masked addend equals adding addend * mask."""
    torch.manual_seed(0)
    x, w = _data(2, 64, 9, 11, 128, 3, "cuda")
    dy = torch.randn(2, 128, 9, 11, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    add = torch.randn(2, 64, 9, 11, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    bits = torch.randint(0, 256, (add.numel() // 8,), device="cuda", dtype=torch.uint8)
    dense = conv.MaskedGrad(add, bits).materialize()
    for v in conv.variants_for(64):
        a = conv.conv2d_bwd_data(dy, w, 1, v, addend=add, addmask=bits)
        b = conv.conv2d_bwd_data(dy, w, 1, v, addend=dense)
        assert torch.equal(a, b), v


@pytest.mark.gpu
@pytest.mark.parametrize("cin,stride", [(128, 2), (64, 1)])
def test_residual_mask_handoff_matches_materialized(cin, stride):
    """A downsample block whose bn3 hands (dy, ReLU bits) to down_bn (ResidualMask) gives the same
    gradients, bit for bit, as bn3 writing dy * mask for down_bn; the handoff is taken. (down_bn
    reduces its own sums here in both arms: with them summed in bn3's dx pass the order differs,
    see test_residual_bn_sums_in_bn3_dx_pass.)"""
    from arena_amd.models import resnet as R
    from arena_amd.ops import batchnorm as B
    conv.set_mode("ours")
    B.set_res_sums(False)
    taken = []
    orig = B.ResidualMask.take

    def spy(self):
        m = orig(self)
        taken.append(m is not None)
        return m

    try:
        torch.manual_seed(0)
        blk = R.Bottleneck(cin, 64, stride).cuda().to(memory_format=torch.channels_last)
        with torch.no_grad():
            blk.bn3.weight.uniform_(0.5, 1.5)
        x0 = torch.randn(4, cin, 14, 14, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        g = torch.randn(4, 256, 14 // stride, 14 // stride, device="cuda").to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        B.ResidualMask.take = spy
        out = {}
        for on in (True, False):
            conv.set_masked_join(on)
            taken.clear()
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = blk(x)
            y.backward(g)
            out[on] = (x.grad.clone(), {n: p.grad.clone() for n, p in blk.named_parameters()},
                       list(taken))
        assert out[True][2] == [True] and out[False][2] == [False], (out[True][2], out[False][2])
        assert torch.equal(out[True][0], out[False][0])
        for n, gp in out[False][1].items():
            assert torch.equal(out[True][1][n], gp), n
    finally:
        B.ResidualMask.take = orig
        B.set_res_sums(True)
        conv.set_masked_join(True)
        conv.set_mode(None)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,stride", [(128, 2), (64, 1), (512, 2)])
def test_residual_bn_sums_in_bn3_dx_pass(cin, stride):
    """down_bn's backward sums added by bn3's dx pass (bn_bwd x2=...) instead of down_bn's own
    reduction: the path is taken, and every gradient matches the self-reducing path to bf16
    rounding (the fp32 / fp64 summation order differs)."""
    from arena_amd.models import resnet as R
    from arena_amd.ops import batchnorm as B
    conv.set_mode("ours")
    got = []
    orig = B.ResidualMask.take_sums

    def spy(self):
        s_ = orig(self)
        got.append(s_ is not None)
        return s_

    try:
        torch.manual_seed(0)
        mid = 64 if cin <= 128 else 128
        blk = R.Bottleneck(cin, mid, stride).cuda().to(memory_format=torch.channels_last)
        with torch.no_grad():
            blk.bn3.weight.uniform_(0.5, 1.5)
        x0 = torch.randn(4, cin, 14, 14, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        g = torch.randn(4, mid * 4, 14 // stride, 14 // stride, device="cuda").to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        B.ResidualMask.take_sums = spy
        out = {}
        for on in (True, False):
            B.set_res_sums(on)
            got.clear()
            blk.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = blk(x)
            y.backward(g)
            out[on] = (x.grad.float(), {n: p.grad.float() for n, p in blk.named_parameters()},
                       list(got))
        assert out[True][2] == [True] and out[False][2] == [False], (out[True][2], out[False][2])
        torch.testing.assert_close(out[True][0], out[False][0], rtol=2e-2, atol=2e-2)
        for n, gp in out[False][1].items():
            scale = max(1.0, float(gp.abs().max()))
            torch.testing.assert_close(out[True][1][n] / scale, gp / scale, rtol=2e-2,
                                       atol=2e-2, msg=n)
    finally:
        B.ResidualMask.take_sums = orig
        B.set_res_sums(True)
        conv.set_mode(None)


def test_masked_grad_materialize_and_join_registration_cpu():
    """MaskedGrad.materialize (the fallback for consumers without a masked epilogue) applies the
    NHWC bit order of the BN kernels' ReLU mask; a join offers the masked form only when its first
    registrant takes it."""
    torch.manual_seed(0)
    g = torch.randn(2, 16, 3, 5).contiguous(memory_format=torch.channels_last)
    keep = torch.rand(2, 16, 3, 5) > 0.5
    flat = keep.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.uint8)   # NHWC order, 8 per byte
    bits = (flat << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    dense = conv.MaskedGrad(g, bits).materialize()
    assert torch.equal(dense, torch.where(keep, g, torch.zeros_like(g)))
    assert dense.is_contiguous(memory_format=torch.channels_last)
    j = conv.GradJoin().register(takes_masked=True).register()
    assert j.active() and j.peer_takes_masked()
    j2 = conv.GradJoin().register(takes_masked=False).register()
    assert j2.active() and not j2.peer_takes_masked()
    assert not conv.GradJoin().register(takes_masked=True).peer_takes_masked()
