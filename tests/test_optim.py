"""MasterSGD (bf16 weights + fp32 masters, one multi-tensor kernel) vs torch.optim.SGD in fp32.

CPU: the PyTorch reference path of ``mt_sgd_master``; GPU: the HIP kernel
(``csrc/ops/mlp_kernels.hip::mt_sgd_master_kernel``)."""
import pytest
import torch

from arena_amd.ops.optim import MasterSGD, OptimizerGroup


def _params(dev):
    g = torch.Generator().manual_seed(0)
    shapes = [(64, 3, 7, 7), (256, 64, 1, 1), (64, 64, 3, 3), (1000, 2048), (8, 4)]
    ps = []
    for i, s in enumerate(shapes):
        t = torch.randn(s, generator=g) * 0.05
        if len(s) == 4 and i % 2 == 0:
            t = t.contiguous(memory_format=torch.channels_last)
        ps.append(torch.nn.Parameter(t.to(dev)))
    return ps


def _run(dev, steps=5):
    ps = _params(dev)
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = MasterSGD(ps, lr=0.1, momentum=0.9, weight_decay=4e-5)
    ropt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, weight_decay=4e-5)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        grads = [torch.randn(p.shape, generator=g) for p in ref]
        for p, r, gr in zip(ps, ref, grads):
            gb = gr.to(dev).to(torch.bfloat16)
            if p.is_contiguous(memory_format=torch.channels_last) and p.dim() == 4:
                gb = gb.contiguous(memory_format=torch.channels_last)
            p.grad = gb
            r.grad = gb.float()
        opt.step()
        ropt.step()
    for p, r, off in zip(ps, ref, opt.offsets):
        assert p.dtype == torch.bfloat16 and p.stride() == r.stride()
        m = opt.master.as_strided(p.shape, p.stride(), off)
        torch.testing.assert_close(m, r.detach(), rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(p.float(), r.detach(), rtol=1e-2, atol=1e-3)
        assert torch.equal(p, m.to(torch.bfloat16))


def test_master_sgd_matches_torch_sgd_cpu():
    _run("cpu")


def test_optimizer_group_and_checks():
    ps = _params("cpu")
    opt = OptimizerGroup(MasterSGD(ps[:2], lr=0.1), torch.optim.SGD(ps[2:], lr=0.1))
    ps[0].grad = torch.zeros(ps[0].shape, dtype=torch.bfloat16)  # contiguous vs channels_last
    with pytest.raises(RuntimeError, match="strides"):
        opt.step()
    opt.zero_grad()
    assert all(p.grad is None for p in ps)
    with pytest.raises(ValueError):
        MasterSGD([torch.nn.Parameter(torch.zeros(3))], lr=0.1)


def test_master_sgd_state_roundtrip():
    ps = _params("cpu")
    opt = MasterSGD(ps, lr=0.1, momentum=0.9)
    for p in ps:
        p.grad = torch.ones(p.shape, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last if p.dim() == 4 and p.is_contiguous(
                memory_format=torch.channels_last) else torch.contiguous_format)
    opt.step()
    st = opt.state_dict()
    ps2 = _params("cpu")
    opt2 = MasterSGD(ps2, lr=0.5)
    opt2.load_state_dict(st)
    assert opt2.lr == 0.1 and opt2.momentum == 0.9
    for a, b in zip(ps, ps2):
        assert torch.equal(a, b)
    assert torch.equal(opt2.mom, opt.mom)


def test_master_sgd_state_is_layout_independent():
    """A checkpoint saved from a channels_last (NHWC) run loads into a contiguous (NCHW) model
    with the same logical weights and momentum (advisor r1: flat memory-order state)."""
    ps = _params("cpu")                       # mixes channels_last and contiguous 4-D weights
    opt = MasterSGD(ps, lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(5)
    for p in ps:
        p.grad = torch.randn(p.shape, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last if p.dim() == 4 and p.is_contiguous(
                memory_format=torch.channels_last) else torch.contiguous_format)
    opt.step()
    st = opt.state_dict()
    assert all(t.is_contiguous() for t in st["master"] + st["momentum_buffer"])
    ps2 = [torch.nn.Parameter(p.detach().float().contiguous()) for p in _params("cpu")]
    opt2 = MasterSGD(ps2, lr=0.5)
    opt2.load_state_dict(st)
    for a, b, ma, mb in zip(ps, ps2, opt.master_params(), opt2.master_params()):
        assert b.is_contiguous()
        assert torch.equal(a, b) and torch.equal(ma, mb)
    for (pa, oa), (pb, ob) in zip(zip(ps, opt.offsets), zip(ps2, opt2.offsets)):
        ma = opt.mom.as_strided(pa.shape, pa.stride(), oa)
        mb = opt2.mom.as_strided(pb.shape, pb.stride(), ob)
        assert torch.equal(ma, mb)
    # a state for a different parameter set is refused (same total numel is not enough)
    ps3 = [torch.nn.Parameter(torch.zeros(8, 4)), torch.nn.Parameter(torch.zeros(4, 8))]
    st3 = MasterSGD(ps3, lr=0.1).state_dict()
    ps4 = [torch.nn.Parameter(torch.zeros(4, 8)), torch.nn.Parameter(torch.zeros(8, 4))]
    with pytest.raises(ValueError, match="shape"):
        MasterSGD(ps4, lr=0.1).load_state_dict(st3)
    with pytest.raises(ValueError, match="2 masters"):
        MasterSGD(ps4[:1], lr=0.1).load_state_dict(st3)


def test_master_sgd_accepts_1x1_channels_last_grad():
    """AccumulateGrad keeps a gradient whose strides differ only on size-1 dims: for a 1x1 conv
    weight a channels_last gradient has the same memory order as a contiguous parameter."""
    p = torch.nn.Parameter(torch.randn(16, 8, 1, 1))
    ref = torch.nn.Parameter(p.detach().clone())
    opt = MasterSGD([p], lr=0.1, momentum=0.9)
    g = torch.empty_strided((16, 8, 1, 1), (8, 1, 8, 8), dtype=torch.bfloat16)  # channels_last
    g.copy_(torch.randn(16, 8, 1, 1))
    assert g.stride() != p.stride()
    p.grad = g
    opt.step()
    ref.grad = g.float()
    torch.optim.SGD([ref], lr=0.1, momentum=0.9).step()
    torch.testing.assert_close(opt.master_params()[0], ref.detach())


def test_master_sgd_sync_from_params_after_model_load():
    """model.load_state_dict after the optimizer exists: sync_from_params makes the next step
    start from the loaded weights instead of the stale masters."""
    model = torch.nn.Linear(8, 4, bias=False)
    opt = MasterSGD(model.parameters(), lr=0.1)
    new = {"weight": torch.full((4, 8), 0.5)}
    model.load_state_dict(new)
    opt.sync_from_params()
    model.weight.grad = torch.ones(4, 8, dtype=torch.bfloat16)
    opt.step()
    torch.testing.assert_close(model.weight.float(), torch.full((4, 8), 0.4), rtol=0, atol=2e-3)
    # re-binding the parameter's data: sync adopts it as a view of the flat buffer again
    model.weight.data = torch.full((4, 8), 0.25, dtype=torch.bfloat16)
    opt.sync_from_params()
    assert model.weight.data_ptr() == opt.wbf.data_ptr()
    model.weight.grad = torch.zeros(4, 8, dtype=torch.bfloat16)
    opt.step()
    torch.testing.assert_close(model.weight.float(), torch.full((4, 8), 0.25))


def test_optimizer_group_state_count_checked():
    ps = _params("cpu")
    grp = OptimizerGroup(MasterSGD(ps[:2], lr=0.1), torch.optim.SGD(ps[2:], lr=0.1))
    st = grp.state_dict()
    st["opts"] = st["opts"][:1]
    with pytest.raises(ValueError, match="1 optimizers"):
        grp.load_state_dict(st)


@pytest.mark.gpu
def test_master_sgd_kernel_matches_torch_sgd_gpu():
    from arena_amd.ops import _ext
    _ext.load()
    _run("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_shard_sgd_kernel_matches_reference(dtype):
    """The RCCL backend's shard update (``shard_sgd`` HIP kernel) against its fp32 torch
    reference: bit-exact with exact hyperparameters (lr 2^-4, momentum 1/2, wd 2^-10, scale 1/4:
    every product exact, each result rounds once whatever FMAs the compiler forms), and within
    fp32 / bf16 rounding with real ones."""
    from arena_amd.ops import fused
    n = 4096 + 12
    for lr, mu, wd, sc, exact in ((2.0 ** -4, 0.5, 2.0 ** -10, 0.25, True),
                                  (0.05, 0.9, 1e-3, 1.0 / 3, False)):
        g = torch.Generator().manual_seed(5)
        grad = (torch.randn(n, generator=g) * 0.1).to(dtype)
        w = torch.randn(n, generator=g)
        m = torch.randn(n, generator=g) * 0.01
        wr, mr = w.clone(), m.clone()
        wbr = torch.empty(n, dtype=torch.bfloat16) if dtype == torch.bfloat16 else None
        fused.shard_sgd(grad, wr, mr, wbr, lr=lr, momentum=mu, weight_decay=wd, scale=sc)
        wg, mg = w.cuda(), m.cuda()
        wbg = torch.empty(n, dtype=torch.bfloat16, device="cuda") if wbr is not None else None
        fused.shard_sgd(grad.cuda(), wg, mg, wbg, lr=lr, momentum=mu, weight_decay=wd, scale=sc)
        torch.cuda.synchronize()
        if exact:
            assert torch.equal(wg.cpu(), wr) and torch.equal(mg.cpu(), mr)
        else:
            assert float((wg.cpu() - wr).abs().max()) <= 4 * 2.0 ** -23 * float(wr.abs().max())
            assert float((mg.cpu() - mr).abs().max()) <= 4 * 2.0 ** -23 * float(mr.abs().max())
        if wbr is not None:
            assert torch.equal(wbg.cpu(), wg.cpu().to(torch.bfloat16))   # RNE of the master
