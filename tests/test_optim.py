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


@pytest.mark.gpu
def test_master_sgd_kernel_matches_torch_sgd_gpu():
    from arena_amd.ops import _ext
    _ext.load()
    _run("cuda")
