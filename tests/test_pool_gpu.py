"""NHWC max-pool HIP kernels vs PyTorch's max_pool2d on fp32 copies of the same data (MI355X).

Forward values are exact (max is exact in any precision) and the window scan order (kh-major,
first strict maximum) matches PyTorch's, so even ties pick the same input; the backward sums the
same <= ceil(k/s)^2 gradients in fp32 (bf16 rounded once at the end).
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [  # (N, C, H, W, k, s, p)
    (2, 64, 112, 112, 3, 2, 1),   # ResNet stem
    (3, 16, 15, 17, 3, 2, 1),     # odd sizes: partial windows at the far edge
    (2, 8, 8, 8, 2, 2, 0),
    (2, 24, 9, 10, 3, 1, 1),      # stride 1: every input sits in up to 9 windows
    (1, 32, 13, 13, 5, 3, 2),
    (2, 8, 10, 10, 1, 2, 0),      # k < s: the last row/column lies in no window (dx = 0)
]


def _ref(x, dy, k, s, p):
    xr = x.detach().float().requires_grad_(True)
    y = F.max_pool2d(xr, k, s, p)
    y.backward(dy.float())
    return y.detach(), xr.grad


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("ties", [False, True])
def test_maxpool_matches_pytorch(case, dtype, ties):
    from arena_amd.ops import pool
    N, C, H, W, k, s, p = case
    g = torch.Generator(device="cuda").manual_seed(hash((case, ties)) % 2**31)
    x = torch.randn(N, C, H, W, device="cuda", generator=g)
    if ties:  # few distinct values: most windows hold several equal maxima
        x = torch.randint(-2, 3, (N, C, H, W), device="cuda", generator=g).float()
    x = x.to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    assert pool.kernel_ok(x, k, s, p)
    y = pool.max_pool2d(x, k, s, p)
    assert y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn(y.shape, device="cuda", generator=g).to(dtype)
    y.backward(dy)
    y_ref, dx_ref = _ref(x, dy, k, s, p)
    assert torch.equal(y.float(), y_ref)
    if dtype == torch.float32:
        torch.testing.assert_close(x.grad, dx_ref, rtol=1e-6, atol=1e-6)
    else:
        torch.testing.assert_close(x.grad.float(), dx_ref.to(dtype).float(), rtol=8e-3, atol=1e-2)


def test_resnet_stem_uses_the_kernel():
    from arena_amd.models.resnet import resnet
    from arena_amd.ops.pool import MaxPool2dNHWC
    m = resnet("resnet_tiny", num_classes=10, width=8)
    assert isinstance(m.stem[2], MaxPool2dNHWC)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_global_avg_pool_matches_adaptive_pool(dtype):
    """ResNet head pool: output and gradient of the channels_last global average pool against
    F.adaptive_avg_pool2d; the gradient comes back channels_last."""
    from arena_amd.ops.pool import global_avg_pool
    x = torch.randn(6, 256, 7, 7, device="cuda").to(dtype).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    y = global_avg_pool(x)
    y2 = torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x2, 1), 1)
    assert y.shape == y2.shape and torch.allclose(y.float(), y2.float(), rtol=1e-2, atol=1e-3)
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    assert torch.allclose(x.grad.float(), x2.grad.float(), rtol=1e-2, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,classes", [(128, 1000), (5, 37), (33, 64), (6, 1030), (3, 2500)])
def test_fused_cross_entropy_matches_torch(dtype, rows, classes):
    """Fused softmax cross-entropy (mean) against F.cross_entropy on the fp32-upcast logits:
    loss and logits gradient (scaled by a non-unit upstream gradient), run-to-run identical."""
    from arena_amd.ops.pool import cross_entropy
    g = torch.Generator(device="cuda").manual_seed(rows + classes)
    x = (torch.randn(rows, classes, device="cuda", generator=g) * 3).to(dtype).requires_grad_(True)
    y = torch.randint(0, classes, (rows,), device="cuda", generator=g)
    x2 = x.detach().clone().requires_grad_(True)
    loss = cross_entropy(x, y)
    ref = F.cross_entropy(x2.float(), y)
    assert loss.dtype == torch.float32 and loss.shape == ()
    assert torch.allclose(loss, ref, rtol=1e-5, atol=1e-5), (float(loss), float(ref))
    assert torch.equal(loss, cross_entropy(x.detach(), y))
    (loss * 0.75).backward()
    (ref * 0.75).backward()
    assert x.grad.dtype == dtype
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert torch.allclose(x.grad.float(), x2.grad.float(), rtol=tol, atol=tol * 1e-2)
