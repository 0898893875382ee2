"""NHWC bf16 pooling kernels (ENAS ``reduction`` op) vs the fp32 PyTorch formula: forward and
the gathered backward, max and average, windows / strides the ENAS search space produces,
channel padding (3 channels) and non-covering strides (trailing rows no window reaches)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("is_max", [True, False])
@pytest.mark.parametrize("N,C,H,P,S", [(8, 16, 32, 2, 2), (4, 24, 16, 3, 2), (2, 3, 32, 2, 2), (3, 8, 9, 2, 2),
                                       (2, 32, 8, 3, 1), (5, 64, 4, 2, 1)])
def test_pool_nhwc_matches_torch(is_max, N, C, H, P, S):
    from katib_amd.ops import pool as hpool

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(N * 100 + C)
    x = torch.randn(N, C, H, H, device=dev, generator=gen).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    xr = x.float().detach().requires_grad_(True)
    ref = F.max_pool2d(xr, P, S) if is_max else F.avg_pool2d(xr, P, S)
    xh = x.detach().requires_grad_(True)
    out = hpool.pool2d(xh, P, S, is_max)
    assert out.shape == ref.shape and out.dtype == torch.bfloat16
    torch.testing.assert_close(out.float(), ref.detach(), rtol=1e-2, atol=1e-2)
    g = torch.randn(ref.shape, device=dev, generator=gen)
    ref.backward(g)
    out.backward(g.to(torch.bfloat16))
    torch.testing.assert_close(xh.grad.float(), xr.grad, rtol=2e-2, atol=2e-2)


def test_pool_ties_pick_the_first_maximum():
    """Constant windows: torch routes the gradient to the first tap (row-major); so must we."""
    from katib_amd.ops import pool as hpool

    dev = torch.device("cuda", 0)
    x = torch.ones(2, 8, 4, 4, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xh = x.clone().requires_grad_(True)
    out = hpool.pool2d(xh, 2, 2, True)
    out.float().sum().backward()
    xr = x.float().clone().requires_grad_(True)
    F.max_pool2d(xr, 2, 2).sum().backward()
    torch.testing.assert_close(xh.grad.float(), xr.grad)
