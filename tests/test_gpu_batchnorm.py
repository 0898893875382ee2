"""NHWC bf16 batch norm (+ residual + ReLU) HIP kernels (ops/batchnorm.py) vs an fp32 PyTorch
reference of the same op on the same bf16 inputs: output, running statistics, and the
gradients of input, residual, weight and bias; eval mode with running statistics."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("shape", [(8, 64, 16, 16), (4, 128, 8, 8), (2, 512, 4, 4), (3, 24, 5, 7), (16, 64, 32, 32)])
@pytest.mark.parametrize("residual,relu", [(False, False), (False, True), (True, True)])
def test_bn_train_matches_fp32(shape, residual, relu):
    from katib_amd.ops.batchnorm import BatchNorm2d

    N, C, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(5)
    x = (torch.randn(shape, device=DEV, generator=g) * 2 + 0.3).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    r = torch.randn(shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last) if residual else None
    bn = BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.5, 0.5, generator=g)
    ref = torch.nn.BatchNorm2d(C).to(DEV)
    ref.load_state_dict(bn.state_dict())
    xh = x.clone().requires_grad_(True)
    rh = r.clone().requires_grad_(True) if residual else None
    y = bn(xh, residual=rh, relu=relu)
    xf = x.float().requires_grad_(True)
    rf = r.float().requires_grad_(True) if residual else None
    yr = ref(xf)
    if residual:
        yr = yr + rf
    if relu:
        yr = F.relu(yr)
    assert _rel(y, yr) < 2e-2
    assert _rel(bn.running_mean, ref.running_mean) < 1e-4 and _rel(bn.running_var, ref.running_var) < 1e-3
    gy = torch.randn(shape, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    yr.backward(gy.float())
    assert _rel(xh.grad, xf.grad) < 3e-2
    assert _rel(bn.weight.grad, ref.weight.grad) < 2e-2 and _rel(bn.bias.grad, ref.bias.grad) < 2e-2
    if residual:
        assert _rel(rh.grad, rf.grad) < 1e-2
    bn.eval()
    ref.eval()
    with torch.no_grad():
        ye = bn(x, residual=r, relu=relu)
        yre = ref(x.float()) + (r.float() if residual else 0)
        yre = F.relu(yre) if relu else yre
    assert _rel(ye, yre) < 2e-2
