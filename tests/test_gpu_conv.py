"""Implicit-GEMM HIP convolution (ops/conv.py) vs an fp32 PyTorch reference of the same op
on the same bf16-rounded operands: forward, input gradient and weight gradient."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# N, C, H, W, K, R, S, stride, pad, dilation
SHAPES = [
    (4, 64, 32, 32, 64, 3, 3, 1, 1, 1),     # ResNet-18 layer1
    (4, 64, 32, 32, 128, 3, 3, 2, 1, 1),    # downsampling 3x3
    (4, 64, 32, 32, 128, 1, 1, 2, 0, 1),    # 1x1 stride-2 shortcut
    (2, 3, 32, 32, 64, 3, 3, 1, 1, 1),      # image stem (C padded to 8)
    (2, 32, 17, 19, 48, 5, 5, 1, 2, 1),     # odd spatial, K not a tile multiple
    (2, 16, 16, 16, 32, 3, 3, 1, 2, 2),     # dilated
    (2, 24, 15, 15, 40, 7, 7, 2, 3, 1),     # 7x7 stride 2 (ENAS child op)
    (4, 256, 8, 8, 512, 3, 3, 2, 1, 1),
    (8, 512, 4, 4, 512, 3, 3, 1, 1, 1),
    (2, 128, 16, 16, 128, 3, 3, 1, 1, 1),   # LDS-patch 3x3 path, 16-pixel rows
    (64, 64, 32, 32, 128, 3, 3, 1, 1, 1),   # LDS-patch path, 128-channel tiles
    (4, 64, 8, 8, 128, 3, 3, 1, 1, 1),      # LDS-patch path, 2 images per tile
]


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_matches_fp32_reference(shape):
    from katib_amd.ops import conv as hc

    N, C, H, W, K, R, S, st, pd, dl = shape
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(N, C, H, W, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, C, R, S, device=dev, generator=g) * (1.0 / (C * R * S) ** 0.5)).to(torch.bfloat16).float()
    OH = (H + 2 * pd - dl * (R - 1) - 1) // st + 1
    OW = (W + 2 * pd - dl * (S - 1) - 1) // st + 1
    gy = torch.randn(N, K, OH, OW, device=dev, generator=g).to(torch.bfloat16)

    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pd, dilation=dl)
    yr.backward(gy.float())

    xh = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wh = w.clone().requires_grad_(True)
    yh = hc.conv2d(xh, wh, stride=st, padding=pd, dilation=dl)
    assert yh.shape == yr.shape and yh.dtype == torch.bfloat16
    yh.backward(gy.contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert _rel(yh, yr) < 1e-2, _rel(yh, yr)
    assert xh.grad.dtype == torch.bfloat16 and _rel(xh.grad, xr.grad) < 1e-2, _rel(xh.grad, xr.grad)
    assert wh.grad.dtype == torch.float32 and _rel(wh.grad, wr.grad) < 2e-3, _rel(wh.grad, wr.grad)


def test_conv_module_dropin():
    from katib_amd.ops import conv as hc

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(16, 32, 3, 1, 1, bias=True).to(dev)
    mod = hc.Conv2d(16, 32, 3, 1, 1, bias=True).to(dev)
    mod.load_state_dict(ref.state_dict())
    x = torch.randn(2, 16, 12, 12, device=dev).to(torch.bfloat16)
    with torch.no_grad():
        ref.weight.copy_(ref.weight.to(torch.bfloat16).float())
        mod.weight.copy_(ref.weight)
    y = mod(x.contiguous(memory_format=torch.channels_last))
    yr = ref(x.float())
    assert _rel(y, yr) < 1e-2


@pytest.mark.parametrize("k,s,size", [(3, 2, 32), (5, 2, 15), (7, 1, 8), (3, 2, 7), (5, 1, 16)])
def test_same_conv_asymmetric_padding(k, s, size):
    """TF 'same' padding (bottom/right-heavy) through the kernel's gather, as the ENAS child uses it."""
    from katib_amd.ops import conv as hc

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(2, 16, size, size, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(24, 16, k, k, device=dev, generator=g) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(24, device=dev, generator=g)
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    t = total // 2
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(F.pad(xr, (t, total - t, t, total - t)), wr, b, stride=s)
    xh = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wh = w.clone().requires_grad_(True)
    yh = hc.same_conv2d(xh, wh, b, s)
    assert yh.shape == yr.shape
    gy = torch.randn(yr.shape, device=dev, generator=g).to(torch.bfloat16)
    yr.backward(gy.float())
    yh.backward(gy)
    assert _rel(yh, yr) < 1e-2
    assert _rel(xh.grad, xr.grad) < 1e-2
    assert _rel(wh.grad, wr.grad) < 2e-3


@pytest.mark.parametrize("stride,C", [(1, 32), (2, 32), (1, 64)])
def test_dgrad_residual_epilogue(stride, C):
    """conv_dgrad(add_d, add_y): dx + (add_y > 0 ? add_d : 0) in the GEMM epilogue (the ResNet
    residual join), on the unit-stride and the phase-split strided paths."""
    from katib_amd.ops import conv as hc

    k = hc.kernels()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    N, H, K, R = 4, 16, 64, 3  # C = 64 at stride 1: the LDS-patch 3x3 kernel
    OH = (H + 2 - R) // stride + 1
    geom = [N, H, H, C, K, R, R, OH, OH, stride, stride, 1, 1, 1, 1]
    w = (torch.randn(K, R, R, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    wt = w.permute(3, 1, 2, 0).contiguous()
    dy = torch.randn(N, OH, OH, K, device=dev, generator=g).to(torch.bfloat16)
    add_d = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    add_y = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    dx = torch.empty(N, H, H, C, device=dev, dtype=torch.bfloat16)
    plain = torch.empty_like(dx)
    k.conv_dgrad(dy, wt, plain, geom)
    k.conv_dgrad(dy, wt, dx, geom, add_d, add_y)
    ref_plain = torch.nn.grad.conv2d_input((N, C, H, H), w.permute(0, 3, 1, 2).float(),
                                           dy.permute(0, 3, 1, 2).float(), stride=stride, padding=1)
    assert _rel(plain.permute(0, 3, 1, 2), ref_plain) < 1e-2
    ref = plain.float() + torch.where(add_y.float() > 0, add_d.float(), torch.zeros_like(add_d.float()))
    assert _rel(dx, ref) < 1e-2
    k.conv_dgrad(dy, wt, dx, geom, add_d)
    assert _rel(dx, plain.float() + add_d.float()) < 1e-2
