"""NHWC depthwise HIP convolution (ops/dwconv.py) vs an fp32 PyTorch reference of the same
op (grouped conv2d with TF 'same' padding) on the same bf16-rounded operands: forward,
input gradient, weight gradient and bias gradient; and the ENAS child ops using it."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


# N, C, H, W, K, stride, depth multiplier
SHAPES = [
    (4, 32, 32, 32, 3, 1, 1),
    (4, 32, 32, 32, 5, 2, 1),
    (2, 64, 16, 16, 7, 1, 2),
    (2, 48, 15, 15, 3, 2, 2),   # odd size: asymmetric 'same' padding
    (2, 16, 8, 8, 7, 2, 1),
    (3, 96, 17, 9, 5, 1, 1),    # non-square, odd
    (4, 3, 32, 32, 3, 1, 1),    # 3-channel image input: channels zero-padded to 8 around the kernel
    (2, 3, 32, 32, 5, 2, 2),
    (2, 12, 9, 9, 3, 1, 2),
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("bias", [True, False])
def test_depthwise_matches_fp32_reference(shape, bias):
    from katib_amd.ops import dwconv as hd

    N, C, H, W, K, s, dm = shape
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(N, C, H, W, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(C * dm, 1, K, K, device=dev, generator=g) / K).to(torch.bfloat16).float()
    b = torch.randn(C * dm, device=dev, generator=g) if bias else None
    assert hd.supported(x, w, C, s)
    pads = []
    outs = []
    for size in (H, W):
        out = -(-size // s)
        total = max((out - 1) * s + K - size, 0)
        pads.append((total // 2, total - total // 2))
        outs.append(out)
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if bias else None
    yr = F.conv2d(F.pad(xr, (pads[1][0], pads[1][1], pads[0][0], pads[0][1])), wr, br, stride=s, groups=C)
    xh = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wh = w.clone().requires_grad_(True)
    bh = b.clone().requires_grad_(True) if bias else None
    yh = hd.depthwise_same(xh, wh, bh, s)
    assert yh.shape == yr.shape == (N, C * dm, outs[0], outs[1]) and yh.dtype == torch.bfloat16
    gy = torch.randn(yr.shape, device=dev, generator=g).to(torch.bfloat16)
    yr.backward(gy.float())
    yh.backward(gy.contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    assert _rel(yh, yr) < 1e-2, _rel(yh, yr)
    assert xh.grad.dtype == torch.bfloat16 and _rel(xh.grad, xr.grad) < 1e-2, _rel(xh.grad, xr.grad)
    assert wh.grad.dtype == torch.float32 and _rel(wh.grad, wr.grad) < 2e-3, _rel(wh.grad, wr.grad)
    if bias:
        assert _rel(bh.grad, br.grad) < 2e-3


def test_enas_child_ops_use_hip_depthwise(monkeypatch):
    """depthwise_convolution and separable_convolution layers route through the HIP kernel."""
    from katib_amd.ops import dwconv as hd
    from katib_amd.workloads.enas_child import Op

    calls = []
    orig = hd.depthwise_same
    monkeypatch.setattr(hd, "depthwise_same", lambda *a: calls.append(1) or orig(*a))
    dev = torch.device("cuda", 0)
    x = torch.randn(8, 32, 16, 16, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for cfg in ({"opt_type": "depthwise_convolution", "filter_size": "5", "stride": "2", "depth_multiplier": "2"},
                {"opt_type": "separable_convolution", "filter_size": "3", "num_filter": "48", "stride": "1",
                 "depth_multiplier": "1"}):
        op = Op(cfg, 32, 16).to(dev).to(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = op(x)
        y.float().sum().backward()
        assert y.shape[1] == op.cout and y.shape[2] == op.hw
    assert len(calls) == 2


def test_enas_child_has_no_miopen_convolution(monkeypatch):
    """Every convolution of a child whose first op is a separable conv on the 3-channel image
    (the repro architecture) runs on the HIP kernels: nn.Conv2d.forward is never reached."""
    import json
    import os

    import torch.nn as nn
    from katib_amd.workloads.enas_child import ChildNet

    def refuse(self, x):
        raise AssertionError("MIOpen / PyTorch conv fallback reached: %s" % (tuple(self.weight.shape),))

    monkeypatch.setattr(nn.Conv2d, "forward", refuse)
    cfg = json.load(open(os.path.join(os.path.dirname(__file__), "..", "scripts", "enas_repro_arch.json")))
    arch = cfg["architecture"]
    arch = json.loads(arch) if isinstance(arch, str) else arch
    nn_config = json.loads(cfg["nn_config"].replace("'", '"'))
    dev = torch.device("cuda", 0)
    net = ChildNet(arch, nn_config).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 32, 32, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = net(x)
    y.float().sum().backward()
    torch.cuda.synchronize()
    assert y.shape == (4, 10) and torch.isfinite(y.float()).all()
