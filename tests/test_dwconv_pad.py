"""Channel padding around the HIP depthwise kernel (ops/dwconv.py depthwise_same): for C not a
multiple of 8 the input, weight and bias are zero-padded to 8 channels and the first C*DM
output channels are kept. Checked on CPU with the kernel replaced by an fp32 grouped conv2d of
the same 'same'-padding semantics: outputs and input / weight / bias gradients must match the
unpadded grouped convolution."""
import pytest
import torch
import torch.nn.functional as F


def _same_grouped(x, w, b, s):
    K = w.shape[-1]
    pads = []
    for size in x.shape[2:]:
        out = -(-size // s)
        total = max((out - 1) * s + K - size, 0)
        pads.append((total // 2, total - total // 2))
    xp = F.pad(x.float(), (pads[1][0], pads[1][1], pads[0][0], pads[0][1]))
    return F.conv2d(xp, w, b, stride=s, groups=x.shape[1])


@pytest.mark.parametrize("C,dm,K,s", [(3, 1, 3, 1), (3, 2, 5, 2), (12, 2, 3, 1), (5, 1, 7, 2)])
def test_padded_depthwise_matches_unpadded(monkeypatch, C, dm, K, s):
    from katib_amd.ops import dwconv as hd

    calls = []

    def fake_apply(x, w, b, stride):
        calls.append(x.shape[1])
        assert x.shape[1] % 8 == 0 and w.shape[0] == x.shape[1] * dm
        return _same_grouped(x, w, b, stride)

    monkeypatch.setattr(hd._DwFn, "apply", fake_apply)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, C, 11, 11, generator=g).to(torch.bfloat16).float()  # the op casts to bf16
    w = torch.randn(C * dm, 1, K, K, generator=g)
    b = torch.randn(C * dm, generator=g)
    xa, wa, ba = (t.clone().requires_grad_(True) for t in (x, w, b))
    xb, wb, bb = (t.clone().requires_grad_(True) for t in (x, w, b))
    ya = hd.depthwise_same(xa, wa, ba, s)
    yb = _same_grouped(xb, wb, bb, s)
    assert ya.shape == yb.shape
    gy = torch.randn(yb.shape, generator=g)
    ya.backward(gy)
    yb.backward(gy)
    assert calls == [(C + 7) // 8 * 8]
    torch.testing.assert_close(ya, yb)
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-2, atol=1e-2)  # dx comes back through bf16
    torch.testing.assert_close(wa.grad, wb.grad)
    torch.testing.assert_close(ba.grad, bb.grad)
