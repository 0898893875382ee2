"""Fused MLP kernels (csrc/hip/mlp.hip) vs fp32 PyTorch references on the same bf16 operands:
gathered linear + bias + ReLU, masked dgrad, weight gradient with the fused SGD-momentum
update, few-class cross-entropy; and the trial's HIP path learning like the module path."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


@pytest.fixture(scope="module")
def k():
    from katib_amd.ops.conv import kernels

    return kernels()


@pytest.mark.parametrize("M,N,K", [(128, 256, 784), (64, 1024, 784), (200, 16, 136), (512, 512, 1024)])
def test_lin_fwd_gather_bias_relu_and_mask(k, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(1000, K, device=DEV, generator=g).to(torch.bfloat16)
    idx = torch.randint(0, 1000, (M,), device=DEV, generator=g)
    w = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV, generator=g)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    k.lin_fwd(x, idx, w, b, None, y, True)
    ref = F.relu(x[idx].float() @ w.float().t() + b)
    assert _rel(y, ref) < 1e-2
    mask = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    y2 = torch.empty_like(y)
    k.lin_fwd(x[idx].contiguous(), None, w, None, mask, y2, False)
    ref2 = (x[idx].float() @ w.float().t()) * (mask.float() > 0)
    assert _rel(y2, ref2) < 1e-2


@pytest.mark.parametrize("M,N,K", [(128, 256, 784), (64, 16, 128), (300, 512, 256)])
def test_wgrad_sgd(k, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(1000, K, device=DEV, generator=g).to(torch.bfloat16)
    idx = torch.randint(0, 1000, (M,), device=DEV, generator=g)
    dy = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV, generator=g)
    wm = torch.randn(N, K, device=DEV, generator=g)
    b, bm = torch.randn(N, device=DEV, generator=g), torch.randn(N, device=DEV, generator=g)
    w16, w16t = torch.empty(N, K, device=DEV, dtype=torch.bfloat16), torch.empty(K, N, device=DEV, dtype=torch.bfloat16)
    lr = torch.full((1,), 0.05, device=DEV)
    gw = dy.float().t() @ x[idx].float()
    gb = dy.float().sum(0)
    wm_ref, bm_ref = 0.9 * wm + gw, 0.9 * bm + gb
    w_ref, b_ref = w - 0.05 * wm_ref, b - 0.05 * bm_ref
    k.lin_wgrad_sgd(dy, x, idx, w, wm, w16, w16t, b, bm, lr, 0.9)
    assert _rel(wm, wm_ref) < 1e-2 and _rel(w, w_ref) < 1e-3
    assert _rel(bm, bm_ref) < 1e-2 and _rel(b, b_ref) < 1e-3
    assert _rel(w16, w_ref) < 1e-2 and _rel(w16t, w_ref.t()) < 1e-2


def test_xent_small(k):
    g = torch.Generator(device=DEV).manual_seed(3)
    M = 300
    lg = torch.randn(M, 16, device=DEV, generator=g).to(torch.bfloat16)
    y = torch.randint(0, 10, (M,), device=DEV, generator=g)
    dl = torch.empty_like(lg)
    st = torch.zeros(2, device=DEV)
    k.xent_small(lg, y, None, dl, 10, st)
    ref = F.cross_entropy(lg[:, :10].float(), y)
    p = torch.softmax(lg[:, :10].float(), 1)
    p[torch.arange(M), y] -= 1
    assert abs(float(st[0]) - float(ref)) < 1e-3
    assert int(st[1]) == int((lg[:, :10].float().argmax(1) == y).sum())
    assert _rel(dl[:, :10], p / M) < 1e-2 and float(dl[:, 10:].abs().max()) == 0.0


@pytest.mark.parametrize("hidden,bs", [(256, 128), (1024, 512), (128, 64)])
def test_mnist_mlp_hip_learns_like_module(hidden, bs):
    from katib_amd.workloads import mnist_mlp

    common = ["--epochs", "2", "--hidden", str(hidden), "--batch-size", str(bs), "--num-train", "20000",
              "--num-valid", "2000", "--lr", "0.05"]
    a_hip = mnist_mlp.main(common + ["--impl", "hip"])
    a_mod = mnist_mlp.main(common + ["--impl", "module"])
    assert a_hip > 0.5 and abs(a_hip - a_mod) < 0.05, (a_hip, a_mod)
