"""The fused ResNet-18 train step (ops/resnet_step.py) against plain fp32 PyTorch: the same
initial weights trained by autograd + torch.optim.SGD(nesterov) with nn.Conv2d / nn.BatchNorm2d.
The fused step keeps bf16 activations and MFMA operands (fp32 masters, statistics and
accumulators), so the comparison is at bf16 tolerance."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

LR, MOM, WD = 0.05, 0.9, 5e-4


def _models(width):
    from katib_amd.ops import batchnorm as hbn
    from katib_amd.ops import conv as hconv
    from katib_amd.workloads import resnet_cifar as rc

    torch.manual_seed(0)
    rc.Conv, rc.BN = hconv.Conv2d, hbn.BatchNorm2d
    ours = rc.ResNet18(width)
    try:
        rc.Conv, rc.BN = torch.nn.Conv2d, rc._TorchBN
        ref = rc.ResNet18(width)
    finally:
        rc.Conv, rc.BN = hconv.Conv2d, hbn.BatchNorm2d
    ref.load_state_dict(ours.state_dict())
    return ours, ref


def _data(n, dev):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, 3, 32, 32, generator=g).to(dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (n,), generator=g).to(dev)
    return x, y


def _cmp(a, b):
    cos = float(F.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0))
    return cos, float(a.norm() / b.norm().clamp_min(1e-20))


def _grads_at(params, ref, xb, yb, autocast):
    """Training-mode gradients of the plain PyTorch model (fp32, or PyTorch's own bf16 autocast on
    MIOpen) at the given weights."""
    import copy

    m = copy.deepcopy(ref)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(params[n])
            p.grad = None
    if autocast:
        m = m.to(memory_format=torch.channels_last)
        xb = xb.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        loss = F.cross_entropy(m(xb), yb)
    loss.backward()
    return {n: p.grad.detach().float() for n, p in m.named_parameters()}


def test_fused_step_matches_fp32_autograd_sgd():
    from katib_amd.ops.resnet_step import FusedResNetStep

    dev = torch.device("cuda", 0)
    ours, ref = _models(16)
    ours = ours.to(dev).to(memory_format=torch.channels_last).train()
    ref = ref.to(dev).train()
    p0 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    tx, ty = _data(96, dev)
    B = 32
    idx = torch.zeros(B, dtype=torch.long, device=dev)
    loss_buf = torch.zeros((), device=dev)
    step = FusedResNetStep(ours, tx, ty, idx, loss_buf, LR, MOM, WD, nesterov=True)
    opt = torch.optim.SGD(ref.parameters(), lr=LR, momentum=MOM, weight_decay=WD, nesterov=True)
    perm = torch.randperm(96, generator=torch.Generator().manual_seed(2)).to(dev)
    ours_p = dict(ours.named_parameters())
    mom_est = {n: torch.zeros_like(p) for n, p in p0.items()}
    for s in range(3):
        idx.copy_(perm[s * B:(s + 1) * B])
        before = float(loss_buf)
        p_prev = {n: p.detach().clone() for n, p in ours_p.items()}
        step.step()
        ours_loss = float(loss_buf) - before
        xb = tx.index_select(0, idx).float()
        loss = F.cross_entropy(ref(xb), ty.index_select(0, idx))
        opt.zero_grad()
        loss.backward()
        # recover our gradient from the update: dp = -lr ((1 + mu) d + mu^2 m_prev), d = g + wd p,
        # m = mu m_prev + d, and compare it per tensor with the fp32 one. bf16 activations cost
        # accuracy towards the input layers (random data and labels: small, cancelling gradients),
        # so the bar is the same comparison for PyTorch's own bf16 autocast step on the reference's
        # weights and batch
        # weights of the fused step before this update: the fp32 and autocast gradients are taken there
        # (the two trajectories drift apart, and gradients at different weights are not comparable)
        at_ours = _grads_at(p_prev, ref, xb, ty.index_select(0, idx), autocast=False)
        auto = _grads_at(p_prev, ref, xb, ty.index_select(0, idx), autocast=True)
        bad = []
        for n, pr in ref.named_parameters():
            dp = ours_p[n].detach() - p_prev[n]
            d = (-dp / LR - MOM * MOM * mom_est[n]) / (1 + MOM)
            mom_est[n] = MOM * mom_est[n] + d
            g_ours = d - WD * p_prev[n]
            cos, ratio = _cmp(g_ours, at_ours[n])
            cos_a, ratio_a = _cmp(auto[n], at_ours[n])
            print("step %d grad %-28s fused cos %.4f ratio %.4f | torch bf16 autocast cos %.4f ratio %.4f"
                  % (s, n, cos, ratio, cos_a, ratio_a))
            # the norm ratio of the small BN-parameter gradients wanders by ~0.1-0.2 under bf16 in both
            # implementations; 0.25 still catches a missing / doubled term
            if cos < min(0.97, cos_a - 0.05) or abs(ratio - 1) > 0.25:
                bad.append((s, n, round(cos, 4), round(ratio, 4), round(cos_a, 4), round(ratio_a, 4)))
        assert not bad, bad
        opt.step()
        assert abs(ours_loss - float(loss)) < 0.03 * abs(float(loss)) + 1e-3, (s, ours_loss, float(loss))
    torch.cuda.synchronize()
    # end state: the trajectories drift apart (random data and labels, lr 0.05 with momentum: the
    # per-step gradients were compared above at our own weights), so only what does not depend on
    # the drift is compared - the step counters, and the stem BN running statistics (the stem
    # weights see one bf16-noise update per step)
    ours_b, ref_b = dict(ours.named_buffers()), dict(ref.named_buffers())
    for n, br in ref_b.items():
        if n.endswith("num_batches_tracked"):
            assert int(ours_b[n]) == int(br) == 3, n
        else:
            assert torch.isfinite(ours_b[n]).all(), n
    for n in ("stem_bn.running_mean", "stem_bn.running_var"):
        assert torch.allclose(ours_b[n], ref_b[n], rtol=0.05, atol=0.02), n


def test_fused_step_captures_and_learns():
    from katib_amd.ops.resnet_step import FusedResNetStep
    from katib_amd.workloads.common import CapturedStep

    dev = torch.device("cuda", 0)
    ours, _ = _models(16)
    ours = ours.to(dev).to(memory_format=torch.channels_last).train()
    tx, ty = _data(64, dev)
    idx = torch.arange(64, device=dev)
    loss_buf = torch.zeros((), device=dev)
    fused = FusedResNetStep(ours, tx, ty, idx, loss_buf, 0.02, MOM, WD)
    step = CapturedStep(fused.step)
    losses = []
    for _ in range(12):
        before = float(loss_buf)
        step()
        losses.append(float(loss_buf) - before)
    assert step.graph is not None
    assert all(l == l for l in losses)  # no NaN
    assert losses[-1] < 0.7 * losses[0], losses


def test_fused_step_rejects_non_channels_last():
    from katib_amd.ops.resnet_step import FusedResNetStep

    dev = torch.device("cuda", 0)
    ours, _ = _models(8)
    ours = ours.to(dev)  # contiguous (NCHW) weights
    tx, ty = _data(8, dev)
    with pytest.raises(ValueError):
        FusedResNetStep(ours, tx, ty, torch.arange(8, device=dev), torch.zeros((), device=dev), 0.1, 0.9, 0.0)
