"""The fused ResNet-18 training step: forward, loss, backward and SGD as a fixed sequence of
katib_hip launches over pre-allocated buffers - no autograd tape, no allocator traffic and
no framework (``at::native``) kernels, so the whole step captures into one HIP graph whose
every node is a hand-written kernel.

What it replaces, launch for launch (round-5 profile ``profiles/resnet18_step_kernels_r05.txt``):

* per-convolution bf16 weight casts, the ``[C][R][S][K]`` transpose for the input gradient and
  the zero-fill of the fp32 weight-gradient accumulator -> one multi-tensor SGD launch
  (``rn_sgd``) that updates every parameter, zeroes its gradient accumulator and re-emits the
  bf16 filter images the next step's convolutions read;
* autograd's gradient sums at the residual joins -> the input-gradient GEMM's epilogue adds the
  (ReLU-masked) residual-branch gradient (``conv_dgrad(add_d, add_y)``);
* the batch ``index_select`` + channel pad of the 3-channel images -> ``rn_gather``;
* pooling, the linear head, softmax cross-entropy and its backward, ``loss_buf += loss`` ->
  ``rn_head`` (two launches);
* ``num_batches_tracked += 1`` -> the BN statistics-finalize kernel.

The math is the reference trial's loop (BASELINE config 3: a PyTorch CIFAR ResNet-18 trained
with SGD + Nesterov momentum + weight decay, cross-entropy loss; ``examples/v1beta1/
trial-images`` style ``train()`` with ``optimizer.zero_grad(); loss.backward();
optimizer.step()``): the same parameters (``model``'s fp32 masters are updated in place, so
``model.eval()`` sees every step) and torch.optim.SGD's update rule
(``d = g + wd p; m = mu m + d; p -= lr (d + mu m)``), with bf16 activations / MFMA operands
and fp32 statistics, accumulators and masters. Checked against a plain fp32 PyTorch
autograd + torch.optim.SGD reference in ``tests/test_gpu_resnet_step.py``.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from .. import _hipload


def kernels():
    try:
        return _hipload.hipkern()
    except ImportError as e:
        raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)


def _nhwc_storage(p: torch.Tensor) -> torch.Tensor:
    """[K, C, R, S] channels_last parameter -> its storage as a contiguous [K, R, S, C] view."""
    v = p.detach().permute(0, 2, 3, 1)
    if not v.is_contiguous():
        raise ValueError("fused ResNet step: conv weights must be channels_last (model.to(memory_format="
                         "torch.channels_last))")
    return v


class _Conv:
    def __init__(self, mod: nn.Conv2d, B: int, H: int, W: int, dgrad: bool, dev):
        if mod.groups != 1 or mod.bias is not None or mod.padding_mode != "zeros":
            raise ValueError("fused ResNet step: bias-free, groups=1, zero-padded convolutions only")
        K, C, R, S = mod.weight.shape
        self.C, self.C8, self.K = C, (C + 7) // 8 * 8, K
        (sh, sw), (ph, pw), (dh, dw) = mod.stride, mod.padding, mod.dilation
        OH = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
        OW = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
        self.out_hw = (OH, OW)
        self.geom = [B, H, W, self.C8, K, R, S, OH, OW, sh, sw, ph, pw, dh, dw]
        self.p = _nhwc_storage(mod.weight)
        RS = R * S
        self.g = torch.zeros(K * RS * self.C8, device=dev)
        self.m = torch.zeros(K * RS * C, device=dev)
        self.wk = torch.empty(K * RS * self.C8, device=dev, dtype=torch.bfloat16)
        self.wt = torch.empty(K * RS * self.C8, device=dev, dtype=torch.bfloat16) if dgrad else None
        self.y = torch.empty(B, OH, OW, K, device=dev, dtype=torch.bfloat16)  # conv output = BN input
        self.dy = torch.empty_like(self.y)  # gradient at the conv output (BN backward writes it)
        self.RS = RS

    def seg(self):
        return (self.p, self.g, self.m, self.wk, self.wt, self.K, self.C, self.C8, self.RS)


class _BN:
    def __init__(self, mod: nn.BatchNorm2d, conv: _Conv, relu: bool, dev):
        if not (mod.affine and mod.track_running_stats):
            raise ValueError("fused ResNet step: affine BN with running statistics only")
        C = mod.num_features
        self.mod, self.relu, self.conv = mod, relu, conv
        self.eps = mod.eps
        self.momentum = mod.momentum if mod.momentum is not None else 0.1
        self.mean = torch.empty(C, device=dev)
        self.invstd = torch.empty(C, device=dev)
        self.gg = torch.zeros(C, device=dev)
        self.gb = torch.zeros(C, device=dev)
        self.mg = torch.zeros(C, device=dev)
        self.mb = torch.zeros(C, device=dev)
        self.y = torch.empty_like(conv.y)

    def segs(self):
        return [(self.mod.weight.detach(), self.gg, self.mg, None, None, 0, 0, 0, 0),
                (self.mod.bias.detach(), self.gb, self.mb, None, None, 0, 0, 0, 0)]

    def fwd(self, k, res=None):
        C = self.mean.numel()
        k.bn_fwd_train(self.conv.y.view(-1, C), None if res is None else res.view(-1, C), self.y.view(-1, C),
                       self.mod.weight.detach(), self.mod.bias.detach(), self.mod.running_mean,
                       self.mod.running_var, self.mean, self.invstd, self.eps, self.momentum, self.relu,
                       self.mod.num_batches_tracked)

    def bwd(self, k, dy, mask_y):
        """dy at this BN's output (masked by ``mask_y`` > 0, the ReLU after it) -> conv.dy."""
        C = self.mean.numel()
        k.bn_bwd(dy.view(-1, C), None if mask_y is None else mask_y.view(-1, C), self.conv.y.view(-1, C),
                 self.mod.weight.detach(), self.mean, self.invstd, self.conv.dy.view(-1, C), None, self.gg, self.gb,
                 accumulate=True)


class FusedResNetStep:
    """One training step of ``workloads.resnet_cifar.ResNet18`` over static buffers.

    ``tx`` [N, 3, H, W] bf16 channels_last and ``ty`` [N] int64 are the device-resident data
    set, ``idx`` [B] int64 the batch indices the caller refreshes before each call,
    ``loss_buf`` a float32 scalar the step adds the batch loss to."""

    def __init__(self, model, tx, ty, idx, loss_buf, lr, momentum, weight_decay, nesterov=True):
        self.k = k = kernels()
        dev = tx.device
        self.model, self.ty, self.idx, self.loss_buf = model, ty, idx, loss_buf
        self.lr, self.mom, self.wd, self.nesterov = float(lr), float(momentum), float(weight_decay), bool(nesterov)
        self.txn = tx.permute(0, 2, 3, 1)
        if not self.txn.is_contiguous() or tx.dtype != torch.bfloat16:
            raise ValueError("fused ResNet step: images must be bf16 channels_last")
        B = idx.numel()
        _, _, H, W = tx.shape
        stem = _Conv(model.stem_conv, B, H, W, dgrad=False, dev=dev)
        self.x0 = torch.empty(B, H, W, stem.C8, device=dev, dtype=torch.bfloat16)
        self.stem, self.stem_bn = stem, _BN(model.stem_bn, stem, True, dev)
        self.blocks = []
        h, w = stem.out_hw
        for blk in model.layers:
            c1 = _Conv(blk.conv1, B, h, w, True, dev)
            b1 = _BN(blk.bn1, c1, True, dev)
            c2 = _Conv(blk.conv2, B, *c1.out_hw, True, dev)
            b2 = _BN(blk.bn2, c2, True, dev)
            cs = bs = None
            if blk.short_conv is not None:
                cs = _Conv(blk.short_conv, B, h, w, True, dev)
                bs = _BN(blk.short_bn, cs, False, dev)
            dtmp = torch.empty(B, h, w, c1.C8, device=dev, dtype=torch.bfloat16) if cs is not None else None
            din = torch.empty(B, h, w, c1.C8, device=dev, dtype=torch.bfloat16)
            self.blocks.append((c1, b1, c2, b2, cs, bs, dtmp, din))
            h, w = c2.out_hw
        fc = model.fc
        Cf, Kc = fc.in_features, fc.out_features
        self.fc_w, self.fc_b = fc.weight.detach(), fc.bias.detach()
        self.fc_gw, self.fc_gb = torch.zeros(Kc, Cf, device=dev), torch.zeros(Kc, device=dev)
        self.fc_mw, self.fc_mb = torch.zeros(Kc, Cf, device=dev), torch.zeros(Kc, device=dev)
        self.HW = h * w
        self.d_last = torch.empty(B, h, w, Cf, device=dev, dtype=torch.bfloat16)
        self.pooled = torch.empty(B, Cf, device=dev)
        self.dl = torch.empty(B, Kc, device=dev)
        self.loss_n = torch.empty(B, device=dev)
        segs = [stem.seg()] + self.stem_bn.segs()
        for c1, b1, c2, b2, cs, bs, _, _ in self.blocks:
            for c, b in ((c1, b1), (c2, b2), (cs, bs)):
                if c is not None:
                    segs += [c.seg()] + b.segs()
        segs += [(self.fc_w, self.fc_gw, self.fc_mw, None, None, 0, 0, 0, 0),
                 (self.fc_b, self.fc_gb, self.fc_mb, None, None, 0, 0, 0, 0)]
        self.table, self.nseg, self.tiles = k.rn_sgd_table(segs)
        self.refresh_filters()

    def refresh_filters(self):
        """Re-emit the bf16 filter images from the fp32 masters (after an outside weight change)."""
        self.k.rn_sgd(self.table, self.nseg, self.tiles, 0.0, 0.0, 0.0, False, False)

    def reset_momentum(self):
        for t in self._momenta():
            t.zero_()

    def _momenta(self):
        out = [self.stem.m, self.stem_bn.mg, self.stem_bn.mb, self.fc_mw, self.fc_mb]
        for c1, b1, c2, b2, cs, bs, _, _ in self.blocks:
            for c, b in ((c1, b1), (c2, b2), (cs, bs)):
                if c is not None:
                    out += [c.m, b.mg, b.mb]
        return out

    def step(self) -> torch.Tensor:
        k = self.k
        stem, sbn = self.stem, self.stem_bn
        # ---- forward
        k.rn_gather(self.txn, self.idx, self.x0)
        k.conv_fwd(self.x0, stem.wk, stem.y, stem.geom)
        sbn.fwd(k)
        a = sbn.y
        ins = []
        for c1, b1, c2, b2, cs, bs, _, _ in self.blocks:
            ins.append(a)
            k.conv_fwd(a, c1.wk, c1.y, c1.geom)
            b1.fwd(k)
            k.conv_fwd(b1.y, c2.wk, c2.y, c2.geom)
            res = a
            if cs is not None:
                k.conv_fwd(a, cs.wk, cs.y, cs.geom)
                bs.fwd(k)
                res = bs.y
            b2.fwd(k, res)
            a = b2.y
        B, C = a.shape[0], a.shape[-1]
        k.rn_head(a.view(B, self.HW, C), self.fc_w, self.fc_b, self.ty, self.idx, self.d_last.view(B, self.HW, C),
                  self.pooled, self.dl, self.loss_n, self.fc_gw, self.fc_gb, self.loss_buf)
        # ---- backward
        d = self.d_last
        for (c1, b1, c2, b2, cs, bs, dtmp, din), a_in in zip(reversed(self.blocks), reversed(ins)):
            out = b2.y
            b2.bwd(k, d, out)
            k.conv_wgrad(b1.y, c2.dy, c2.g.view(c2.K, -1), c2.geom)
            k.conv_dgrad(c2.dy, c2.wt, b1.conv.dy, c2.geom)  # conv2 dgrad -> bn1 output grad (reuses c1.dy)
            b1.bwd(k, c1.dy, b1.y)  # in place: c1.dy holds d(a1) going in, d(c1) coming out
            k.conv_wgrad(a_in, c1.dy, c1.g.view(c1.K, -1), c1.geom)
            if cs is not None:
                bs.bwd(k, d, out)
                k.conv_wgrad(a_in, cs.dy, cs.g.view(cs.K, -1), cs.geom)
                k.conv_dgrad(cs.dy, cs.wt, dtmp, cs.geom)
                k.conv_dgrad(c1.dy, c1.wt, din, c1.geom, dtmp)
            else:
                k.conv_dgrad(c1.dy, c1.wt, din, c1.geom, d, out)
            d = din
        sbn.bwd(k, d, sbn.y)
        k.conv_wgrad(self.x0, stem.dy, stem.g.view(stem.K, -1), stem.geom)
        # ---- optimizer (+ gradient zeroing + bf16 filter images for the next step)
        k.rn_sgd(self.table, self.nseg, self.tiles, self.lr, self.mom, self.wd, self.nesterov, True)
        return self.loss_buf
