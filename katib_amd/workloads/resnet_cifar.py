"""ResNet-18 on CIFAR-10-shaped data (BASELINE config 3: HyperBand + median-stop).

``--epochs`` is the HyperBand resource. The network is the CIFAR ResNet-18 variant
(3x3 stem, no max-pool, [2, 2, 2, 2] basic blocks, 64-512 channels). MI355X
specifics: channels-last activations, bf16 autocast (fp32 master weights), every
convolution on the hand-written implicit-GEMM MFMA kernels (``ops/conv.py``,
``--conv torch`` switches back to MIOpen), every batch norm with its residual add and
ReLU fused on the NHWC kernels (``ops/batchnorm.py``, ``--bn torch`` for MIOpen),
device-resident synthetic data, and the
whole train step (forward, loss, backward, SGD+Nesterov momentum) captured as one
HIP graph.

Per epoch it prints ``epoch=<e> loss=<l> Validation-accuracy=<a>``; the median-stop
rule compares the objective after ``start_step`` reports.
"""

from __future__ import annotations

import argparse

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import batchnorm as hbn
from ..ops import conv as hconv
from .common import CapturedStep, Timer, device, global_avg_pool, pattern_images, report

Conv = hconv.Conv2d  # HIP implicit GEMM on GPU, stock nn.Conv2d on CPU
BN = hbn.BatchNorm2d  # HIP NHWC batch norm (+ residual + ReLU) on GPU, stock module on CPU


class _TorchBN(nn.BatchNorm2d):
    """MIOpen batch norm with the same (residual, relu) calling convention."""

    def forward(self, x, residual=None, relu=False):
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y


def parse_args(argv):
    p = argparse.ArgumentParser(description="ResNet-18 CIFAR-10 trial (katib-amd)")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--weight-decay", type=float, default=5e-4)
    p.add_argument("--batch-size", type=int, default=256)
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--num-train", type=int, default=50000)
    p.add_argument("--num-valid", type=int, default=10000)
    p.add_argument("--width", type=int, default=64)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--capture", type=int, default=1)
    p.add_argument("--max-steps", type=int, default=0, help="cap steps per epoch (0 = full epoch)")
    p.add_argument("--conv", default="hip", choices=["hip", "torch"], help="convolution backend on GPU")
    p.add_argument("--bn", default="hip", choices=["hip", "torch"], help="batch-norm backend on GPU")
    p.add_argument("--step", default="fused", choices=["fused", "module"],
                   help="GPU train step: 'fused' = ops/resnet_step.py (every launch a katib_hip kernel: no "
                        "autograd tape, one multi-tensor SGD launch); 'module' = the nn.Module + autograd + "
                        "torch.optim path (also used with --conv/--bn torch and on CPU)")
    return p.parse_args(argv)


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = Conv(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = BN(cout)
        self.conv2 = Conv(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = BN(cout)
        self.short_conv = self.short_bn = None
        if stride != 1 or cin != cout:
            self.short_conv, self.short_bn = Conv(cin, cout, 1, stride, bias=False), BN(cout)

    def forward(self, x):
        out = self.bn1(self.conv1(x), relu=True)
        sc = x if self.short_conv is None else self.short_bn(self.short_conv(x))
        return self.bn2(self.conv2(out), residual=sc, relu=True)  # relu(bn2(conv2) + shortcut), one kernel


class ResNet18(nn.Module):
    def __init__(self, width=64, classes=10):
        super().__init__()
        w = width
        self.stem_conv, self.stem_bn = Conv(3, w, 3, 1, 1, bias=False), BN(w)
        layers, cin = [], w
        for i, cout in enumerate((w, 2 * w, 4 * w, 8 * w)):
            stride = 1 if i == 0 else 2
            layers += [BasicBlock(cin, cout, stride), BasicBlock(cout, cout, 1)]
            cin = cout
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        x = self.layers(self.stem_bn(self.stem_conv(x), relu=True))
        return self.fc(global_avg_pool(x))


def main(argv=None):
    global Conv, BN
    args = parse_args(argv if argv is not None else [])
    Conv = hconv.Conv2d if args.conv == "hip" else nn.Conv2d
    BN = hbn.BatchNorm2d if args.bn == "hip" else _TorchBN
    dev = device()
    torch.manual_seed(args.seed)
    cuda = dev.type == "cuda"
    mf = torch.channels_last if cuda else torch.contiguous_format
    x, y = pattern_images(args.num_train + args.num_valid, seed=4321, dev=dev,
                          dtype=torch.bfloat16 if cuda else torch.float32)
    x = x.contiguous(memory_format=mf)
    tx, ty, vx, vy = x[:args.num_train], y[:args.num_train], x[args.num_train:], y[args.num_train:]
    model = ResNet18(args.width).to(dev).to(memory_format=mf)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay,
                          nesterov=True)
    bs = min(args.batch_size, args.num_train)
    steps = args.num_train // bs
    if args.max_steps:
        steps = min(steps, args.max_steps)
    idx = torch.zeros(bs, dtype=torch.long, device=dev)
    loss_buf = torch.zeros((), device=dev)

    def train_step():
        xb = tx.index_select(0, idx).contiguous(memory_format=mf)
        yb = ty.index_select(0, idx)
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=cuda):
            loss = F.cross_entropy(model(xb.float() if not cuda else xb), yb)
        # set_to_none: backward writes each parameter's gradient instead of filling a zeroed buffer
        # and adding into it (two framework launches per parameter inside the captured step)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        loss_buf.add_(loss.detach().float())
        return loss_buf

    if cuda and args.step == "fused" and args.conv == "hip" and args.bn == "hip":
        from ..ops.resnet_step import FusedResNetStep

        model.train()
        fused = FusedResNetStep(model, tx, ty, idx, loss_buf, args.lr, args.momentum, args.weight_decay, nesterov=True)
        train_step = fused.step  # noqa: F811 - same contract: static idx in, loss_buf out
    step = CapturedStep(train_step, enabled=bool(args.capture))
    gen = torch.Generator(device=dev).manual_seed(args.seed)
    timer = Timer()
    acc = 0.0
    for epoch in range(args.epochs):
        model.train()
        perm = torch.randperm(args.num_train, device=dev, generator=gen)[:steps * bs].view(steps, bs)
        loss_buf.zero_()
        for s in range(steps):
            idx.copy_(perm[s])
            step()
        model.eval()
        correct = torch.zeros((), device=dev)
        with torch.no_grad(), torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=cuda):
            for i in range(0, args.num_valid, 1024):
                correct += (model(vx[i:i + 1024]).argmax(1) == vy[i:i + 1024]).sum()
        acc = float(correct) / max(args.num_valid, 1)
        report(epoch=epoch, loss=float(loss_buf) / max(steps, 1), **{"Validation-accuracy": acc})
    report(train_seconds=timer.elapsed())
    return acc


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
