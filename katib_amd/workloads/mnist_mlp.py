"""MNIST MLP trial (BASELINE config 2: TPE over lr / batch size / hidden width).

The reference's trials/hour data point (docs/workflow-design.md:41-43, B1) tunes an
MNIST MLP; this is the MI355X workload for that experiment: an MLP
784 -> hidden -> hidden/2 -> 10 trained with SGD + momentum on a learnable synthetic
MNIST-shaped set held in HBM. The whole train step (forward, cross-entropy,
backward, SGD update) is captured once per trial as a HIP graph and replayed, so a
trial is a handful of graph launches per epoch - the per-trial cost the scheduler
sees is dominated by the work, not by Python or kernel-launch overhead. Run in a
warm worker (``entrypoint: katib_amd.workloads.mnist_mlp:main``) a trial also skips
interpreter start and HIP context creation.

Prints ``epoch=<e> loss=<l> Validation-accuracy=<a>`` per epoch (default StdOut
collector format).
"""

from __future__ import annotations

import argparse
import math

import torch
import torch.nn.functional as F

from .common import CapturedStep, Timer, device, report, teacher_vectors


def parse_args(argv):
    p = argparse.ArgumentParser(description="MNIST MLP trial (katib-amd)")
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--num-train", type=int, default=60000)
    p.add_argument("--num-valid", type=int, default=10000)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--capture", type=int, default=1)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    return p.parse_args(argv)


class MLP(torch.nn.Module):
    def __init__(self, hidden: int):
        super().__init__()
        self.fc1 = torch.nn.Linear(784, hidden)
        self.fc2 = torch.nn.Linear(hidden, max(hidden // 2, 10))
        self.fc3 = torch.nn.Linear(max(hidden // 2, 10), 10)

    def forward(self, x):
        return self.fc3(F.relu(self.fc2(F.relu(self.fc1(x)))))


def main(argv=None):
    args = parse_args(argv if argv is not None else [])
    dev = device()
    torch.manual_seed(args.seed)
    x, y = teacher_vectors(args.num_train + args.num_valid, seed=1234, dev=dev)
    tx, ty = x[:args.num_train], y[:args.num_train]
    vx, vy = x[args.num_train:], y[args.num_train:]
    model = MLP(args.hidden).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum)
    bs = max(1, min(args.batch_size, args.num_train))
    steps = args.num_train // bs
    amp = args.dtype == "bf16" and dev.type == "cuda"
    idx = torch.zeros(bs, dtype=torch.long, device=dev)
    loss_buf = torch.zeros((), device=dev)

    def train_step():
        xb, yb = tx.index_select(0, idx), ty.index_select(0, idx)
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
            loss = F.cross_entropy(model(xb), yb)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        loss_buf.add_(loss.detach())
        return loss_buf

    step = CapturedStep(train_step, enabled=bool(args.capture))
    # zero grads exist before capture (set_to_none=False keeps the same buffers)
    for p_ in model.parameters():
        p_.grad = torch.zeros_like(p_)
    gen = torch.Generator(device=dev).manual_seed(args.seed)
    timer = Timer()
    acc = 0.0
    for epoch in range(args.epochs):
        perm = torch.randperm(args.num_train, device=dev, generator=gen)[:steps * bs].view(steps, bs)
        loss_buf.zero_()
        for s in range(steps):
            idx.copy_(perm[s])
            step()
        with torch.no_grad(), torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
            pred = model(vx).argmax(1)
            acc = float((pred == vy).float().mean())
        loss = float(loss_buf) / max(steps, 1)
        if not math.isfinite(loss):
            loss = float("nan")
        report(epoch=epoch, loss=loss, **{"Validation-accuracy": acc})
    report(**{"train_seconds": timer.elapsed()})
    return acc


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
