"""ENAS child-network trial (drop-in for the reference ``enas-cnn-cifar10`` trial image:
``RunTrial.py:23-100``, ``ModelConstructor.py:24-81``, ``op_library.py:22-155``).

Takes the ``--architecture`` / ``--nn_config`` strings the enas suggestion service
emits, builds the child CNN layer by layer - layer ``l`` consumes the concatenation of
layer ``l-1`` and every earlier layer selected by its skip bits, smaller feature maps
zero-padded (half / half+1) to the largest one - with the op types of the search
space: ``convolution`` (ReLU, Conv 'same', BN), ``separable_convolution`` (ReLU,
depthwise x depth_multiplier + pointwise, BN), ``depthwise_convolution`` (ReLU,
depthwise, BN), ``reduction`` (max/avg pool, identity on 1x1 maps); then global average
pooling, Dropout(0.4) and a dense softmax classifier, trained with Adam(1e-3) on
batches of 128, printing ``Training-Accuracy``, ``Training-Loss``,
``Validation-Accuracy``, ``Validation-Loss`` per epoch.

MI355X specifics: channels-last bf16 convolutions on the hand-written implicit-GEMM
MFMA kernels (``ops/conv.py``; TF 'same' padding handled inside the kernel's gather),
depthwise convolutions on the NHWC depthwise kernels (``ops/dwconv.py``; the 3-channel
image input is zero-padded to 8 channels there, so no op falls back to MIOpen), batch norm
on the NHWC bf16 HIP kernels (``ops/batchnorm.py``, channel counts that are multiples of
8), max / average pooling of the ``reduction`` op on the NHWC bf16 pool kernels
(``ops/pool.py``), synthetic CIFAR-10-shaped data in HBM, and data parallelism
over the trial's GPUs (``WORLD_SIZE`` ranks, RCCL all-reduce of the flat gradient)
in place of ``tf.distribute.MirroredStrategy``.
"""

from __future__ import annotations

import argparse
import json
import math
from typing import Dict, List

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import batchnorm as hbn
from ..ops import conv as hconv
from ..ops import pool as hpool
from ..ops import dwconv as hdw
from .common import CapturedStep, Timer, device, global_avg_pool, pattern_images, report


def _same_pad(size: int, k: int, s: int):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2, out


class _SameConv(nn.Module):
    """TF/Keras ``padding='same'`` convolution (asymmetric padding for even kernels / strides)."""

    def __init__(self, cin, cout, k, s, groups=1, bias=True):
        super().__init__()
        self.k, self.s = k, s
        self.conv = nn.Conv2d(cin, cout, k, s, 0, groups=groups, bias=bias)

    def forward(self, x):
        c = self.conv
        if hconv.supported(x, c.weight, c.groups):  # HIP implicit-GEMM (MFMA) path
            return hconv.same_conv2d(x, c.weight, c.bias, self.s)
        if c.groups > 1 and hdw.supported(x, c.weight, c.groups, self.s):  # HIP depthwise (NHWC) path
            return hdw.depthwise_same(x, c.weight, c.bias, self.s)
        t, b, _ = _same_pad(x.shape[2], self.k, self.s)
        l, r, _ = _same_pad(x.shape[3], self.k, self.s)
        return self.conv(F.pad(x, (l, r, t, b)))


class Op(nn.Module):
    def __init__(self, cfg: Dict, cin: int, hw: int):
        super().__init__()
        self.kind = cfg["opt_type"]
        self.identity = False

        # like op_library.py:51-59, parameters are read from the embedding entry's top level; the
        # enas service nests them under ``opt_params``, so its children run with these defaults
        # (a reference quirk kept for parity; top-level keys, as in the tests, are honoured)
        def geti(k, d):
            return int(cfg[k]) if k in cfg and cfg[k] is not None else d

        if self.kind == "convolution":
            f, k, s = geti("num_filter", 64), geti("filter_size", 3), geti("stride", 1)
            self.body = nn.Sequential(_SameConv(cin, f, k, s), hbn.BatchNorm2d(f, eps=1e-3, momentum=0.01))
            self.cout, self.hw = f, -(-hw // s)
        elif self.kind == "separable_convolution":
            f, k, s, dm = geti("num_filter", 64), geti("filter_size", 3), geti("stride", 1), geti("depth_multiplier", 1)
            self.body = nn.Sequential(_SameConv(cin, cin * dm, k, s, groups=cin, bias=False),
                                      hconv.Conv2d(cin * dm, f, 1), hbn.BatchNorm2d(f, eps=1e-3, momentum=0.01))
            self.cout, self.hw = f, -(-hw // s)
        elif self.kind == "depthwise_convolution":
            k, s, dm = geti("filter_size", 3), geti("stride", 1), geti("depth_multiplier", 1)
            self.body = nn.Sequential(_SameConv(cin, cin * dm, k, s, groups=cin),
                                      hbn.BatchNorm2d(cin * dm, eps=1e-3, momentum=0.01))
            self.cout, self.hw = cin * dm, -(-hw // s)
        elif self.kind == "reduction":
            if hw == 1:
                self.identity = True  # op_library.py:127-131
                self.cout, self.hw = cin, hw
            else:
                p = geti("pool_size", 2)
                st = geti("stride", p)
                self.is_max = cfg.get("reduction_type", "max_pooling") == "max_pooling"
                self.p, self.st = p, st
                self.pool = nn.MaxPool2d(p, st) if self.is_max else nn.AvgPool2d(p, st)
                self.cout, self.hw = cin, (hw - p) // st + 1
        else:
            raise ValueError("unknown opt_type %r" % self.kind)

    def forward(self, x):
        if self.kind == "reduction":
            if self.identity:
                return x
            if hpool.supported(x, self.p, self.st):  # HIP NHWC bf16 pooling (no MIOpen in the graph)
                return hpool.pool2d(x, self.p, self.st, self.is_max)
            return self.pool(x)
        return self.body(F.relu(x))


def _concat(xs: List[torch.Tensor]):
    if len(xs) == 1:
        return xs[0]
    m = max(x.shape[2] for x in xs)
    out = []
    for x in xs:
        d = m - x.shape[2]
        if d:
            h = d // 2
            x = F.pad(x, (h, d - h, h, d - h))
        out.append(x)
    return torch.cat(out, 1)


class ChildNet(nn.Module):
    def __init__(self, arch, nn_config):
        super().__init__()
        self.arch = arch
        self.num_layers = int(nn_config["num_layers"])
        c, h, w = _chw(nn_config["input_sizes"])
        emb = nn_config["embedding"]
        chans, sizes = [c], [h]
        self.ops = nn.ModuleList()
        for l in range(1, self.num_layers + 1):
            opt = arch[l - 1][0]
            skip = arch[l - 1][1:l + 1]
            ins = [l - 1] + [i for i in range(l - 1) if l > 1 and skip[i] == 1]
            cin = sum(chans[i] for i in ins)
            hw = max(sizes[i] for i in ins)
            op = Op(emb[str(opt)], cin, hw)
            self.ops.append(op)
            chans.append(op.cout)
            sizes.append(op.hw)
        self.inputs = [[l - 1] + [i for i in range(l - 1) if l > 1 and arch[l - 1][1:l + 1][i] == 1]
                       for l in range(1, self.num_layers + 1)]
        self.drop = nn.Dropout(0.4)
        self.fc = nn.Linear(chans[-1], int(nn_config["output_sizes"][-1]))

    def forward(self, x):
        layers = [x]
        for op, ins in zip(self.ops, self.inputs):
            layers.append(op(_concat([layers[i] for i in ins])))
        return self.fc(self.drop(global_avg_pool(layers[-1])))


def _chw(sizes):
    """nn_config input_sizes are Keras NHWC ([32, 32, 3])."""
    if len(sizes) == 3 and sizes[2] <= 4 < sizes[0]:
        return int(sizes[2]), int(sizes[0]), int(sizes[1])
    return int(sizes[0]), int(sizes[1]), int(sizes[2])


def _unquote(s: str) -> str:
    """Exec-form container args keep literal quotes (``--architecture="[[...]]"``)."""
    s = s.strip()
    if len(s) >= 2 and s[0] == s[-1] and s[0] in "\"'":
        s = s[1:-1]
    return s


def parse_args(argv):
    p = argparse.ArgumentParser(description="ENAS child CNN trial (katib-amd)")
    p.add_argument("--architecture", type=str, default="")
    p.add_argument("--nn_config", type=str, default="")
    p.add_argument("--num_epochs", type=int, default=10)
    p.add_argument("--num_gpus", type=int, default=1)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--num-train", type=int, default=50000)
    p.add_argument("--num-valid", type=int, default=10000)
    # HIP-graph-captured train step (default); --capture 0 runs it eagerly
    p.add_argument("--capture", type=int, default=1)
    p.add_argument("--seed", type=int, default=0)
    return p.parse_args(argv)


class ChildTrainer:
    """The trial's model, optimizer and (optionally HIP-graph-captured) train step; ``main``
    drives it epoch by epoch, tests drive it step by step."""

    def __init__(self, arch, nn_config, num_train=50000, num_valid=10000, batch_size=128, capture=True, seed=0,
                 comm=None):
        from ..parallel.comm import Comm

        dev = device()
        cuda = dev.type == "cuda"
        torch.manual_seed(seed)
        self.comm = comm or (Comm.from_env(dev.type) if cuda else Comm())
        self.dev, self.cuda = dev, cuda
        mf = torch.channels_last if cuda else torch.contiguous_format
        c, h, w = _chw(nn_config["input_sizes"])
        x, y = pattern_images(num_train + num_valid, (c, h, w), seed=777, dev=dev,
                              dtype=torch.bfloat16 if cuda else torch.float32, noise=2.0)
        x = x.contiguous(memory_format=mf)
        self.tx, self.ty, self.vx, self.vy = x[:num_train], y[:num_train], x[num_train:], y[num_train:]
        self.model = model = ChildNet(arch, nn_config).to(dev).to(memory_format=mf)
        comm = self.comm
        if comm.world_size > 1:  # every rank starts from rank 0's weights
            flat0 = torch.nn.utils.parameters_to_vector(model.parameters()).detach()
            comm.broadcast_(flat0)
            torch.nn.utils.vector_to_parameters(flat0, model.parameters())
        self.opt = opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=cuda, capturable=cuda)
        self.params = list(model.parameters())
        for p_ in self.params:
            p_.grad = torch.zeros_like(p_)
        self.bs = batch_size
        self.shard = num_train // comm.world_size
        self.steps = max(1, self.shard // batch_size)
        self.idx = idx = torch.zeros(batch_size, dtype=torch.long, device=dev)
        self.acc_buf = acc_buf = torch.zeros(2, device=dev)  # loss sum, correct
        tx, ty = self.tx, self.ty

        def train_step():
            xb, yb = tx.index_select(0, idx), ty.index_select(0, idx)
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=cuda):
                logits = model(xb)
            loss = F.cross_entropy(logits.float(), yb)
            opt.zero_grad(set_to_none=False)
            loss.backward()
            acc_buf[0].add_(loss.detach())
            acc_buf[1].add_((logits.argmax(1) == yb).sum())
            if comm.world_size == 1:
                opt.step()
            return acc_buf

        # captured by default: the NaN seen in round 2 came from PyTorch reductions on
        # channels-last bf16 tensors (GAP mean, bias sums), now HIP kernels / a pooling window
        self.step_fn = CapturedStep(train_step, enabled=bool(capture) and comm.world_size == 1, no_miopen=True)

    def step(self, batch_idx: torch.Tensor):
        self.idx.copy_(batch_idx)
        self.step_fn()
        if self.comm.world_size > 1:
            flat = torch.cat([p_.grad.reshape(-1) for p_ in self.params])
            self.comm.allreduce_mean_(flat)
            torch.nn.utils.vector_to_parameters(flat, [p_.grad for p_ in self.params])
            self.opt.step()

    @torch.no_grad()
    def validate(self, num_valid=None, chunk=1000):
        """Eager eval-mode pass over the validation split -> (mean loss, accuracy)."""
        self.model.eval()
        n = self.vx.shape[0] if num_valid is None else num_valid
        vl, vc = 0.0, 0.0
        with torch.autocast(device_type=self.dev.type, dtype=torch.bfloat16, enabled=self.cuda):
            for i in range(0, n, chunk):
                lg = self.model(self.vx[i:i + chunk]).float()
                vl += float(F.cross_entropy(lg, self.vy[i:i + chunk], reduction="sum"))
                vc += float((lg.argmax(1) == self.vy[i:i + chunk]).sum())
        self.model.train()
        return vl / max(n, 1), vc / max(n, 1)


def main(argv=None):
    args = parse_args(argv if argv is not None else [])
    arch = json.loads(_unquote(args.architecture).replace("'", '"'))
    nn_config = json.loads(_unquote(args.nn_config).replace("'", '"'))
    print(">>> arch received by trial\n%s" % arch, flush=True)
    tr = ChildTrainer(arch, nn_config, args.num_train, args.num_valid, args.batch_size, bool(args.capture), args.seed)
    comm, dev, bs, steps = tr.comm, tr.dev, tr.bs, tr.steps
    gen = torch.Generator(device=dev).manual_seed(args.seed + comm.rank)
    timer = Timer()
    va = 0.0
    for epoch in range(args.num_epochs):
        tr.model.train()
        perm = torch.randperm(tr.shard, device=dev, generator=gen)[:steps * bs].view(steps, bs) + comm.rank * tr.shard
        tr.acc_buf.zero_()
        for s in range(steps):
            tr.step(perm[s])
        vl, va = tr.validate(args.num_valid)
        if comm.rank == 0:
            print("\nTotal Epoch {}/{}".format(epoch + 1, args.num_epochs))
            print("Training-Accuracy={}".format(float(tr.acc_buf[1]) / (steps * bs)))
            print("Training-Loss={}".format(float(tr.acc_buf[0]) / steps))
            print("Validation-Accuracy={}".format(va))
            print("Validation-Loss={}".format(vl), flush=True)
    if comm.rank == 0:
        report(train_seconds=timer.elapsed())
    return va


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
