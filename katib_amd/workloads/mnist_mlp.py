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

On a GPU the default ``--impl hip`` trains on the fused kernels of
``csrc/hip/mlp.hip``: one train step is nine graph-captured launches -
three fused linear+bias+ReLU forwards (the first gathers the minibatch rows from the
device-resident dataset itself), a few-class cross-entropy that also emits the logit
gradient, two dgrad GEMMs with the ReLU-derivative mask in their epilogue, and three
weight-gradient GEMMs that apply SGD with momentum to the fp32 masters (and refresh
the bf16 weight / transposed-weight shadows) in their epilogue. ``--impl module`` is the
``nn.Module`` + autocast + ``torch.optim.SGD`` path (CPU default, oracle).

Prints ``epoch=<e> loss=<l> Validation-accuracy=<a>`` per epoch (default StdOut
collector format).
"""

from __future__ import annotations

import time as _time

_T_MODULE = _time.time()  # cold-trial phases: the module starts importing (interpreter + katib_amd up)

import argparse  # noqa: E402
import math  # noqa: E402

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from .common import CapturedStep, Timer, device, phase, process_start_time, report, teacher_vectors  # noqa: E402

_T_TORCH = _time.time()


_SET_TO_NONE = __import__("os").environ.get("KATIB_MLP_SET_TO_NONE", "1") != "0"


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
    p.add_argument("--impl", default="auto", choices=["auto", "hip", "module"])
    # the reference's B1 experiment (docs/workflow-design.md:58-108) tunes these two as well
    p.add_argument("--num-layers", type=int, default=0,
                   help="hidden layers of width --hidden (0: the 784-h-h/2-10 net of the fused HIP path)")
    p.add_argument("--optimizer", default="sgd", choices=["sgd", "adam", "ftrl"])
    p.add_argument("--unroll", type=int, default=1,
                   help="train steps per captured HIP graph replay (the batch index comes from a device-side "
                        "step counter into the epoch's permutation, so one replay runs that many SGD steps); "
                        "1 (default) = one replay + one index copy per step. Measured on the B1 trials (3 per "
                        "GPU): 16 is slower (median trial 3.4-3.7 vs 2.4 s: the larger graph's capture and the "
                        "counter / gather kernels cost more than the per-step replay launches they remove, "
                        "profiles/b1_trial_phases_r05.txt)")
    return p.parse_args(argv)


class DeepMLP(torch.nn.Module):
    """784 -> hidden x num_layers -> 10 (the B1 experiment's ``num-layers``)."""

    def __init__(self, hidden: int, num_layers: int):
        super().__init__()
        dims = [784] + [hidden] * num_layers
        self.hidden = torch.nn.ModuleList(torch.nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:]))
        self.out = torch.nn.Linear(dims[-1], 10)

    def forward(self, x):
        for fc in self.hidden:
            x = F.relu(fc(x))
        return self.out(x)


class Ftrl(torch.optim.Optimizer):
    """FTRL-proximal (McMahan et al. 2013) as MXNet's ``Ftrl`` optimizer - the B1 experiment's
    third optimizer choice: z += g - (sqrt(n + g^2) - sqrt(n)) / lr * w; n += g^2;
    w = (sign(z) * l1 - z) / ((beta + sqrt(n)) / lr + wd) where |z| > l1, else 0. Tensor ops only,
    so the step is HIP-graph capturable."""

    def __init__(self, params, lr=0.1, lamda1=0.01, beta=1.0, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, lamda1=lamda1, beta=beta, weight_decay=weight_decay))
        for g in self.param_groups:
            for p in g["params"]:
                st = self.state[p]
                st["z"] = torch.zeros_like(p)
                st["n"] = torch.zeros_like(p)

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            lr, l1, beta, wd = g["lr"], g["lamda1"], g["beta"], g["weight_decay"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                z, n, grad = st["z"], st["n"], p.grad
                sq_old = n.sqrt()
                n.addcmul_(grad, grad)
                z.add_(grad).sub_((n.sqrt() - sq_old) / lr * p)
                p.copy_((torch.sign(z) * l1 - z) / ((beta + n.sqrt()) / lr + wd) * (z.abs() > l1))


class MLP(torch.nn.Module):
    def __init__(self, hidden: int):
        super().__init__()
        self.fc1 = torch.nn.Linear(784, hidden)
        self.fc2 = torch.nn.Linear(hidden, max(hidden // 2, 10))
        self.fc3 = torch.nn.Linear(max(hidden // 2, 10), 10)

    def forward(self, x):
        return self.fc3(F.relu(self.fc2(F.relu(self.fc1(x)))))


class HipMLP:
    """784 -> h -> h/2 -> 10 on the fused HIP kernels; parameters initialised from an
    ``MLP`` module (same init as the module path). The output layer is padded to 16 rows
    (zero weights, zero gradients) so every GEMM dimension is a multiple of 8."""

    def __init__(self, ref: MLP, lr: float, momentum: float, dev):
        from ..ops.conv import kernels

        self.k = kernels()
        self.momentum = momentum
        self.lr = torch.full((1,), lr, device=dev, dtype=torch.float32)
        self.layers = []
        for i, fc in enumerate((ref.fc1, ref.fc2, ref.fc3)):
            w = fc.weight.detach().float()
            b = fc.bias.detach().float()
            if i == 2:
                w = torch.cat([w, w.new_zeros(16 - w.shape[0], w.shape[1])])
                b = torch.cat([b, b.new_zeros(16 - b.shape[0])])
            w = w.to(dev).contiguous()
            b = b.to(dev).contiguous()
            self.layers.append({"w": w, "wm": torch.zeros_like(w), "w16": w.to(torch.bfloat16),
                                "w16t": w.t().contiguous().to(torch.bfloat16), "b": b, "bm": torch.zeros_like(b)})
        self.stats = torch.zeros(2, device=dev, dtype=torch.float32)

    def forward(self, x, idx=None, save=False):
        k, L = self.k, self.layers
        M = idx.numel() if idx is not None else x.shape[0]
        acts = []
        h = x
        for i, l in enumerate(L):
            y = torch.empty((M, l["w"].shape[0]), device=x.device, dtype=torch.bfloat16)
            k.lin_fwd(h, idx if i == 0 else None, l["w16"], l["b"], None, y, i < 2)
            acts.append(y)
            h = y
        return acts if save else acts[-1]

    def train_step(self, x, y, idx):
        k, L = self.k, self.layers
        h1, h2, lg = self.forward(x, idx, save=True)
        M = idx.numel()
        dl = torch.empty_like(lg)
        k.xent_small(lg, y, idx, dl, 10, self.stats)
        dh2 = torch.empty_like(h2)
        k.lin_fwd(dl, None, L[2]["w16t"], None, h2, dh2, False)  # dgrad before the update of W3
        self._sgd(dl, h2, None, L[2])
        dh1 = torch.empty_like(h1)
        k.lin_fwd(dh2, None, L[1]["w16t"], None, h1, dh1, False)
        self._sgd(dh2, h1, None, L[1])
        self._sgd(dh1, x, idx, L[0])
        return self.stats

    def _sgd(self, dy, x, idx, l):
        self.k.lin_wgrad_sgd(dy, x, idx, l["w"], l["wm"], l["w16"], l["w16t"], l["b"], l["bm"], self.lr,
                             self.momentum)


def main(argv=None):
    phase("process", process_start_time())
    phase("module", _T_MODULE)
    phase("torch", _T_TORCH)
    args = parse_args(argv if argv is not None else [])
    dev = device()
    if dev.type == "cuda":
        torch.zeros(1, device=dev).add_(1)
        torch.cuda.synchronize()
    phase("hip_init")
    torch.manual_seed(args.seed)
    x, y = teacher_vectors(args.num_train + args.num_valid, seed=1234, dev=dev)
    phase("data")
    tx, ty = x[:args.num_train], y[:args.num_train]
    vx, vy = x[args.num_train:], y[args.num_train:]
    custom = args.num_layers > 0 or args.optimizer != "sgd"
    model = (DeepMLP(args.hidden, args.num_layers or 2) if custom else MLP(args.hidden)).to(dev)
    impl = args.impl if args.impl != "auto" else ("hip" if dev.type == "cuda" and not custom else "module")
    if impl == "hip":
        if custom:
            raise SystemExit("--impl hip runs the 784-h-h/2-10 net with SGD only")
        return _main_hip(args, dev, model, tx, ty, vx, vy)
    if args.optimizer == "adam":
        opt = torch.optim.Adam(model.parameters(), lr=args.lr, capturable=dev.type == "cuda")
    elif args.optimizer == "ftrl":
        opt = Ftrl(model.parameters(), lr=args.lr)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum)
    bs = max(1, min(args.batch_size, args.num_train))
    steps = args.num_train // bs
    amp = args.dtype == "bf16" and dev.type == "cuda"
    idx = torch.zeros(bs, dtype=torch.long, device=dev)
    loss_buf = torch.zeros((), device=dev)
    correct_buf = torch.zeros((), device=dev)
    # launch-bound inner loop (batch-64 MLP steps are ~30 tiny kernels): U steps per graph replay, each
    # taking its batch indices from row `counter` of the epoch's permutation (device-side, no host copy)
    U = max(1, args.unroll) if (dev.type == "cuda" and args.capture) else 1
    perm_rows = torch.zeros(max(steps, 1), bs, dtype=torch.long, device=dev)
    counter = torch.zeros(1, dtype=torch.long, device=dev)

    def train_step():
        if U > 1:
            idx_ = perm_rows.index_select(0, counter).view(-1)
            counter.add_(1)
        else:
            idx_ = idx
        xb, yb = tx.index_select(0, idx_), ty.index_select(0, idx_)
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
            logits = model(xb)
            loss = F.cross_entropy(logits, yb)
        # set_to_none: backward writes each gradient instead of a fill + an accumulate-add per
        # parameter (the captured step replays into the graph pool's same addresses; ~19 of the
        # ~75 kernels of a 3-layer bf16 step, profiles/b1_module_step_r05.log). =0: the old form.
        opt.zero_grad(set_to_none=_SET_TO_NONE)
        loss.backward()
        opt.step()
        loss_buf.add_(loss.detach())
        correct_buf.add_((logits.detach().argmax(1) == yb).sum())
        return loss_buf

    def train_chunk():
        for _ in range(U):
            out = train_step()
        return out

    step = CapturedStep(train_step, enabled=bool(args.capture))
    # one eager warm-up chunk (U real steps) creates the optimizer state and the allocator blocks
    chunk = CapturedStep(train_chunk, enabled=bool(args.capture), warmup=1) if U > 1 else None
    # zero grads exist before the first (eager) step: the capturable-Adam state pre-step below needs them
    for p_ in model.parameters():
        p_.grad = torch.zeros_like(p_)
    if args.optimizer == "adam" and dev.type == "cuda":  # capturable Adam: state on the device before capture
        opt.step()
        with torch.no_grad():
            for p_, st in opt.state.items():
                for v in st.values():
                    if torch.is_tensor(v):
                        v.zero_()
    gen = torch.Generator(device=dev).manual_seed(args.seed)
    phase("model")
    timer = Timer()
    acc = 0.0
    for epoch in range(args.epochs):
        perm = torch.randperm(args.num_train, device=dev, generator=gen)[:steps * bs].view(steps, bs)
        loss_buf.zero_()
        correct_buf.zero_()
        if U > 1:
            perm_rows[:steps].copy_(perm)
            counter.zero_()
            for c in range(steps // U):
                chunk()
                if epoch == 0 and c == chunk.warmup:
                    phase("captured")  # warm-up chunks + graph capture + first replay issued
            for _ in range(steps % U):
                step()
        else:
            for s in range(steps):
                idx.copy_(perm[s])
                step()
                if epoch == 0 and s == step.warmup:
                    phase("captured")  # warm-up steps + graph capture + first replay issued
        with torch.no_grad(), torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
            pred = model(vx).argmax(1)
            acc = float((pred == vy).float().mean())
        loss = float(loss_buf) / max(steps, 1)
        if not math.isfinite(loss):
            loss = float("nan")
        report(epoch=epoch, loss=loss, **{"Validation-accuracy": acc,
                                         "Train-accuracy": float(correct_buf) / max(steps * bs, 1)})
        if epoch == 0:
            phase("first_metric")
    report(**{"train_seconds": timer.elapsed()})
    phase("trained")
    return acc


def _main_hip(args, dev, model, tx, ty, vx, vy):
    net = HipMLP(model, args.lr, args.momentum, dev)
    txb, vxb = tx.to(torch.bfloat16).contiguous(), vx.to(torch.bfloat16).contiguous()
    bs = max(1, min(args.batch_size, args.num_train))
    steps = args.num_train // bs
    idx = torch.zeros(bs, dtype=torch.long, device=dev)
    step = CapturedStep(lambda: net.train_step(txb, ty, idx), enabled=bool(args.capture))
    gen = torch.Generator(device=dev).manual_seed(args.seed)
    timer = Timer()
    acc = 0.0
    for epoch in range(args.epochs):
        perm = torch.randperm(args.num_train, device=dev, generator=gen)[:steps * bs].view(steps, bs)
        net.stats.zero_()
        for s in range(steps):
            idx.copy_(perm[s])
            step()
        with torch.no_grad():
            acc = float((net.forward(vxb)[:, :10].argmax(1) == vy).float().mean())
        loss = float(net.stats[0]) / max(steps, 1)
        report(epoch=epoch, loss=loss if math.isfinite(loss) else float("nan"), **{"Validation-accuracy": acc})
    report(**{"train_seconds": timer.elapsed()})
    return acc


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
