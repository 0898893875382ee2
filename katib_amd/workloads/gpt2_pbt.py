"""GPT-2-small language model trial for Population Based Training (BASELINE config 5).

Each PBT trial continues training from its parent's checkpoint (the PBT service
prepares the trial's checkpoint directory from the parent's, reference
``pkg/suggestion/v1beta1/pbt/service.py:260-268``), trains ``--steps`` steps with
the trial's hyperparameters, evaluates, and writes its own checkpoint back.

Model: GPT-2 small (12 layers, d=768, 12 heads, context 1024, vocab 50257, tied
embeddings, GELU MLP, pre-LayerNorm) - 124M parameters. On MI355X (``--impl flat``,
the default on a GPU) the model is :class:`katib_amd.models.gpt2.GPT2Flat`: flat fp32
master / bf16 shadow / bf16 gradient buffers, a hand-written backward, the gfx950
kernels of ``csrc/hip/transformer.hip`` (flash attention, fused residual LayerNorm,
GELU, vocabulary cross-entropy, one-launch AdamW with global-norm clipping) around
hipBLASLt GEMMs, the whole step (forward, backward, optimizer) replayed as one HIP
graph. ``--impl module`` is the plain ``nn.Module`` + autocast + ``torch.optim.AdamW``
path (the CPU default and the numerical oracle). Data: synthetic Markov-chain tokens
resident in HBM.

Checkpoints: the parent's state is fetched GPU-to-GPU from the warm worker that
trained it (:mod:`katib_amd.parallel.p2p_ckpt`, peer copy over xGMI); ``model.pt`` +
``optim.pt`` (``torch.save``, loaded with ``weights_only=True``) in
``$KATIB_TRIAL_CHECKPOINT_DIR`` (or ``--checkpoint-dir``) are the durable fallback.

Prints ``step=<n> loss=<l>`` while training and ``Validation-loss=<l>
Validation-accuracy=<token accuracy>`` at the end.
"""

from __future__ import annotations

import argparse
import math
import os
import time
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models.gpt2 import GPT2Flat
from ..ops.transformer import get_ops
from ..parallel import p2p_ckpt
from .common import CapturedStep, Timer, device, markov_tokens, report


@dataclass
class GPTConfig:
    vocab: int = 50257
    ctx: int = 1024
    n_layer: int = 12
    n_head: int = 12
    d: int = 768
    dropout: float = 0.0


PRESETS = {
    "gpt2-small": GPTConfig(),
    "tiny": GPTConfig(vocab=512, ctx=64, n_layer=2, n_head=2, d=64),
    # smallest shape the hand-written kernels take (D = 256k, head dim 64, T % 128 == 0)
    "mini": GPTConfig(vocab=512, ctx=128, n_layer=2, n_head=4, d=256),
}


def hip_supported(cfg: GPTConfig, T: int) -> bool:
    """Shapes the gfx950 GPT-2 kernels accept (transformer_bind.cpp checks the same)."""
    k = cfg.d // 256
    return (cfg.d % 256 == 0 and k in (1, 2, 3, 4, 5, 6, 8) and cfg.d == 64 * cfg.n_head
            and T % 128 == 0)


class Block(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.ln1 = nn.LayerNorm(c.d)
        self.qkv = nn.Linear(c.d, 3 * c.d)
        self.proj = nn.Linear(c.d, c.d)
        self.ln2 = nn.LayerNorm(c.d)
        self.fc = nn.Linear(c.d, 4 * c.d)
        self.fc2 = nn.Linear(4 * c.d, c.d)
        self.h = c.n_head

    def forward(self, x):
        B, T, D = x.shape
        q, k, v = self.qkv(self.ln1(x)).split(D, dim=2)
        q = q.view(B, T, self.h, D // self.h).transpose(1, 2)
        k = k.view(B, T, self.h, D // self.h).transpose(1, 2)
        v = v.view(B, T, self.h, D // self.h).transpose(1, 2)
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        x = x + self.proj(a.transpose(1, 2).reshape(B, T, D))
        return x + self.fc2(F.gelu(self.fc(self.ln2(x)), approximate="tanh"))


class GPT(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.c = c
        self.wte = nn.Embedding(c.vocab, c.d)
        self.wpe = nn.Embedding(c.ctx, c.d)
        self.blocks = nn.ModuleList(Block(c) for _ in range(c.n_layer))
        self.ln_f = nn.LayerNorm(c.d)
        self.apply(self._init)
        for n, p in self.named_parameters():
            if n.endswith("proj.weight") or n.endswith("fc2.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * c.n_layer))

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.02)
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, 0.02)

    def forward(self, idx):
        B, T = idx.shape
        x = self.wte(idx) + self.wpe(torch.arange(T, device=idx.device))
        for b in self.blocks:
            x = b(x)
        return F.linear(self.ln_f(x), self.wte.weight)  # tied LM head

    def n_params(self):
        return sum(p.numel() for p in self.parameters()) - self.wpe.weight.numel()


def parse_args(argv):
    p = argparse.ArgumentParser(description="GPT-2 PBT trial (katib-amd)")
    p.add_argument("--lr", type=float, default=3e-4)
    p.add_argument("--weight-decay", type=float, default=0.1)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch-size", type=int, default=8)
    p.add_argument("--seq-len", type=int, default=0, help="0 = model context")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--eval-batches", type=int, default=4)
    p.add_argument("--model", default="gpt2-small", choices=sorted(PRESETS))
    p.add_argument("--num-tokens", type=int, default=4_000_000)
    p.add_argument("--checkpoint-dir", default="")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--capture", type=int, default=1)
    p.add_argument("--p2p", type=int, default=1, help="hand checkpoints GPU-to-GPU (parallel.p2p_ckpt)")
    p.add_argument("--save-files", type=int, default=1, help="also write model.pt/optim.pt (durable copy)")
    p.add_argument("--impl", default="auto", choices=["auto", "flat", "module"],
                   help="flat: flat-buffer model on the HIP kernels (GPU default); module: nn.Module + autograd")
    p.add_argument("--ops", default="auto", choices=["auto", "hip", "torch"], help="kernel backend of --impl flat")
    return p.parse_args(argv)


def _tensors(obj):
    """Every tensor of a (nested) checkpoint state."""
    if torch.is_tensor(obj):
        yield obj
    elif isinstance(obj, dict):
        for v in obj.values():
            yield from _tensors(v)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            yield from _tensors(v)


def _ckpt_dir(args):
    return args.checkpoint_dir or os.environ.get("KATIB_TRIAL_CHECKPOINT_DIR", "")


def _load_state(model, opt, st, flat: bool) -> bool:
    """Load a {"model", "optim", "step"} checkpoint into either implementation; the
    optimizer moments carry over only between like implementations."""
    model.load_state_dict(st["model"])
    o = st.get("optim")
    if flat and isinstance(o, dict) and "exp_avg" in o:
        model.load_optim_state(o)
        return True
    if not flat and isinstance(o, dict) and "state" in o:
        opt.load_state_dict(o)
        return True
    return False


def main(argv=None):
    args = parse_args(argv if argv is not None else [])
    dev = device()
    cuda = dev.type == "cuda"
    torch.manual_seed(args.seed)
    cfg = PRESETS[args.model]
    T = args.seq_len or cfg.ctx
    toks = markov_tokens(args.num_tokens, vocab=cfg.vocab, seed=99, dev=dev)
    n_train = int(len(toks) * 0.9)
    flat = (args.impl == "flat") or (args.impl == "auto" and cuda and hip_supported(cfg, T))
    if flat:
        ops = get_ops(args.ops if args.ops != "auto" else ("hip" if cuda else "torch"), dev)
        model = GPT2Flat(cfg, dev, ops, dtype=torch.bfloat16 if cuda else torch.float32, seed=args.seed)
        opt = None
    else:
        model = GPT(cfg).to(dev)
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr, betas=(0.9, 0.95), weight_decay=args.weight_decay,
                                fused=cuda, foreach=not cuda, capturable=cuda)
    start_step = 0
    ck = _ckpt_dir(args)
    source = "init"
    t_load = time.time()
    st = p2p_ckpt.fetch(ck, dev) if (ck and cuda and args.p2p) else None  # parent's weights, GPU to GPU
    if st is not None:
        source = "p2p"
    elif ck and os.path.exists(os.path.join(ck, "model.pt")):
        ost = torch.load(os.path.join(ck, "optim.pt"), map_location=dev, weights_only=True)
        st = {"model": torch.load(os.path.join(ck, "model.pt"), map_location=dev, weights_only=True),
              "optim": ost["optim"], "step": ost["step"]}
        source = "file"
    if st is not None:
        moments = _load_state(model, opt, st, flat)
        start_step = int(st["step"])
        nbytes = sum(t.numel() * t.element_size() for t in _tensors(st))
        report(checkpoint_source=source, checkpoint_load_seconds=time.time() - t_load,
               checkpoint_optimizer_state=int(moments), checkpoint_bytes=nbytes)
    B = args.batch_size
    offs = torch.zeros(B, dtype=torch.long, device=dev)
    ar = torch.arange(T + 1, device=dev)
    loss_buf = torch.zeros((), device=dev)

    def batch(o):
        w = toks[(o[:, None] + ar[None, :])]
        return w[:, :-1], w[:, 1:]

    if flat:
        def train_step():
            xb, yb = batch(offs)
            loss = model.forward_backward(xb, yb)
            model.optimizer_step(weight_decay=args.weight_decay, max_norm=1.0)
            loss_buf.copy_(loss.detach())
            return loss_buf

        def set_lr(v):
            model.lr_t.fill_(v)
    else:
        for g in opt.param_groups:  # the trial's (possibly perturbed) hyperparameters
            g["lr"] = args.lr
            g["weight_decay"] = args.weight_decay
        lr_t = torch.tensor(args.lr, device=dev) if cuda else args.lr
        if cuda:
            for g in opt.param_groups:
                g["lr"] = lr_t
        for p_ in model.parameters():
            p_.grad = torch.zeros_like(p_)

        def train_step():
            xb, yb = batch(offs)
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=cuda):
                logits = model(xb)
            loss = F.cross_entropy(logits.float().view(-1, cfg.vocab), yb.reshape(-1))
            opt.zero_grad(set_to_none=False)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
            loss_buf.copy_(loss.detach())
            return loss_buf

        def set_lr(v):
            if cuda:
                lr_t.fill_(v)
            else:
                for g in opt.param_groups:
                    g["lr"] = v

    # Only the flat model is graph-captured: replaying the nn.Module step (autocast + fused
    # capturable AdamW) from a graph diverges on ROCm, so that reference path stays eager.
    step = CapturedStep(train_step, enabled=bool(args.capture) and flat)
    gen = torch.Generator(device=dev).manual_seed(args.seed * 1000 + start_step)
    timer = Timer()
    steady = min(5, args.steps // 3)  # steps before this one include graph capture
    t_steady, elapsed = None, 0.0
    for i in range(args.steps):
        s = start_step + i
        if i == steady:
            if cuda:
                torch.cuda.synchronize()
            t_steady = Timer()
        set_lr(args.lr * min(1.0, (s + 1) / max(args.warmup, 1)))
        offs.copy_(torch.randint(0, n_train - T - 1, (B,), device=dev, generator=gen))
        step()
        if (i + 1) % 10 == 0 or i == args.steps - 1:
            report(step=s + 1, loss=float(loss_buf))
    elapsed = timer.elapsed()
    steady_s = t_steady.elapsed() if t_steady is not None else elapsed
    if not flat:
        model.eval()
    tot, correct, n = 0.0, 0.0, 0
    with torch.no_grad(), torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=cuda and not flat):
        eg = torch.Generator(device=dev).manual_seed(7)
        for _ in range(args.eval_batches):
            o = torch.randint(n_train, len(toks) - T - 1, (B,), device=dev, generator=eg)
            xb, yb = batch(o)
            if flat:  # one pass over the bf16 logits: loss + top-1 (HipOps.xent_eval)
                l_, c_ = model.ops.xent_eval(model.forward(xb), yb.reshape(-1), cfg.vocab)
                tot += float(l_)
                correct += float(c_)
            else:
                logits = model(xb).float()
                tot += float(F.cross_entropy(logits.view(-1, cfg.vocab), yb.reshape(-1), reduction="sum"))
                correct += float((logits.view(-1, cfg.vocab).argmax(-1) == yb.reshape(-1)).sum())
            n += yb.numel()
    if ck:
        os.makedirs(ck, exist_ok=True)
        end_step = start_step + args.steps
        optim_state = model.optim_state() if flat else opt.state_dict()
        if cuda and args.p2p:
            p2p_ckpt.publish({"model": model.state_dict(), "optim": optim_state, "step": end_step}, ck)
        if args.save_files:
            torch.save(model.state_dict(), os.path.join(ck, "model.pt"))
            torch.save({"optim": optim_state, "step": end_step}, os.path.join(ck, "optim.pt"))
    tokens_per_s = (args.steps - steady) * B * T / max(steady_s, 1e-9) if t_steady is not None else \
        args.steps * B * T / max(elapsed, 1e-9)
    report(**{"Validation-loss": tot / n, "Validation-accuracy": correct / n, "tokens_per_s": tokens_per_s})
    return tot / n


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
