"""ENAS LSTM controller (reference ``pkg/suggestion/v1beta1/nas/enas/Controller.py:19-257``),
re-implemented in PyTorch.

Same parameterisation as the reference TF graph: ``w_lstm [2H, 4H]`` (i, f, o, g
gates, no bias), ``g_emb [1, H]``, ``w_emb [n_ops, H]``, ``w_soft [H, n_ops]`` and
skip attention ``w_1, w_2 [H, H]``, ``v [H, 1]``; uniform(-0.01, 0.01) init.
Sampling: per layer an op (categorical over temperature/tanh-scaled logits) then,
for layer > 0, one binary skip decision per previous layer from the attention
logits ``[-q, q]``. Training: REINFORCE ``loss = sum(logp) * (R - baseline)`` +
``skip_weight * mean(KL(skip || target))`` with an EMA baseline and Adam.

The controller is ~55k parameters: each sampling step is a chain of [1 x 2H] x
[2H x 4H] GEMVs - launch-latency bound on any GPU, so it runs on the host by
default (``device="cpu"``); the suggestion path therefore never competes with
trials for the MI355X.
"""

from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F


class EnasController(torch.nn.Module):
    def __init__(self, num_layers=12, num_operations=16, hidden_size=64, temperature: Optional[float] = 5.0,
                 tanh_const: Optional[float] = 2.25, entropy_weight: Optional[float] = 1e-5, baseline_decay=0.999,
                 learning_rate=5e-5, skip_target=0.4, skip_weight: Optional[float] = 0.8, seed: Optional[int] = None):
        super().__init__()
        self.num_layers = num_layers
        self.num_operations = num_operations
        self.H = hidden_size
        self.temperature = temperature
        self.tanh_const = tanh_const
        self.entropy_weight = entropy_weight
        self.baseline_decay = baseline_decay
        self.skip_target = skip_target
        self.skip_weight = skip_weight
        self.gen = torch.Generator()
        if seed is not None:
            self.gen.manual_seed(seed)
        H = hidden_size
        u = lambda *s: torch.nn.Parameter(torch.empty(*s).uniform_(-0.01, 0.01, generator=self.gen))
        self.w_lstm = u(2 * H, 4 * H)
        self.g_emb = u(1, H)
        self.w_emb = u(num_operations, H)
        self.w_soft = u(H, num_operations)
        self.attn_w_1 = u(H, H)
        self.attn_w_2 = u(H, H)
        self.attn_v = u(H, 1)
        self.register_buffer("baseline", torch.zeros(()))
        self.train_step = 0
        self.opt = torch.optim.Adam(self.parameters(), lr=learning_rate)

    @staticmethod
    def _lstm(x, c, h, w):
        ifog = torch.cat([x, h], dim=1) @ w
        i, f, o, g = ifog.chunk(4, dim=1)
        nc = torch.sigmoid(i) * torch.tanh(g) + torch.sigmoid(f) * c
        nh = torch.sigmoid(o) * torch.tanh(nc)
        return nc, nh

    def _shape_logits(self, logits):
        if self.temperature is not None:
            logits = logits / self.temperature
        if self.tanh_const is not None:
            logits = self.tanh_const * torch.tanh(logits)
        return logits

    def sample(self) -> Tuple[List[int], torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        """Returns (flat arc, sum log_prob, sum entropy, mean skip KL, skip count)."""
        H = self.H
        c = torch.zeros(1, H)
        h = torch.zeros(1, H)
        inputs = self.g_emb
        arc, logps, ents, kls = [], [], [], []
        skip_count = torch.zeros(())
        all_h, all_hw = [], []
        targets = torch.tensor([1.0 - self.skip_target, self.skip_target])
        for layer in range(self.num_layers):
            c, h = self._lstm(inputs, c, h, self.w_lstm)
            logits = self._shape_logits(h @ self.w_soft)
            op = torch.multinomial(F.softmax(logits, -1), 1, generator=self.gen).view(1)
            arc.append(int(op))
            lp = -F.cross_entropy(logits, op, reduction="sum")
            logps.append(lp)
            ents.append((-lp * torch.exp(lp)).detach())
            inputs = self.w_emb[op]
            c, h = self._lstm(inputs, c, h, self.w_lstm)
            if layer > 0:
                q = torch.tanh(h @ self.attn_w_2 + torch.cat(all_hw, 0)) @ self.attn_v  # [layer, 1]
                sl = self._shape_logits(torch.cat([-q, q], dim=1))  # [layer, 2]
                skip = torch.multinomial(F.softmax(sl, -1), 1, generator=self.gen).view(-1)
                arc.extend(int(s) for s in skip)
                sp = torch.sigmoid(sl)
                kls.append(torch.sum(sp * torch.log(sp / targets)))
                lps = -F.cross_entropy(sl, skip, reduction="none")
                logps.append(lps.sum())
                ents.append(torch.sum(-lps * torch.exp(lps)).detach())
                sf = skip.float().view(1, layer)
                skip_count = skip_count + sf.sum()
                inputs = (sf @ torch.cat(all_h, 0)) / (1.0 + sf.sum())
            else:
                inputs = self.g_emb
            all_h.append(h)
            all_hw.append(h @ self.attn_w_1)
        kl = torch.stack(kls).mean() if kls else torch.zeros(())
        return arc, torch.stack(logps).sum(), torch.stack(ents).sum(), kl, skip_count

    @torch.no_grad()
    def sample_arc(self) -> List[int]:
        return self.sample()[0]

    def train_once(self, reward: float):
        arc, logp, ent, kl, skip_count = self.sample()
        r = torch.tensor(float(reward))
        if self.entropy_weight is not None:
            r = r + self.entropy_weight * ent
        self.baseline -= (1 - self.baseline_decay) * (self.baseline - r.detach())
        loss = logp * (r.detach() - self.baseline)
        if self.skip_weight is not None:
            loss = loss + self.skip_weight * kl
        self.opt.zero_grad()
        loss.backward()
        gn = math.sqrt(sum(float((p.grad ** 2).sum()) for p in self.parameters() if p.grad is not None))
        self.opt.step()
        self.train_step += 1
        norm = self.num_layers * (self.num_layers - 1) / 2
        return {"loss": float(loss.detach()), "entropy": float(ent.detach()), "grad_norm": gn,
                "baseline": float(self.baseline),
                "skip_rate": float(skip_count) / norm if norm else 0.0}

    def state(self):
        return {"params": {k: v.detach().clone() for k, v in self.state_dict().items()},
                "opt": self.opt.state_dict(), "train_step": self.train_step}

    def load(self, st):
        self.load_state_dict(st["params"])
        self.opt.load_state_dict(st["opt"])
        self.train_step = st["train_step"]
