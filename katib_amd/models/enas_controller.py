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
[2H x 4H] GEMVs, hundreds of dependent tiny ops per arc. As PyTorch ops that is
launch-latency bound on any GPU, so this module (:class:`EnasController`) runs on
the host and serves as the numerics oracle. On MI355X the service uses
:class:`EnasControllerHip`: the whole controller - sampling, BPTT, Adam, all
``controller_train_steps`` REINFORCE steps - is ONE persistent-workgroup HIP launch
(``csrc/hip/enas_ctrl.hip``), and the arcs of a GetSuggestions call are one more
launch with a workgroup per arc.

REINFORCE loss as in the reference (``Controller.py:200-222``):
``loss = sum(CE of the sampled actions) * (R - baseline) + skip_weight * mean(KL)``,
where CE = -log p, so minimising it raises the log-probability of arcs whose reward
beats the baseline.
"""

from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence, Tuple

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

    def sample(self, forced: Optional[Sequence[int]] = None
               ) -> Tuple[List[int], torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        """Returns (flat arc, sum log_prob, sum entropy, mean skip KL, skip count).
        ``forced`` replays a given flat arc instead of drawing one (gradient checks)."""
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
            pos = len(arc)
            if forced is not None:
                op = torch.tensor([int(forced[pos])])
            else:
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
                if forced is not None:
                    skip = torch.tensor([int(v) for v in forced[len(arc):len(arc) + layer]])
                else:
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

    def train_once(self, reward: float, forced: Optional[Sequence[int]] = None):
        arc, logp, ent, kl, skip_count = self.sample(forced)
        r = torch.tensor(float(reward))
        if self.entropy_weight is not None:
            r = r + self.entropy_weight * ent
        self.baseline -= (1 - self.baseline_decay) * (self.baseline - r.detach())
        loss = -logp * (r.detach() - self.baseline)  # sum of CE (= -log p) times the advantage
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

    def train(self, reward: float, steps: int, log_every: int = 0) -> List[dict]:
        """``steps`` REINFORCE steps at a fixed reward; returns the log of every
        ``log_every``-th step (service.py:311-334 loop)."""
        logs = []
        for step in range(1, steps + 1):
            log = self.train_once(reward)
            if log_every and step % log_every == 0:
                logs.append(log)
        return logs

    def sample_arcs(self, n: int) -> List[List[int]]:
        return [self.sample_arc() for _ in range(n)]

    def named_flat(self) -> dict:
        return {k: v.detach() for k, v in self.named_parameters()}

    def state(self):
        return {"params": {k: v.detach().clone() for k, v in self.state_dict().items()},
                "opt": self.opt.state_dict(), "train_step": self.train_step}

    def load(self, st):
        self.load_state_dict(st["params"])
        self.opt.load_state_dict(st["opt"])
        self.train_step = st["train_step"]


PARAM_ORDER = ("w_lstm", "g_emb", "w_emb", "w_soft", "attn_w_1", "attn_w_2", "attn_v")


class EnasControllerHip(EnasController):
    """The same controller on MI355X through the persistent-workgroup HIP kernel.

    Parameters (same init stream as :class:`EnasController`), Adam moments and the
    baseline live on the GPU in flat buffers laid out as the kernel expects
    (``PARAM_ORDER``, row-major). ``train`` runs all its REINFORCE steps in one launch;
    ``sample_arcs(n)`` draws n arcs in one launch (one workgroup per arc). Sampling uses
    a counter-based RNG (seed, call counter), so arcs differ from the torch backend's
    draws for the same seed; with ``forced`` arcs both backends compute the same losses,
    gradients and updates (tests/test_gpu_enas.py).
    """

    def __init__(self, *args, device=None, **kw):
        super().__init__(*args, **kw)
        import importlib

        self._K = importlib.import_module("katib_amd._hipkern")  # raises if the extension is not built
        K = self._K
        # every kernel limit is checked here, at construction, so make_controller("auto") can
        # fall back to the torch controller instead of failing later in enas_sample/enas_train
        if self.H > min(64, getattr(K, "ENAS_MAX_H", 64)):
            raise ValueError("the HIP ENAS controller supports controller_hidden_size <= 64")
        if not 1 <= self.num_operations <= getattr(K, "ENAS_MAX_OPS", 1024):
            raise ValueError("the HIP ENAS controller supports at most %d operations" % K.ENAS_MAX_OPS)
        if not 1 <= self.num_layers <= getattr(K, "ENAS_MAX_LAYERS", 64):
            raise ValueError("the HIP ENAS controller supports at most %d layers" % K.ENAS_MAX_LAYERS)
        if K.enas_lds_bytes(self.H, self.num_operations, self.num_layers) > getattr(K, "ENAS_LDS_LIMIT", 160 * 1024):
            raise ValueError("the ENAS controller does not fit the 160 KB LDS of one CU")
        self.device = torch.device(device or "cuda")
        params = dict(self.named_parameters())
        self.flat = torch.cat([params[n].detach().reshape(-1) for n in PARAM_ORDER]).to(self.device).contiguous()
        n = self.flat.numel()
        assert n == self._K.enas_n_params(self.H, self.num_operations)
        self.m = torch.zeros(n, device=self.device)
        self.v = torch.zeros(n, device=self.device)
        self.g = torch.zeros(n, device=self.device)
        self.base_t = torch.zeros(1, device=self.device)
        self.arc_len = self.num_layers * (self.num_layers + 1) // 2
        self.tape_floats = int(self._K.enas_tape_floats(self.H, self.num_operations, self.num_layers))
        self._tape = torch.empty(0, device=self.device)
        self.adam_t = 0
        self.rng_offset = 0
        seed = kw.get("seed")
        self.rng_seed = int(seed) if seed is not None else int.from_bytes(os.urandom(7), "little")
        self.cfg = {"temperature": self.temperature, "tanh_const": self.tanh_const,
                    "entropy_weight": self.entropy_weight, "skip_weight": self.skip_weight,
                    "skip_target": float(self.skip_target), "baseline_decay": float(self.baseline_decay),
                    "lr": float(self.opt.defaults["lr"]), "beta1": 0.9, "beta2": 0.999, "eps": 1e-8}

    def _tape_for(self, blocks):
        need = blocks * self.tape_floats
        if self._tape.numel() < need:
            self._tape = torch.empty(need, device=self.device)
        return self._tape

    def sample_arcs(self, n: int, forced: Optional[Sequence[int]] = None) -> List[List[int]]:
        arcs = torch.empty(n, self.arc_len, dtype=torch.int32, device=self.device)
        f = None if forced is None else torch.tensor(list(forced), dtype=torch.int32, device=self.device)
        self._K.enas_sample(self.flat, arcs, self._tape_for(n), self.num_layers, self.num_operations, self.H, self.cfg,
                            self.rng_seed, self.rng_offset, f)
        self.rng_offset += n
        return arcs.cpu().tolist()

    @torch.no_grad()
    def sample_arc(self) -> List[int]:
        return self.sample_arcs(1)[0]

    def train_steps(self, reward: float, steps: int, forced: Optional[Sequence[int]] = None):
        """``steps`` REINFORCE steps in ONE kernel launch; returns (logs [steps, 8], arcs)."""
        arcs = torch.empty(steps, self.arc_len, dtype=torch.int32, device=self.device)
        logs = torch.empty(steps, self._K.ENAS_LOG_FIELDS, device=self.device)
        f = None if forced is None else torch.tensor(list(forced), dtype=torch.int32, device=self.device)
        self._K.enas_train(self.flat, self.m, self.v, self.g, self._tape_for(1), arcs, logs, self.base_t,
                           self.num_layers, self.num_operations, self.H, self.cfg, float(reward), steps, self.adam_t,
                           self.rng_seed, self.rng_offset, f)
        self.adam_t += steps
        self.rng_offset += steps
        self.train_step += steps
        return logs.cpu(), arcs.cpu()

    def train_once(self, reward: float, forced: Optional[Sequence[int]] = None):
        return self._log_dict(self.train_steps(reward, 1, forced)[0][0])

    def train(self, reward: float, steps: int, log_every: int = 0) -> List[dict]:
        logs, _ = self.train_steps(reward, steps)
        if not log_every:
            return []
        return [self._log_dict(logs[i - 1]) for i in range(log_every, steps + 1, log_every)]

    @staticmethod
    def _log_dict(row):
        return {"loss": float(row[0]), "entropy": float(row[1]), "grad_norm": float(row[2]),
                "baseline": float(row[3]), "skip_rate": float(row[4])}

    def named_flat(self) -> dict:
        out, off = {}, 0
        params = dict(self.named_parameters())
        for n in PARAM_ORDER:
            k = params[n].numel()
            out[n] = self.flat[off:off + k].view(params[n].shape)
            off += k
        return out

    def state(self):
        return {"backend": "hip", "flat": self.flat.cpu(), "m": self.m.cpu(), "v": self.v.cpu(),
                "baseline": float(self.base_t), "adam_t": self.adam_t, "rng_seed": self.rng_seed,
                "rng_offset": self.rng_offset, "train_step": self.train_step}

    def load(self, st):
        if st.get("backend") != "hip":
            super().load(st)
            params = dict(self.named_parameters())
            self.flat.copy_(torch.cat([params[n].detach().reshape(-1) for n in PARAM_ORDER]))
            return
        self.flat.copy_(st["flat"])
        self.m.copy_(st["m"])
        self.v.copy_(st["v"])
        self.base_t.fill_(st["baseline"])
        self.adam_t, self.rng_seed = st["adam_t"], st["rng_seed"]
        self.rng_offset, self.train_step = st["rng_offset"], st["train_step"]


def make_controller(backend: Optional[str] = None, **kw) -> EnasController:
    """``backend``: "hip" (MI355X kernel), "torch" (host oracle) or "auto" (default, env
    ``KATIB_AMD_ENAS_BACKEND``): the HIP kernel when a GPU and the extension are present and
    the search space fits its limits (operations, layers, 160 KB LDS).

    The controller runs on the scheduler's current GPU (cuda:0 unless the scheduler process
    is pinned): GetSuggestions shares that GPU with whatever trial is placed on it, for the
    ~16 ms of one ENAS suggestion call (50 REINFORCE steps in one workgroup). Set
    ``KATIB_AMD_ENAS_BACKEND=torch`` to keep the scheduler off the GPU entirely."""
    backend = (backend or os.environ.get("KATIB_AMD_ENAS_BACKEND", "auto")).lower()
    if backend == "torch":
        return EnasController(**kw)
    if backend == "hip":
        return EnasControllerHip(**kw)
    if torch.cuda.is_available() and kw.get("hidden_size", 64) <= 64:
        try:
            return EnasControllerHip(**kw)
        except (ImportError, OSError, ValueError):  # no extension, or a kernel limit is exceeded
            pass
    return EnasController(**kw)
