"""GPT-2 as a flat-buffer functional network with a hand-written backward.

The PBT trial of BASELINE config 5 trains GPT-2 small (124M parameters). Instead of
autograd over ``nn.Module`` parameters (per-parameter gradient tensors, an extra
accumulate kernel per parameter, autocast re-casting every weight each forward), the
whole model lives in five flat buffers:

* ``p32``  fp32 master weights          * ``m``, ``v``  AdamW moments (fp32)
* ``w16``  bf16 shadow weights the GEMMs read (written by the AdamW kernel)
* ``g16``  bf16 gradients, every slice written exactly once per step by the backward

so one optimizer launch (global-norm clip + AdamW + bf16 cast) updates every parameter,
a checkpoint is five contiguous buffers (``state_dict``/``load_state_dict`` keep the
``nn.Module`` names of :class:`katib_amd.workloads.gpt2_pbt.GPT`), and the whole step
(forward, backward, optimizer) is one HIP-graph replay. Plain GEMMs go to hipBLASLt
(``torch.addmm``/``torch.mm`` with ``out=`` straight into the gradient slices); LayerNorm,
GELU, attention, cross-entropy and AdamW are the kernels of :mod:`katib_amd.ops.transformer`.

The residual stream is fp32 ([B*T, d]); its gradient is one fp32 buffer updated in
place through the whole backward. The tied LM head uses a vocabulary padded to a
multiple of 64 (50257 -> 50304) so logits rows are 16-byte aligned; pad rows of the
embedding stay zero and the cross-entropy kernels ignore the pad columns.

The reference's own trial images delegate all of this to framework autograd (e.g.
``examples/v1beta1/trial-images/pytorch-mnist/mnist.py:32-48``); GPT-2 is new scope from
BASELINE.json config 5.
"""

from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

# attn-proj / fc2 bias gradients summed by the LayerNorm backward that writes their output gradient
_LN_BIAS = True  # (module attribute; False: a separate column-sum pass per bias, as before)

from ..utils.tracing import gpu_range


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


@dataclass
class Spec:
    name: str
    shape: Tuple[int, ...]
    init: str  # normal | normal_proj | zeros | ones
    off: int = 0
    store_shape: Tuple[int, ...] = ()

    @property
    def numel(self) -> int:
        n = 1
        for s in self.store_shape or self.shape:
            n *= s
        return n


class GPT2Flat:
    def __init__(self, cfg, device, ops, dtype=torch.bfloat16, seed: int = 0):
        self.cfg = cfg
        self.device = torch.device(device)
        self.ops = ops
        self.dtype = dtype
        self.V = cfg.vocab
        self.Vp = (cfg.vocab + 63) // 64 * 64
        d = cfg.d
        specs: List[Spec] = [Spec("wte.weight", (cfg.vocab, d), "normal", store_shape=(self.Vp, d)),
                             Spec("wpe.weight", (cfg.ctx, d), "normal")]
        for i in range(cfg.n_layer):
            pre = "blocks.%d." % i
            specs += [Spec(pre + "ln1.weight", (d,), "ones"), Spec(pre + "ln1.bias", (d,), "zeros"),
                      Spec(pre + "qkv.weight", (3 * d, d), "normal"), Spec(pre + "qkv.bias", (3 * d,), "zeros"),
                      Spec(pre + "proj.weight", (d, d), "normal_proj"), Spec(pre + "proj.bias", (d,), "zeros"),
                      Spec(pre + "ln2.weight", (d,), "ones"), Spec(pre + "ln2.bias", (d,), "zeros"),
                      Spec(pre + "fc.weight", (4 * d, d), "normal"), Spec(pre + "fc.bias", (4 * d,), "zeros"),
                      Spec(pre + "fc2.weight", (d, 4 * d), "normal_proj"), Spec(pre + "fc2.bias", (d,), "zeros")]
        specs += [Spec("ln_f.weight", (d,), "ones"), Spec("ln_f.bias", (d,), "zeros")]
        off = 0
        for s in specs:
            s.off = off
            off += _pad8(s.numel)
        self.specs = {s.name: s for s in specs}
        self.order = [s.name for s in specs]
        self.P = off
        dev = self.device
        self.p32 = torch.zeros(off, device=dev, dtype=torch.float32)
        self.w16 = torch.zeros(off, device=dev, dtype=dtype)
        self.g16 = torch.zeros(off, device=dev, dtype=dtype)
        self.m = torch.zeros(off, device=dev, dtype=torch.float32)
        self.v = torch.zeros(off, device=dev, dtype=torch.float32)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.float32)
        self.lr_t = torch.full((1,), 3e-4, device=dev, dtype=torch.float32)
        self.sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        self.gscale = torch.ones(1, device=dev, dtype=torch.float32)
        self.p = {n: self._view(self.p32, n) for n in self.order}
        self.w = {n: self._view(self.w16, n) for n in self.order}
        self.g = {n: self._view(self.g16, n) for n in self.order}
        self._init(seed)

    # ---------------------------------------------------------------- parameters
    def _view(self, buf, name):
        s = self.specs[name]
        return buf[s.off:s.off + s.numel].view(s.store_shape or s.shape)

    def _init(self, seed):
        gen = torch.Generator(device="cpu").manual_seed(seed)
        std_proj = 0.02 / math.sqrt(2 * self.cfg.n_layer)
        for n in self.order:
            s = self.specs[n]
            if s.init == "ones":
                t = torch.ones(s.shape)
            elif s.init == "zeros":
                t = torch.zeros(s.shape)
            else:
                t = torch.randn(s.shape, generator=gen) * (0.02 if s.init == "normal" else std_proj)
            self.p[n][:s.shape[0]].copy_(t)
        self.w16.copy_(self.p32)

    def n_params(self) -> int:
        return sum(math.prod(self.specs[n].shape) for n in self.order if n != "wpe.weight")

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {n: self.p[n][:self.specs[n].shape[0]] for n in self.order}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        for n in self.order:
            s = self.specs[n]
            t = sd[n]
            if tuple(t.shape) != s.shape:
                raise ValueError("%s: checkpoint shape %s != model shape %s" % (n, tuple(t.shape), s.shape))
            self.p[n][:s.shape[0]].copy_(t)
        self.w16.copy_(self.p32)

    def optim_state(self) -> Dict[str, torch.Tensor]:
        return {"exp_avg": self.m, "exp_avg_sq": self.v, "step": self.step_t}

    def load_optim_state(self, st: Dict[str, torch.Tensor]):
        self.m.copy_(st["exp_avg"])
        self.v.copy_(st["exp_avg_sq"])
        self.step_t.copy_(st["step"].reshape(1))

    # ---------------------------------------------------------------- forward
    def _lin(self, x, name):
        return self.ops.linear(x, self.w[name + ".weight"], self.w[name + ".bias"])

    def _embed(self, idx):
        B, T = idx.shape
        x = F.embedding(idx.reshape(-1), self.w["wte.weight"]).float()
        return (x.view(B, T, -1) + self.w["wpe.weight"][:T].float()).view(B * T, -1)

    def forward(self, idx, save: bool = False):
        """Logits [B*T, Vp] (pad columns are zero-weight rows; ignore them)."""
        c, ops = self.cfg, self.ops
        B, T = idx.shape
        H = c.n_head
        resid = self._embed(idx)
        pending = None
        acts = []
        for i in range(c.n_layer):
            pre = "blocks.%d." % i
            sa, h1, mu1, rs1 = ops.ln_fwd(resid, pending, self.w[pre + "ln1.weight"], self.w[pre + "ln1.bias"])
            qkv = self._lin(h1, pre + "qkv")
            o, lse = ops.attn_fwd(qkv, B, T, H, c.d // H)
            a = self._lin(o, pre + "proj")
            sb, h2, mu2, rs2 = ops.ln_fwd(sa, a, self.w[pre + "ln2.weight"], self.w[pre + "ln2.bias"])
            u, gl = ops.linear_gelu(h2, self.w[pre + "fc.weight"], self.w[pre + "fc.bias"])  # GELU in the epilogue
            pending = self._lin(gl, pre + "fc2")
            resid = sb
            if save:
                acts.append((sa, h1, mu1, rs1, qkv, o, lse, sb, h2, mu2, rs2, u, gl))
        sf, hf, muf, rsf = ops.ln_fwd(resid, pending, self.w["ln_f.weight"], self.w["ln_f.bias"])
        logits = ops.linear(hf, self.w["wte.weight"], None)  # tied LM head
        if save:
            self._saved = (acts, sf, hf, muf, rsf)
        return logits

    # ---------------------------------------------------------------- training step
    def forward_backward(self, idx, tgt):
        """Mean next-token cross-entropy; fills every slice of ``g16``."""
        c, ops = self.cfg, self.ops
        B, T = idx.shape
        M, H, d = B * T, c.n_head, c.d
        tgt = tgt.reshape(-1)
        with gpu_range("gpt2.forward"):
            logits = self.forward(idx, save=True)
        return self._backward(idx, tgt, logits)

    def _backward(self, idx, tgt, logits):
        c, ops = self.cfg, self.ops
        B, T = idx.shape
        M, H, d = B * T, c.n_head, c.d
        with gpu_range("gpt2.backward"):
            return self._backward_body(idx, tgt, logits, B, T, M, H, d)

    def _backward_body(self, idx, tgt, logits, B, T, M, H, d):
        c, ops = self.cfg, self.ops
        acts, sf, hf, muf, rsf = self._saved
        self._saved = None
        # forward + backward of the cross-entropy in one pass over the logits (the gradient overwrites them)
        loss_rows, lse_ce, dlog = ops.xent_train(logits, tgt, self.gscale, self.V)
        # mean as a GEMV, not torch.mean: a single-output reduction over B*T rows takes
        # PyTorch's cross-workgroup path, which reads stale staging memory when replayed from a
        # HIP graph on this ROCm stack (katib_amd/utils/graphcheck.py)
        n = loss_rows.numel()
        loss = (loss_rows.view(1, n) @ torch.ones(n, 1, device=loss_rows.device, dtype=loss_rows.dtype)).view(()) / n
        g = self.g
        torch.mm(dlog.t(), hf, out=g["wte.weight"])  # tied LM head (pad rows get 0)
        dh = torch.mm(dlog, self.w["wte.weight"])
        del dlog, logits
        G = torch.empty((M, d), device=self.device, dtype=torch.float32)  # residual-stream gradient
        dr = torch.empty((M, d), device=self.device, dtype=self.dtype)
        # each LayerNorm backward also column-sums the dr it writes: the bias gradient of the linear layer
        # whose output gradient dr is (the top block's fc2 here, proj after ln2, the lower block's fc2 after ln1)
        lb = _LN_BIAS
        ops.ln_bwd(dh, sf, muf, rsf, self.w["ln_f.weight"], G, dr, g["ln_f.weight"], g["ln_f.bias"],
                   accumulate=False, dbias=g["blocks.%d.fc2.bias" % (c.n_layer - 1)] if lb else None)
        for i in reversed(range(c.n_layer)):
            pre = "blocks.%d." % i
            sa, h1, mu1, rs1, qkv, o, lse, sb, h2, mu2, rs2, u, gl = acts.pop()
            # MLP: dr is the gradient of fc2's output
            ops.wgrad(dr, gl, g[pre + "fc2.weight"])  # fc2.bias: summed by the LayerNorm backward that wrote dr
            if not lb:
                ops.colsum(dr, g[pre + "fc2.bias"])
            # GELU backward and the fc.bias column sums in the dgrad epilogue
            du = ops.dgrad_gelu(dr, self.w[pre + "fc2.weight"], u, g[pre + "fc.bias"])
            ops.wgrad(du, h2, g[pre + "fc.weight"])
            dh2 = ops.dgrad(du, self.w[pre + "fc.weight"])
            del du
            ops.ln_bwd(dh2, sb, mu2, rs2, self.w[pre + "ln2.weight"], G, dr, g[pre + "ln2.weight"],
                       g[pre + "ln2.bias"], dbias=g[pre + "proj.bias"] if lb else None)
            # attention: dr is now the gradient of proj's output
            ops.wgrad(dr, o, g[pre + "proj.weight"])
            if not lb:
                ops.colsum(dr, g[pre + "proj.bias"])
            do = ops.dgrad(dr, self.w[pre + "proj.weight"])
            dqkv = ops.attn_bwd(qkv, o, do, lse, B, T, H, d // H)
            ops.wgrad_bgrad(dqkv, h1, g[pre + "qkv.weight"], g[pre + "qkv.bias"])
            dh1 = ops.dgrad(dqkv, self.w[pre + "qkv.weight"])
            del dqkv
            ops.ln_bwd(dh1, sa, mu1, rs1, self.w[pre + "ln1.weight"], G, dr if i > 0 else None,
                       g[pre + "ln1.weight"], g[pre + "ln1.bias"],
                       dbias=g["blocks.%d.fc2.bias" % (i - 1)] if (i > 0 and lb) else None)
        # embeddings: G is the gradient of wte[idx] + wpe[:T]
        Gb = G.to(self.dtype)
        g["wte.weight"].index_add_(0, idx.reshape(-1), Gb)
        gw = g["wpe.weight"]
        torch.sum(Gb.view(B, T, d), 0, out=gw[:T])
        if T < gw.shape[0]:
            gw[T:].zero_()
        return loss

    def optimizer_step(self, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, max_norm=1.0):
        """AdamW on the flat buffers; ``lr_t`` (device scalar) is the learning rate."""
        self.step_t.add_(1.0)
        with gpu_range("gpt2.adamw"):
            self.ops.adamw(self.p32, self.g16, self.m, self.v, self.w16, self.lr_t, self.step_t, beta1, beta2, eps,
                           weight_decay, max_norm, self.sumsq)
