"""Transformer ops for the GPT-2 trial: two interchangeable backends.

* :class:`HipOps`   - the hand-written gfx950 kernels of ``csrc/hip/transformer.hip``
  (fused residual-add LayerNorm, tanh GELU, vocabulary cross-entropy with the gradient
  written in place, flat AdamW with global-norm clipping that emits the bf16 shadow
  weights, causal flash attention forward/backward on MFMA). bf16 activations, fp32
  residual stream and statistics.
* :class:`TorchOps` - plain PyTorch implementations of exactly the same contracts
  (any dtype, any device); the numerical oracle for the HIP kernels and the CPU path.

Contracts (``M`` rows, ``D`` features, ``Vp`` padded vocabulary of which ``V`` are real):

``ln_fwd(x32, r, gamma, beta) -> (xin, y, mean, rstd)``
    ``xin = x32 + r`` (fp32; ``x32`` itself when ``r`` is None), ``y = LN(xin)``.
``ln_bwd(dy, xin, mean, rstd, gamma, G, dr, dgamma, dbeta)``
    ``G += LN'(dy)`` in place (``G`` fp32 residual-stream gradient; ``G`` is *set* when
    ``accumulate=False``), ``dr[:] = G`` cast to the activation dtype when ``dr`` is given,
    ``dgamma/dbeta`` written.
``attn_fwd(qkv, B, T, H) -> (o, lse)``
    causal softmax attention with head dim 64; ``qkv`` is ``[B*T, 3*H*64]`` (q | k | v, heads
    contiguous), ``o`` is ``[B*T, H*64]``, ``lse`` ``[B, H, T]`` = log2-sum-exp2 of the
    scaled scores (in log2 units).
``xent_fwd(logits, tgt, V) -> (loss_rows, lse)``; ``xent_bwd(logits, tgt, lse, gscale, V)``
    writes ``(softmax - onehot) * gscale / N`` over ``logits`` in place.
"""

from __future__ import annotations

import importlib
import math
import os

import torch

from .. import _hipload
import torch.nn.functional as F

LOG2E = 1.4426950408889634


def _kern():
    try:
        return _hipload.hipkern()
    except ImportError as e:
        raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)


# Kernel choices of the GPT-2 step are fixed by measurement, not switched by the environment:
# * one-pass training cross-entropy (xent_fused_k): 783k -> 793k tokens/s against xent_fwd + xent_bwd
#   (profiles/gpt2_xent_fused_ab_r05.log);
# * the fc2 input gradient with the GELU backward in its epilogue (gemm_lt gelu_u): +1.3 % tokens/s
#   against hipBLASLt dgrad + gelu_bwd (profiles/gpt2_gelu_dgrad_ab_r05.log);
# * measured and removed: hipBLASLt's BGRADB weight + bias gradient epilogue (782k -> 743k tokens/s,
#   profiles/lt_epilogue_r05.log) and the fc1 bias gradient from the dgrad epilogue (neutral,
#   profiles/gpt2_gelu_dgrad_bias_ab_r05.log).


class TorchOps:
    name = "torch"

    def __init__(self, eps: float = 1e-5):
        self.eps = eps

    # ---------------------------------------------------------------- LayerNorm
    def ln_fwd(self, x32, r, gamma, beta):
        xin = x32 if r is None else x32 + r.float()
        mean = xin.mean(-1)
        var = ((xin - mean[:, None]) ** 2).mean(-1)
        rstd = torch.rsqrt(var + self.eps)
        y = ((xin - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()).to(gamma.dtype)
        return xin, y, mean, rstd

    def ln_bwd(self, dy, xin, mean, rstd, gamma, G, dr, dgamma, dbeta, accumulate=True, dbias=None):
        D = xin.shape[-1]
        g = dy.float()
        xh = (xin - mean[:, None]) * rstd[:, None]
        dxh = g * gamma.float()
        dx = rstd[:, None] * (dxh - dxh.sum(-1, keepdim=True) / D - xh * (dxh * xh).sum(-1, keepdim=True) / D)
        if accumulate:
            G.add_(dx)
        else:
            G.copy_(dx)
        if dr is not None:
            dr.copy_(G)
        dgamma.copy_((g * xh).sum(0))
        dbeta.copy_(g.sum(0))
        if dbias is not None and dr is not None:
            dbias.copy_(dr.float().sum(0))

    # ---------------------------------------------------------------- GELU
    def gelu_fwd(self, u):
        return F.gelu(u.float(), approximate="tanh").to(u.dtype)

    def gelu_bwd(self, u, dy):
        x = u.float()
        k0, k1 = math.sqrt(2.0 / math.pi), 0.044715
        t = torch.tanh(k0 * (x + k1 * x ** 3))
        d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
        return (dy.float() * d).to(u.dtype)

    # ---------------------------------------------------------------- attention
    def attn_fwd(self, qkv, B, T, H, hd=64):
        q, k, v = qkv.float().view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
        mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
        lse = torch.logsumexp(s, -1)
        o = torch.softmax(s, -1) @ v
        return o.permute(0, 2, 1, 3).reshape(B * T, H * hd).to(qkv.dtype), lse * LOG2E

    def attn_bwd(self, qkv, o, dout, lse, B, T, H, hd=64):
        with torch.enable_grad():
            x = qkv.detach().float().requires_grad_(True)
            q, k, v = x.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
            s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
            mask = torch.ones(T, T, dtype=torch.bool, device=qkv.device).triu(1)
            p = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
            out = (p @ v).permute(0, 2, 1, 3).reshape(B * T, H * hd)
            (g,) = torch.autograd.grad(out, x, dout.float())
        return g.to(qkv.dtype)

    # ---------------------------------------------------------------- cross-entropy
    def xent_fwd(self, logits, tgt, V):
        x = logits[:, :V].float()
        lse = torch.logsumexp(x, -1)
        return lse - x.gather(1, tgt[:, None])[:, 0], lse

    def xent_bwd(self, logits, tgt, lse, gscale, V):
        N = logits.shape[0]
        p = torch.exp(logits[:, :V].float() - lse[:, None])
        p[torch.arange(N, device=logits.device), tgt] -= 1.0
        logits[:, :V] = (p * (gscale.float() / N)).to(logits.dtype)
        logits[:, V:] = 0
        return logits

    def xent_train(self, logits, tgt, gscale, V):
        loss, lse = self.xent_fwd(logits, tgt, V)
        return loss, lse, self.xent_bwd(logits, tgt, lse, gscale, V)

    def xent_eval(self, logits, tgt, V):
        """(summed loss, top-1 hits) over the rows: the validation metric (0-d fp32 tensors)."""
        x = logits[:, :V].float()
        return F.cross_entropy(x, tgt, reduction="sum"), (x.argmax(-1) == tgt).sum().float()

    # ---------------------------------------------------------------- GEMM helpers
    def linear(self, x, w, b):
        """x [M, K] . w[N, K]^T (+ b)."""
        return torch.addmm(b, x, w.t()) if b is not None else torch.mm(x, w.t())

    def linear_gelu(self, x, w, b):
        """(u, gelu_tanh(u)) with u = x . w^T + b."""
        u = self.linear(x, w, b)
        return u, self.gelu_fwd(u)

    def colsum(self, x, out):
        torch.sum(x, 0, out=out)

    def wgrad_bgrad(self, dy, x, dw, db):
        """dw = dy^T x; db = column sums of dy (a linear layer's weight + bias gradients)."""
        self.wgrad(dy, x, dw)
        self.colsum(dy, db)

    def dgrad_gelu(self, dy, w, u, db=None):
        """(dy @ w) * gelu_tanh'(u): the MLP's fc2 input gradient taken back through the GELU;
        ``db``: also its column sums (the fc1 bias gradient)."""
        du = self.gelu_bwd(u, self.dgrad(dy, w))
        if db is not None:
            self.colsum(du, db)
        return du

    def dgrad(self, dy, w):
        return torch.mm(dy, w)

    def wgrad(self, dy, x, out):
        torch.mm(dy.t(), x, out=out)

    # ---------------------------------------------------------------- optimizer
    def adamw(self, p, g, m, v, w16, lr, step, b1, b2, eps, wd, max_norm, sumsq):
        gf = g.float()
        sumsq.copy_((gf * gf).sum().reshape(1))
        if max_norm > 0:
            gf = gf * torch.clamp(max_norm / (sumsq.sqrt() + 1e-6), max=1.0)
        t = step.float()
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        m.mul_(b1).add_(gf, alpha=1 - b1)
        v.mul_(b2).addcmul_(gf, gf, value=1 - b2)
        p.mul_(1 - lr * wd)
        p.sub_(lr / bc1 * m / (v.sqrt() / bc2.sqrt() + eps))
        w16.copy_(p)


class HipOps:
    """The gfx950 kernels. Raises at construction if the extension is missing."""

    name = "hip"

    def __init__(self, eps: float = 1e-5, gemm: str = "auto", gemm_bwd: str = "auto"):
        self.k = _kern()
        self.eps = eps
        self._bmm_f32 = True
        # forward projections on the hand-written MFMA GEMM (gemm_bf16.hip, bias / GELU fused into the
        # epilogue) for the shapes where it measured faster than hipBLASLt on MI355X, hipBLASLt
        # (torch.addmm) for the rest (profiles/gemm_bf16_r03.log: at M = 8192 the 128x128-tile kernel
        # wins the d x d projection 1.23-1.37x and loses qkv 0.87x, fc + GELU 0.96x, fc2 0.80x, the LM
        # head 0.61x). gemm="all": every supported shape (tests), "0": hipBLASLt only; gemm_bwd likewise
        # for the backward GEMMs.
        self.gemm = gemm
        self.gemm_bwd = gemm_bwd

    # (N, K) classes where gemm_bf16 beat hipBLASLt in the measured table
    GEMM_WINS = {(768, 768), (256, 256), (512, 512), (1024, 1024)}

    def _gemm_ok(self, x, w):
        if self.gemm in ("0", "off") or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.dim() != 2:
            return False
        if self.gemm != "all" and (w.shape[0], w.shape[1]) not in self.GEMM_WINS:
            return False
        return x.is_contiguous() and w.is_contiguous() and bool(self.k.gemm_nt_supported(x.shape[0], w.shape[0],
                                                                                        x.shape[1]))

    def linear(self, x, w, b):
        if not self._gemm_ok(x, w):
            return torch.addmm(b, x, w.t()) if b is not None else torch.mm(x, w.t())
        c = torch.empty((x.shape[0], w.shape[0]), device=x.device, dtype=torch.bfloat16)
        self.k.gemm_nt(x, w, b, c, None)
        return c

    def linear_gelu(self, x, w, b):
        if not self._gemm_ok(x, w):
            u = torch.addmm(b, x, w.t())
            return u, self.gelu_fwd(u)
        u = torch.empty((x.shape[0], w.shape[0]), device=x.device, dtype=torch.bfloat16)
        g = torch.empty_like(u)
        self.k.gemm_nt(x, w, b, u, g)
        return u, g

    def ln_fwd(self, x32, r, gamma, beta):
        M, D = x32.shape
        xin = x32 if r is None else torch.empty_like(x32)
        y = torch.empty((M, D), device=x32.device, dtype=torch.bfloat16)
        mean = torch.empty(M, device=x32.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        self.k.ln_fwd(x32, r, None if r is None else xin, gamma, beta, y, mean, rstd, self.eps)
        return xin, y, mean, rstd

    def ln_bwd(self, dy, xin, mean, rstd, gamma, G, dr, dgamma, dbeta, accumulate=True, dbias=None):
        """``dbias``: also the bias gradient of the linear layer whose output gradient ``dr`` is
        (column sums of dr, accumulated by the same kernel instead of a colsum pass)."""
        M, D = xin.shape
        nb = self.k.ln_bwd_blocks(M)
        want = dbias is not None and dr is not None
        part = torch.empty((3 if want else 2, nb, D), device=xin.device, dtype=torch.float32)
        self.k.ln_bwd(dy, xin, mean, rstd, gamma, G if accumulate else None, G, dr, part[0], part[1],
                      part[2] if want else None)
        self.k.ln_reduce(part[0], part[1], dgamma, dbeta, part[2] if want else None, dbias if want else None)

    def gelu_fwd(self, u):
        g = torch.empty_like(u)
        self.k.gelu_fwd(u, g)
        return g

    def gelu_bwd(self, u, dy):
        du = torch.empty_like(u)
        self.k.gelu_bwd(u, dy, du)
        return du

    def dgrad_gelu(self, dy, w, u, db=None):
        """(dy @ w) * gelu_tanh'(u) in one launch: the NN dgrad kernel (gemm_lt) with the GELU backward in
        its epilogue (reads u where it writes the gradient) - against hipBLASLt's dgrad + the gelu_bwd
        pass, which writes the gradient, then re-reads it with u and writes it again. ``db`` (the fc1
        bias gradient): one colsum pass over the result."""
        M, N = dy.shape
        K = w.shape[1]
        if (self._bwd_mode() != "0" and self._lt_ok(dy, w, u) and u.shape == (M, K)
                and M % 128 == 0 and K % 128 == 0 and N % 64 == 0):
            out = torch.empty((M, K), device=dy.device, dtype=torch.bfloat16)
            self.k.gemm_lt(dy, False, w, True, None, out, 1, u)
            if db is not None:
                self.colsum(out, db)
            return out
        du = self.gelu_bwd(u, self.dgrad(dy, w))
        if db is not None:
            self.colsum(du, db)
        return du

    def wgrad_bgrad(self, dy, x, dw, db):
        """dw = dy^T x and db = column sums of dy (a linear layer's weight + bias gradients)."""
        self.wgrad(dy, x, dw)
        self.colsum(dy, db)

    def attn_fwd(self, qkv, B, T, H, hd=64):
        assert hd == 64
        o = torch.empty((B * T, H * hd), device=qkv.device, dtype=torch.bfloat16)
        lse = torch.empty((B, H, T), device=qkv.device, dtype=torch.float32)
        self.k.attn_fwd(qkv, o, lse, B, T, H, 1.0 / math.sqrt(hd))
        return o, lse

    def attn_bwd(self, qkv, o, dout, lse, B, T, H, hd=64):
        dqkv = torch.empty_like(qkv)
        delta = torch.empty_like(lse)
        self.k.attn_bwd(qkv, o, dout, lse, delta, dqkv, B, T, H, 1.0 / math.sqrt(hd))
        return dqkv

    def xent_fwd(self, logits, tgt, V):
        N = logits.shape[0]
        loss = torch.empty(N, device=logits.device, dtype=torch.float32)
        lse = torch.empty_like(loss)
        self.k.xent_fwd(logits, tgt, loss, lse, V)
        return loss, lse

    def xent_bwd(self, logits, tgt, lse, gscale, V):
        self.k.xent_bwd(logits, tgt, lse, gscale, 1.0 / logits.shape[0], V)
        return logits

    def xent_train(self, logits, tgt, gscale, V):
        """(loss_rows, lse, dlogits): forward + backward in one read of the logits (the gradient
        overwrites them); falls back to the two-pass kernels for rows wider than 53248."""
        N = logits.shape[0]
        loss = torch.empty(N, device=logits.device, dtype=torch.float32)
        lse = torch.empty_like(loss)
        if not self.k.xent_fused(logits, tgt, loss, lse, gscale, 1.0 / N, V):
            self.k.xent_fwd(logits, tgt, loss, lse, V)
            self.k.xent_bwd(logits, tgt, lse, gscale, 1.0 / N, V)
        return loss, lse, logits

    def xent_eval(self, logits, tgt, V):
        """(summed loss, top-1 hits) in one pass over the bf16 logits (xent_eval_k): no fp32 copy of the
        logits, no softmax / argmax framework kernels on the PBT member's validation path."""
        N = logits.shape[0]
        out = torch.empty((2, -(-N // 4) * 4), device=logits.device, dtype=torch.float32)  # 16-byte aligned rows
        self.k.xent_eval(logits, tgt, out[0, :N], out[1, :N], V)
        s = out[:, :N].sum(1)
        return s[0], s[1]

    def colsum(self, x, out):
        """Bias gradient: bf16 column sums of [M, N] (two-stage, fp32 partials)."""
        self.k.colsum(x, out)

    # Backward GEMMs on the layout-native kernel (gemm_lt: dgrad NN, wgrad TN, no transposed
    # copies; profiles/gemm_fwd_bwd_table_r05.log, MI355X, median of 5 interleaved rounds, 16k
    # tokens = the PBT member's batch). Against the best hipBLASLt form (split-K batched fp32 +
    # row sum for wgrad, the strided mm for dgrad) the 128^2 two-stage tile (~600-800 TF/s) wins
    # only the qkv wgrad (1.07x); hipBLASLt's 192x256 / 256x256 tiles reach ~1 PF/s on the rest.
    # The d x d dgrad wins at 8k tokens (1.19x). gemm_bwd="0": hipBLASLt for all, "all": gemm_lt
    # wherever supported (tests).
    WGRAD_SPLIT = {(2304, 768): 4}  # (out, in) -> split-K
    DGRAD_WINS = {(768, 768)}  # (out, in) classes of W where the NN kernel won (at <= 8k tokens)

    def _bwd_mode(self):
        return self.gemm_bwd

    def _lt_ok(self, *ts):
        return all(t.dtype == torch.bfloat16 and t.dim() == 2 and t.is_contiguous() for t in ts)

    def dgrad(self, dy, w):
        """``dy @ w`` ([M, K] from dy [M, N], w [N, K]): the NN GEMM where it wins, else hipBLASLt."""
        M, N = dy.shape
        K = w.shape[1]
        mode = self._bwd_mode()
        use = mode == "all" or (mode == "auto" and (N, K) in self.DGRAD_WINS and M <= 8192)
        if use and mode != "0" and self._lt_ok(dy, w) and M % 128 == 0 and K % 128 == 0 and N % 64 == 0:
            out = torch.empty((M, K), device=dy.device, dtype=torch.bfloat16)
            self.k.gemm_lt(dy, False, w, True, None, out)
            return out
        return torch.mm(dy, w)

    def wgrad(self, dy, x, out):
        """``out = dy^T x`` ([N, K] from [M, N], [M, K]). The reduction over M = B*T tokens is
        long and the output small (768 x 768 = 36 tiles of 128^2 for the attention
        projection), so it is split S ways: the layout-native TN kernel (gemm_lt) writes one fp32
        slab per K slice and one row-sum launch adds them into the bf16 gradient."""
        M, N = dy.shape
        K = x.shape[1]
        mode = self._bwd_mode()
        S = self.WGRAD_SPLIT.get((N, K)) if mode == "auto" else (8 if mode == "all" else None)
        if S is not None and self._lt_ok(dy, x) and out.is_contiguous() and N % 128 == 0 and K % 128 == 0:
            while S > 1 and M % (64 * S):
                S //= 2
            if M % 64 == 0:
                if S == 1:
                    self.k.gemm_lt(dy, True, x, True, None, out)
                    return
                part = torch.empty((S, N, K), device=dy.device, dtype=torch.float32)
                self.k.gemm_lt(dy, True, x, True, None, part, S)
                self.k.reduce_rows(part.view(S, N * K), out.view(-1))
                return
        tiles = -(-N // 128) * -(-K // 128)
        S = 1
        while tiles * S < 512 and M % (2 * S) == 0 and M // (2 * S) >= 1024:
            S *= 2
        if S == 1 or not self._bmm_f32:
            torch.mm(dy.t(), x, out=out)
            return
        try:
            part = torch.bmm(dy.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, K), out_dtype=torch.float32)
        except (RuntimeError, TypeError, NotImplementedError):
            self._bmm_f32 = False  # this stack's bmm has no fp32-output bf16 path
            torch.mm(dy.t(), x, out=out)
            return
        self.k.reduce_rows(part.view(S, N * K), out.view(-1))

    def adamw(self, p, g, m, v, w16, lr, step, b1, b2, eps, wd, max_norm, sumsq):
        sumsq.zero_()
        self.k.grad_sumsq(g, sumsq)
        self.k.adamw(p, g, m, v, w16, lr, step, b1, b2, eps, wd, sumsq, max_norm)


def get_ops(name: str = "auto", device=None):
    """``hip`` (fails loudly without the extension), ``torch``, or ``auto`` (hip on a GPU)."""
    if name == "auto":
        name = "hip" if (device is not None and torch.device(device).type == "cuda") else "torch"
    if name == "hip":
        return HipOps()
    if name == "torch":
        return TorchOps()
    raise ValueError("unknown transformer ops backend %r" % name)
