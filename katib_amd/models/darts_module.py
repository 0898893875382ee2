"""Reference-shaped DARTS supernet: a conventional ``nn.Module`` tree trained eagerly with
autograd - the structure of the reference trial image (``examples/v1beta1/trial-images/
darts-cnn-cifar10``: primitives ``operations.py:18-180``, cells / network ``model.py:21-194``,
second-order architect ``architect.py:19-135``, train step ``run_trial.py:185-207``), written
independently for two uses:

* the numerics oracle of ``tests/test_darts_parity.py`` (the flat-buffer functional network of
  :mod:`katib_amd.models.darts_search` must reproduce it), and
* the same-GPU comparator ``module_eager_ms_per_step`` of ``bench.py``: what a reference-shaped
  trainer (module tree, per-op framework kernels, eager autograd) costs per search step here.
"""

from __future__ import annotations

import copy

import torch
import torch.nn as nn
import torch.nn.functional as F


class _Zero(nn.Module):
    def __init__(self, stride):
        super().__init__()
        self.stride = stride

    def forward(self, x):
        return x[:, :, ::self.stride, ::self.stride] * 0.0


class _PoolBN(nn.Module):
    def __init__(self, kind, c, stride):
        super().__init__()
        self.pool = (nn.AvgPool2d(3, stride, 1, count_include_pad=False) if kind == "avg"
                     else nn.MaxPool2d(3, stride, 1))
        self.bn = nn.BatchNorm2d(c, affine=False)

    def forward(self, x):
        return self.bn(self.pool(x))


class _FR(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout // 2, 1, 2, bias=False)
        self.conv2 = nn.Conv2d(cin, cout // 2, 1, 2, bias=False)
        self.bn = nn.BatchNorm2d(cout, affine=False)

    def forward(self, x):
        x = F.relu(x)
        return self.bn(torch.cat([self.conv1(x), self.conv2(x[:, :, 1:, 1:])], 1))


class _Std(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, 1, bias=False)
        self.bn = nn.BatchNorm2d(cout, affine=False)

    def forward(self, x):
        return self.bn(self.conv(F.relu(x)))


class _DW(nn.Module):
    def __init__(self, c, k, stride, pad, dil):
        super().__init__()
        self.dw = nn.Conv2d(c, c, k, stride, pad, dilation=dil, groups=c, bias=False)
        self.pw = nn.Conv2d(c, c, 1, bias=False)
        self.bn = nn.BatchNorm2d(c, affine=False)

    def forward(self, x):
        return self.bn(self.pw(self.dw(F.relu(x))))


def _op(prim, c, stride):
    if prim == "none":
        return _Zero(stride)
    if prim.endswith("pooling_3x3"):
        return _PoolBN(prim[:3], c, stride)
    if prim == "skip_connection":
        return nn.Identity() if stride == 1 else _FR(c, c)
    k = int(prim[-1])
    if prim.startswith("separable"):
        return nn.Sequential(_DW(c, k, stride, k // 2, 1), _DW(c, k, 1, k // 2, 1))
    return _DW(c, k, stride, (k // 2) * 2, 2)


class _Cell(nn.Module):
    def __init__(self, prims, n, cpp, cp, c, red_prev, red):
        super().__init__()
        self.red = red
        self.pre0 = _FR(cpp, c) if red_prev else _Std(cpp, c)
        self.pre1 = _Std(cp, c)
        self.edges = nn.ModuleList()
        for i in range(n):
            for j in range(2 + i):
                self.edges.append(nn.ModuleList([_op(p, c, 2 if red and j < 2 else 1) for p in prims]))
        self.n = n

    def forward(self, s0, s1, ws):
        states = [self.pre0(s0), self.pre1(s1)]
        e = 0
        for i in range(self.n):
            acc = 0
            for j in range(2 + i):
                acc = acc + sum(w * op(states[j]) for w, op in zip(ws[i][j], self.edges[e]))
                e += 1
            states.append(acc)
        return torch.cat(states[2:], 1)


class DartsModuleNet(nn.Module):
    def __init__(self, prims, C, L, N, stem):
        super().__init__()
        prims = list(prims) + ["none"]
        c = stem * C
        self.stem_conv = nn.Conv2d(3, c, 3, padding=1, bias=False)
        self.stem_bn = nn.BatchNorm2d(c)
        cpp, cp, cur = c, c, C
        self.cells = nn.ModuleList()
        red_prev = False
        for i in range(L):
            red = L > 1 and ((L == 2 and i == 1) or (L > 2 and i in (L // 3, 2 * L // 3)))
            if red:
                cur *= 2
            self.cells.append(_Cell(prims, N, cpp, cp, cur, red_prev, red))
            red_prev = red
            cpp, cp = cp, cur * N
        self.classifier = nn.Linear(cp, 10)
        self.alpha_normal = nn.ParameterList([nn.Parameter(torch.zeros(i + 2, len(prims))) for i in range(N)])
        self.alpha_reduce = nn.ParameterList([nn.Parameter(torch.zeros(i + 2, len(prims))) for i in range(N)])

    def weights(self):
        return [p for n, p in self.named_parameters() if "alpha" not in n]

    def alphas(self):
        return list(self.alpha_normal) + list(self.alpha_reduce)

    def forward(self, x):
        wn = [F.softmax(a, -1) for a in self.alpha_normal]
        wr = [F.softmax(a, -1) for a in self.alpha_reduce]
        s0 = s1 = self.stem_bn(self.stem_conv(x))
        for cell in self.cells:
            s0, s1 = s1, cell(s0, s1, wr if cell.red else wn)
        return self.classifier(F.adaptive_avg_pool2d(s1, 1).flatten(1))


def module_search_step(model, vmodel, w_optim, a_optim, tx, ty, vx, vy, lr, mu=0.9, wd=3e-4, clip=5.0):
    """Second-order architect step + clipped SGD weight step."""
    ws = model.weights()
    g = torch.autograd.grad(F.cross_entropy(model(tx), ty), ws)
    with torch.no_grad():
        for w, vw, gi in zip(ws, vmodel.weights(), g):
            m = w_optim.state[w].get("momentum_buffer", 0.0) * mu
            vw.copy_(w - lr * (m + gi + wd * w))
        for a, va in zip(model.alphas(), vmodel.alphas()):
            va.copy_(a)
    vl = F.cross_entropy(vmodel(vx), vy)
    vg = torch.autograd.grad(vl, vmodel.alphas() + vmodel.weights())
    da, dw = vg[:len(model.alphas())], vg[len(model.alphas()):]
    eps = 0.01 / torch.cat([d.reshape(-1) for d in dw]).norm()
    with torch.no_grad():
        for p, d in zip(ws, dw):
            p += eps * d
    dp = torch.autograd.grad(F.cross_entropy(model(tx), ty), model.alphas())
    with torch.no_grad():
        for p, d in zip(ws, dw):
            p -= 2.0 * eps * d
    dn = torch.autograd.grad(F.cross_entropy(model(tx), ty), model.alphas())
    with torch.no_grad():
        for p, d in zip(ws, dw):
            p += eps * d
    a_optim.zero_grad()
    for a, d, p_, n_ in zip(model.alphas(), da, dp, dn):
        a.grad = d - lr * (p_ - n_) / (2.0 * eps)
    a_optim.step()
    w_optim.zero_grad()
    loss = F.cross_entropy(model(tx), ty)
    loss.backward()
    nn.utils.clip_grad_norm_(ws, clip)
    w_optim.step()
    return loss


class ModuleSearch:
    """Eager second-order search on :class:`DartsModuleNet` with the reference's optimizers
    (SGD momentum + weight decay + grad clip on the weights, Adam(0.5, 0.999) on the alphas)."""

    def __init__(self, prims, C, L, N, stem, device, lr=0.025, seed=0):
        torch.manual_seed(seed)
        self.model = DartsModuleNet(prims, C, L, N, stem).to(device)
        with torch.no_grad():
            for a in self.model.alphas():
                a.copy_(1e-3 * torch.randn_like(a))
        self.vmodel = copy.deepcopy(self.model)
        self.model.train()
        self.vmodel.train()
        self.lr = lr
        self.w_optim = torch.optim.SGD(self.model.weights(), lr, momentum=0.9, weight_decay=3e-4)
        self.a_optim = torch.optim.Adam(self.model.alphas(), 3e-4, betas=(0.5, 0.999), weight_decay=1e-3)

    def step(self, tx, ty, vx, vy):
        return module_search_step(self.model, self.vmodel, self.w_optim, self.a_optim, tx, ty, vx, vy, self.lr)
