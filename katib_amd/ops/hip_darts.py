"""Autograd wrappers over the HIP DARTS edge kernels (``katib_amd._hipkern``).

:func:`mixed_edge` runs one whole MixedOp edge (reference
``examples/v1beta1/trial-images/darts-cnn-cifar10/operations.py:164-180``) - all
primitives, their BatchNorms and the softmax-weighted sum - as ~7 forward /
~12 backward kernel launches (``csrc/hip/darts_ops.hip``):

forward   dwpw_fwd x (sep stage 1, sep stage 2, dil3, dil5), pool_fwd (avg+max),
          [pw_fwd x2 for the stride-2 skip], combine_fwd (weighted BN sum +
          running-stat updates)
backward  combine_bwd_reduce (BN-backward reductions + d softmax-weights),
          pw_bwd/dw_bwd per conv stage, pool_bwd (+ identity skip)

Weight gradients are accumulated by the kernels directly into each weight leaf's
``.grad`` when it exists (the flat gradient bucket of
:class:`katib_amd.models.darts_search.DartsSearch`), so no AccumulateGrad
launches follow; detached weights (the Hessian passes) skip weight-gradient work.
Callers that drive autograd with ``backward(inputs=...)`` must list every weight
leaf that requires grad (DartsSearch does).

Importing this module raises if the extension is missing: the HIP path never
silently degrades to PyTorch ops.
"""

from __future__ import annotations

import importlib
from typing import Dict, List, Optional, Sequence, Tuple

import torch

try:
    _K = importlib.import_module("katib_amd._hipkern")
except ImportError as e:  # pragma: no cover - machines without the build
    raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)

F64 = torch.float64


class EdgeSpec:
    """Static description of one edge: primitives, stride, parameter names, BN slots.

    ``slots[prim]`` lists indices into the per-call BN list ``bn`` (pairs of running
    mean/var views) in the layout's order (``DartsLayout._op_params``).
    """

    def __init__(self, prims: Sequence[str], stride: int, pnames: List[str], slots: Dict[str, Tuple[int, ...]]):
        self.prims = list(prims)
        self.stride = stride
        self.pnames = pnames
        self.slots = slots
        self.nbn = sum(len(v) for v in slots.values())
        self.pidx = {n: i for i, n in enumerate(pnames)}


def _bn(stats: Optional[torch.Tensor], rm, rv, count: int, training: bool, eps: float):
    if training:
        return (stats, rm, rv, 1.0 / count, False, eps)
    return (None, rm, rv, 1.0 / count, True, eps)


def _sink(p: torch.Tensor, extra: Dict[int, torch.Tensor], key: int):
    """Where a weight gradient goes: the leaf's existing .grad (bucket view), a fresh
    buffer returned through autograd, or nowhere (weight does not require grad)."""
    if not p.requires_grad:
        return None
    if p.grad is not None and p.is_leaf:
        return p.grad
    g = torch.zeros_like(p)
    extra[key] = g
    return g


class _MixedEdge(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, spec: EdgeSpec, bn, training, momentum, eps, *params):
        S = spec.stride
        x = x.contiguous()
        N, C, H, W = x.shape
        Ho, Wo = (H - 1) // S + 1, (W - 1) // S + 1
        cnt = N * Ho * Wo
        P = dict(zip(spec.pnames, params))
        dev = x.device
        stats = torch.zeros(max(spec.nbn, 1) * 2 * C, dtype=F64, device=dev) if training else None

        def st(i):
            return stats[i * 2 * C:(i + 1) * 2 * C] if training else None

        refs = [_bn(st(i), bn[i][0], bn[i][1], cnt, training, eps) for i in range(spec.nbn)]
        zs, bns, widx, upd, saved = [], [], [], [], {}
        id_idx, xid = -1, None
        for k, prim in enumerate(spec.prims):
            if prim == "none":
                continue
            sl = spec.slots.get(prim, ())
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                pad = K // 2
                d1 = torch.empty(N, C, Ho, Wo, device=dev)
                z1, d2, z2 = torch.empty_like(d1), torch.empty_like(d1), torch.empty_like(d1)
                _K.dwpw_fwd(x, P[prim + ".0.dw"], P[prim + ".0.pw"], K, 1, S, pad, None, d1, z1, st(sl[0]), True)
                _K.dwpw_fwd(z1, P[prim + ".1.dw"], P[prim + ".1.pw"], K, 1, 1, pad, refs[sl[0]], d2, z2,
                            st(sl[1]), True)
                upd.append(refs[sl[0]])
                zs.append(z2)
                bns.append(refs[sl[1]])
                saved[prim] = (d1, z1, d2, z2)
            elif prim.startswith("dilated_convolution"):
                K = int(prim[-1])
                d = torch.empty(N, C, Ho, Wo, device=dev)
                z = torch.empty_like(d)
                _K.dwpw_fwd(x, P[prim + ".dw"], P[prim + ".pw"], K, 2, S, (K // 2) * 2, None, d, z, st(sl[0]), True)
                zs.append(z)
                bns.append(refs[sl[0]])
                saved[prim] = (d, z)
            elif prim in ("avg_pooling_3x3", "max_pooling_3x3"):
                if "pool" not in saved:
                    za = torch.empty(N, C, Ho, Wo, device=dev)
                    zm = torch.empty_like(za)
                    am = torch.empty(N, C, Ho, Wo, dtype=torch.uint8, device=dev)
                    sa = spec.slots.get("avg_pooling_3x3")
                    sm = spec.slots.get("max_pooling_3x3")
                    _K.pool_fwd(x, za, zm, st(sa[0]) if sa else None, st(sm[0]) if sm else None, S, am)
                    saved["pool"] = (za, zm, am)
                zs.append(saved["pool"][0 if prim == "avg_pooling_3x3" else 1])
                bns.append(refs[sl[0]])
            elif prim == "skip_connection":
                if S == 1:
                    id_idx, xid = k, x
                    continue
                z = torch.empty(N, C, Ho, Wo, device=dev)
                _K.pw_fwd(x, P[prim + ".conv1"], z, st(sl[0]), 0, 2, 0)
                _K.pw_fwd(x, P[prim + ".conv2"], z, st(sl[0]), C // 2, 2, 1)
                zs.append(z)
                bns.append(refs[sl[0]])
                saved[prim] = (z,)
            else:
                raise ValueError(prim)
            widx.append(k)
        out = torch.empty(N, C, Ho, Wo, device=dev)
        _K.combine_fwd(zs, bns, widx, w, id_idx, xid, None, None, out, momentum, training, False,
                       upd if training else [])
        ctx.spec = spec
        ctx.meta = (saved, zs, bns, widx, id_idx, refs, training)
        ctx.save_for_backward(x, w, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, *params = ctx.saved_tensors
        spec = ctx.spec
        saved, zs, bns, widx, id_idx, refs, training = ctx.meta
        S = spec.stride
        P = dict(zip(spec.pnames, params))
        N, C, H, W = x.shape
        dev = x.device
        dout = dout.contiguous()
        nops = len(zs)
        nred = (nops + 1) * C + 1
        buf = torch.zeros(nred + w.numel(), dtype=F64, device=dev)
        red, gw = buf[:nred], buf[nred:]
        _K.combine_bwd_reduce(dout, zs, bns, x if id_idx >= 0 else None, red, widx, id_idx, gw)
        S1 = red[:C]
        jpos = {k: j for j, k in enumerate(widx)}

        def src(k, z):  # GradSrc of a weighted, BN'd op output
            j = jpos[k]
            return (dout, z, S1, red[(1 + j) * C:(2 + j) * C], bns[j], w, k)

        need_x = ctx.needs_input_grad[0]
        gx = torch.zeros_like(x) if need_x else None
        scratch = None
        extra: Dict[int, torch.Tensor] = {}

        def sink(name):
            return _sink(P[name], extra, spec.pidx[name])

        pool_done = False
        for k, prim in enumerate(spec.prims):
            if prim == "none":
                continue
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                pad = K // 2
                d1, z1, d2, z2 = saved[prim]
                b1 = refs[spec.slots[prim][0]]
                dd2 = torch.empty_like(d2)
                _K.pw_bwd(src(k, z2), P[prim + ".1.pw"], d2, z1, dd2, None, sink(prim + ".1.pw"), 0, 1, 0, 0, True)
                g1 = torch.empty_like(z1)
                red1 = torch.zeros(2 * C, dtype=F64, device=dev) if training else None
                _K.dw_bwd(z1, b1, P[prim + ".1.dw"], dd2, g1, sink(prim + ".1.dw"), red1, K, 1, 1, pad)
                gs1 = (g1, z1, red1[:C] if training else None, red1[C:] if training else None, b1, None, 0)
                dd1 = torch.empty_like(d1)
                _K.pw_bwd(gs1, P[prim + ".0.pw"], d1, x, dd1, None, sink(prim + ".0.pw"), 0, 1, 0, 0, True)
                if not need_x and scratch is None:
                    scratch = torch.empty_like(x)
                _K.dw_bwd(x, None, P[prim + ".0.dw"], dd1, gx if need_x else scratch, sink(prim + ".0.dw"), None,
                          K, 1, S, pad)
            elif prim.startswith("dilated_convolution"):
                K = int(prim[-1])
                d, z = saved[prim]
                dd = torch.empty_like(d)
                _K.pw_bwd(src(k, z), P[prim + ".pw"], d, x, dd, None, sink(prim + ".pw"), 0, 1, 0, 0, True)
                if not need_x and scratch is None:
                    scratch = torch.empty_like(x)
                _K.dw_bwd(x, None, P[prim + ".dw"], dd, gx if need_x else scratch, sink(prim + ".dw"), None,
                          K, 2, S, (K // 2) * 2)
            elif prim in ("avg_pooling_3x3", "max_pooling_3x3"):
                if pool_done or not need_x:
                    continue
                pool_done = True
                za, zm, am = saved["pool"]
                ga = gm = None
                for kk, pp in enumerate(spec.prims):
                    if pp == "avg_pooling_3x3":
                        ga = src(kk, za)
                    elif pp == "max_pooling_3x3":
                        gm = src(kk, zm)
                _K.pool_bwd(ga, gm, x, dout if id_idx >= 0 else None, w, id_idx, gx, S, am)
            elif prim == "skip_connection" and S != 1:
                (z,) = saved[prim]
                gs = src(k, z)
                _K.pw_bwd(gs, P[prim + ".conv1"], None, x, None, gx, sink(prim + ".conv1"), 0, 2, 0, 1, need_x)
                _K.pw_bwd(gs, P[prim + ".conv2"], None, x, None, gx, sink(prim + ".conv2"), C // 2, 2, 1, 1, need_x)
        if need_x and id_idx >= 0 and not pool_done:
            gx.add_(dout * w[id_idx])
        grads = [None] * len(params)
        for i, g in extra.items():
            grads[i] = g
        gw_out = gw.to(w.dtype) if ctx.needs_input_grad[1] else None
        return (gx, gw_out, None, None, None, None, None, *grads)


def mixed_edge(x, w, spec: EdgeSpec, bn: List[Tuple[torch.Tensor, torch.Tensor]], params: Sequence[torch.Tensor],
               training: bool, momentum: float = 0.1, eps: float = 1e-5):
    """sum_k w_k * op_k(x) for one edge; ``params`` ordered as ``spec.pnames``."""
    return _MixedEdge.apply(x, w, spec, bn, training, momentum, eps, *params)


# --------------------------------------------------------------------------------- preprocess
class _StdConvBN(torch.autograd.Function):
    """ReLU -> 1x1 conv (ReLUConvBN, operations.py) or FactorizedReduce (two stride-2
    1x1 convs on offset grids, channel-concatenated) -> BN(affine=False)."""

    @staticmethod
    def forward(ctx, x, rm, rv, training, momentum, eps, w1, w2):
        x = x.contiguous()
        N, Cin, H, W = x.shape
        fr = w2 is not None
        Cout = w1.shape[0] * (2 if fr else 1)
        Ho, Wo = (H // 2, W // 2) if fr else (H, W)
        cnt = N * Ho * Wo
        stats = torch.zeros(2 * Cout, dtype=F64, device=x.device) if training else None
        z = torch.empty(N, Cout, Ho, Wo, device=x.device)
        if fr:
            _K.pw_fwd(x, w1, z, stats, 0, 2, 0)
            _K.pw_fwd(x, w2, z, stats, Cout // 2, 2, 1)
        else:
            _K.pw_fwd(x, w1, z, stats, 0, 1, 0)
        bn = _bn(stats, rm, rv, cnt, training, eps)
        out = torch.empty_like(z)
        _K.combine_fwd([z], [bn], [0], None, -1, None, None, None, out, momentum, training, False, [])
        ctx.meta = (bn, fr, Cout, training)
        ctx.save_for_backward(x, z, w1, *([w2] if fr else []))
        return out

    @staticmethod
    def backward(ctx, dout):
        x, z, w1, *rest = ctx.saved_tensors
        w2 = rest[0] if rest else None
        bn, fr, Cout, training = ctx.meta
        dout = dout.contiguous()
        red = torch.zeros(2 * Cout + 1, dtype=F64, device=x.device)
        if training:
            _K.combine_bwd_reduce(dout, [z], [bn], None, red, [0], -1, None)
        gs = (dout, z, red[:Cout], red[Cout:2 * Cout], bn, None, 0)
        need_x = ctx.needs_input_grad[0]
        gx = torch.zeros_like(x) if need_x else None
        extra: Dict[int, torch.Tensor] = {}
        s1 = _sink(w1, extra, 1)
        if fr:
            s2 = _sink(w2, extra, 2)
            _K.pw_bwd(gs, w1, None, x, None, gx, s1, 0, 2, 0, 1, need_x)
            _K.pw_bwd(gs, w2, None, x, None, gx, s2, Cout // 2, 2, 1, 1, need_x)
        else:
            _K.pw_bwd(gs, w1, None, x, None, gx, s1, 0, 1, 0, 1, need_x)
        return gx, None, None, None, None, None, extra.get(1), extra.get(2)


def relu_conv_bn(x, w, rm, rv, training, momentum=0.1, eps=1e-5):
    return _StdConvBN.apply(x, rm, rv, training, momentum, eps, w, None)


def factorized_reduce_bn(x, w1, w2, rm, rv, training, momentum=0.1, eps=1e-5):
    return _StdConvBN.apply(x, rm, rv, training, momentum, eps, w1, w2)


def supported(x: torch.Tensor, stride: int) -> bool:
    """Shapes the kernels' 64-pixel tiling handles (CIFAR-style feature maps)."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 4:
        return False
    N, C, H, W = x.shape
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    return (C <= 256 and C * C <= 4096 and Wo <= 64 and 64 % Wo == 0 and Ho % (64 // Wo) == 0
            and H == Ho * stride and W == Wo * stride)
