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

Cross-workgroup sums go to ``REP`` replicas of each accumulator (workgroup b adds
into replica b % REP) so that no address sees more than grid/REP atomic adds; a
``fold_f64`` launch sums the replicas of BN statistics / BN-backward reductions
into replica 0 before their consumers run (which then read one value). Weight gradients are accumulated by the kernels
directly into each weight leaf's ``.grad`` when that is a row-0 view of a buffer
registered with :func:`register_grad_replicas` (the flat gradient bucket of
:class:`katib_amd.models.darts_search.DartsSearch`, folded once per backward pass
with :func:`fold`), so no AccumulateGrad launches follow; detached weights (the
Hessian passes) skip weight-gradient work. Callers that drive autograd with
``backward(inputs=...)`` must list every weight leaf that requires grad
(DartsSearch does).

Importing this module raises if the extension is missing: the HIP path never
silently degrades to PyTorch ops.
"""

from __future__ import annotations

import importlib
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import torch

try:
    _K = importlib.import_module("katib_amd._hipkern")
except ImportError as e:  # pragma: no cover - machines without the build
    raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)

F64 = torch.float64
REP = int(_K.REP)
_REPLICATED: List[Tuple[weakref.ref, int]] = []  # (buffer [REP][n], n)


def register_grad_replicas(buf: torch.Tensor):
    """Declare ``buf`` ([REP][n] fp32, contiguous) a replicated gradient accumulator:
    ``.grad`` views into its row 0 receive kernel atomics into all REP rows."""
    if buf.dim() != 2 or buf.shape[0] != REP or not buf.is_contiguous() or buf.dtype != torch.float32:
        raise ValueError("replicated gradient buffer must be contiguous fp32 [%d][n]" % REP)
    _REPLICATED.append((weakref.ref(buf), buf.shape[1]))


def fold(buf: torch.Tensor):
    """row 0 <- sum of all replica rows; rows 1.. <- 0 (one kernel)."""
    _K.fold_rows(buf)


def _replica_stride(g: torch.Tensor) -> int:
    ptr = g.data_ptr()
    for ref, n in list(_REPLICATED):
        buf = ref()
        if buf is None:
            _REPLICATED.remove((ref, n))
            continue
        base = buf.data_ptr()
        if base <= ptr and ptr + g.numel() * 4 <= base + n * 4:
            return n
    return 0


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


def _bn(stats: Optional[torch.Tensor], rm, rv, count: int, training: bool, eps: float, C: int):
    """BN reference tuple for the kernels; ``stats`` ([REP][2C]) is folded before use."""
    if training:
        return (stats, rm, rv, 1.0 / count, False, eps, 1, 2 * C)
    return (None, rm, rv, 1.0 / count, True, eps, 1, 2 * C)


def _fold_slots(stats, slot: int, idx, n: int):
    segs = [(stats[i * slot:(i + 1) * slot], n, n) for i in idx]
    if segs:
        _K.fold_f64(segs)


class _Sinks:
    """Weight-gradient destinations of one backward call."""

    def __init__(self):
        self.temps = []

    def get(self, p: torch.Tensor, key: int):
        """(pointer tensor, replica stride): the leaf's registered replicated .grad, else
        a temporary [REP][numel] buffer summed in :meth:`finish`; (None, 0) when the
        weight does not require grad."""
        if not p.requires_grad:
            return None, 0
        g = p.grad if p.is_leaf else None
        if g is not None and g.is_contiguous():
            stride = _replica_stride(g)
            if stride:
                return g, stride
        t = torch.zeros(REP, p.numel(), device=p.device, dtype=torch.float32)
        self.temps.append((key, t, g, p))
        return t[0].view_as(p), p.numel()

    def finish(self, grads: List):
        for key, t, g, p in self.temps:
            s = t.sum(0).view_as(p)
            if g is not None:
                g.add_(s)
            else:
                grads[key] = s


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
        slot = REP * 2 * C
        stats = torch.zeros(max(spec.nbn, 1) * slot, dtype=F64, device=dev) if training else None

        def st(i):
            return stats[i * slot:(i + 1) * slot] if training else None

        refs = [_bn(st(i), bn[i][0], bn[i][1], cnt, training, eps, C) for i in range(spec.nbn)]
        zs, bns, widx, upd, saved = {}, {}, [], [], {}
        id_idx, xid = -1, None
        stage1, stage2 = [], []  # BN slots produced before / by the separable convs' second stage
        for k, prim in enumerate(spec.prims):
            if prim == "none":
                continue
            sl = spec.slots.get(prim, ())
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                d1 = torch.empty(N, C, Ho, Wo, device=dev)
                z1 = torch.empty_like(d1)
                _K.dwpw_fwd(x, P[prim + ".0.dw"], P[prim + ".0.pw"], K, 1, S, K // 2, None, d1, z1, st(sl[0]), True)
                saved[prim] = [d1, z1]
                stage1.append(sl[0])
                stage2.append(sl[1])
            elif prim.startswith("dilated_convolution"):
                K = int(prim[-1])
                d = torch.empty(N, C, Ho, Wo, device=dev)
                z = torch.empty_like(d)
                _K.dwpw_fwd(x, P[prim + ".dw"], P[prim + ".pw"], K, 2, S, (K // 2) * 2, None, d, z, st(sl[0]), True)
                zs[k], bns[k] = z, refs[sl[0]]
                saved[prim] = (d, z)
                stage1.append(sl[0])
            elif prim in ("avg_pooling_3x3", "max_pooling_3x3"):
                if "pool" not in saved:
                    za = torch.empty(N, C, Ho, Wo, device=dev)
                    zm = torch.empty_like(za)
                    am = torch.empty(N, C, Ho, Wo, dtype=torch.uint8, device=dev)
                    sa = spec.slots.get("avg_pooling_3x3")
                    sm = spec.slots.get("max_pooling_3x3")
                    _K.pool_fwd(x, za, zm, st(sa[0]) if sa else None, st(sm[0]) if sm else None, S, am)
                    saved["pool"] = (za, zm, am)
                zs[k] = saved["pool"][0 if prim == "avg_pooling_3x3" else 1]
                bns[k] = refs[sl[0]]
                stage1.append(sl[0])
            elif prim == "skip_connection":
                if S == 1:
                    id_idx, xid = k, x
                    continue
                z = torch.empty(N, C, Ho, Wo, device=dev)
                _K.pw_fwd(x, P[prim + ".conv1"], z, st(sl[0]), 0, 2, 0)
                _K.pw_fwd(x, P[prim + ".conv2"], z, st(sl[0]), C // 2, 2, 1)
                zs[k], bns[k] = z, refs[sl[0]]
                saved[prim] = (z,)
                stage1.append(sl[0])
            else:
                raise ValueError(prim)
            widx.append(k)
        if training:
            _fold_slots(stats, slot, stage1, 2 * C)
        for k, prim in enumerate(spec.prims):
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                sl = spec.slots[prim]
                d1, z1 = saved[prim]
                d2, z2 = torch.empty_like(d1), torch.empty_like(d1)
                _K.dwpw_fwd(z1, P[prim + ".1.dw"], P[prim + ".1.pw"], K, 1, 1, K // 2, refs[sl[0]], d2, z2,
                            st(sl[1]), True)
                upd.append(refs[sl[0]])
                zs[k], bns[k] = z2, refs[sl[1]]
                saved[prim] = (d1, z1, d2, z2)
        if training:
            _fold_slots(stats, slot, stage2, 2 * C)
        zs = [zs[k] for k in widx]
        bns = [bns[k] for k in widx]
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
        nw = w.numel()
        buf = torch.zeros(REP * (nred + nw), dtype=F64, device=dev)
        red, gw_rep = buf[:REP * nred], buf[REP * nred:]
        _K.combine_bwd_reduce(dout, zs, bns, x if id_idx >= 0 else None, red, widx, id_idx, gw_rep)
        _K.fold_f64([(red, nred, nred), (gw_rep, nw, nw)])
        S1 = red[:C]
        jpos = {k: j for j, k in enumerate(widx)}

        def src(k, z):  # GradSrc of a weighted, BN'd op output
            j = jpos[k]
            return (dout, z, S1, red[(1 + j) * C:(2 + j) * C], bns[j], w, k, 1, nred)

        need_x = ctx.needs_input_grad[0]
        gx = torch.zeros_like(x) if need_x else None
        scratch = None
        sinks = _Sinks()

        def sink(name):
            return sinks.get(P[name], spec.pidx[name])

        # separable convs: both second stages first, one fold of their BN-backward sums, then stage 1
        seps = [(k, p) for k, p in enumerate(spec.prims) if p.startswith("separable_convolution")]
        red1 = torch.zeros(max(len(seps), 1) * REP * 2 * C, dtype=F64, device=dev) if training else None
        stage_grad = {}
        for i, (k, prim) in enumerate(seps):
            K = int(prim[-1])
            d1, z1, d2, z2 = saved[prim]
            b1 = refs[spec.slots[prim][0]]
            dd2 = torch.empty_like(d2)
            gp, gst = sink(prim + ".1.pw")
            _K.pw_bwd(src(k, z2), P[prim + ".1.pw"], d2, z1, dd2, None, gp, 0, 1, 0, 0, True, gst)
            g1 = torch.empty_like(z1)
            r1 = red1[i * REP * 2 * C:(i + 1) * REP * 2 * C] if training else None
            gp, gst = sink(prim + ".1.dw")
            _K.dw_bwd(z1, b1, P[prim + ".1.dw"], dd2, g1, gp, r1, K, 1, 1, K // 2, gst)
            stage_grad[prim] = (g1, r1, b1)
        if training and seps:
            _K.fold_f64([(red1[i * REP * 2 * C:(i + 1) * REP * 2 * C], 2 * C, 2 * C) for i in range(len(seps))])
        pool_done = False
        for k, prim in enumerate(spec.prims):
            if prim == "none":
                continue
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                pad = K // 2
                d1, z1, d2, z2 = saved[prim]
                g1, r1, b1 = stage_grad[prim]
                gs1 = (g1, z1, r1[:C] if training else None, r1[C:2 * C] if training else None, b1, None, 0, 1, 2 * C)
                dd1 = torch.empty_like(d1)
                gp, gst = sink(prim + ".0.pw")
                _K.pw_bwd(gs1, P[prim + ".0.pw"], d1, x, dd1, None, gp, 0, 1, 0, 0, True, gst)
                if not need_x and scratch is None:
                    scratch = torch.empty_like(x)
                gp, gst = sink(prim + ".0.dw")
                _K.dw_bwd(x, None, P[prim + ".0.dw"], dd1, gx if need_x else scratch, gp, None, K, 1, S, pad, gst)
            elif prim.startswith("dilated_convolution"):
                K = int(prim[-1])
                d, z = saved[prim]
                dd = torch.empty_like(d)
                gp, gst = sink(prim + ".pw")
                _K.pw_bwd(src(k, z), P[prim + ".pw"], d, x, dd, None, gp, 0, 1, 0, 0, True, gst)
                if not need_x and scratch is None:
                    scratch = torch.empty_like(x)
                gp, gst = sink(prim + ".dw")
                _K.dw_bwd(x, None, P[prim + ".dw"], dd, gx if need_x else scratch, gp, None, K, 2, S, (K // 2) * 2,
                          gst)
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
                gp, gst = sink(prim + ".conv1")
                _K.pw_bwd(gs, P[prim + ".conv1"], None, x, None, gx, gp, 0, 2, 0, 1, need_x, gst)
                gp, gst = sink(prim + ".conv2")
                _K.pw_bwd(gs, P[prim + ".conv2"], None, x, None, gx, gp, C // 2, 2, 1, 1, need_x, gst)
        if need_x and id_idx >= 0 and not pool_done:
            gx.add_(dout * w[id_idx])
        grads = [None] * len(params)
        sinks.finish(grads)
        gw_out = gw_rep[:nw].to(w.dtype) if ctx.needs_input_grad[1] else None
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
        stats = torch.zeros(REP * 2 * Cout, dtype=F64, device=x.device) if training else None
        z = torch.empty(N, Cout, Ho, Wo, device=x.device)
        if fr:
            _K.pw_fwd(x, w1, z, stats, 0, 2, 0)
            _K.pw_fwd(x, w2, z, stats, Cout // 2, 2, 1)
        else:
            _K.pw_fwd(x, w1, z, stats, 0, 1, 0)
        if training:
            _K.fold_f64([(stats, 2 * Cout, 2 * Cout)])
        bn = _bn(stats, rm, rv, cnt, training, eps, Cout)
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
        nred = 2 * Cout + 1
        red = torch.zeros(REP * nred, dtype=F64, device=x.device)
        if training:
            _K.combine_bwd_reduce(dout, [z], [bn], None, red, [0], -1, None)
            _K.fold_f64([(red, nred, nred)])
        gs = (dout, z, red[:Cout], red[Cout:2 * Cout], bn, None, 0, 1, nred)
        need_x = ctx.needs_input_grad[0]
        gx = torch.zeros_like(x) if need_x else None
        sinks = _Sinks()
        grads = [None, None, None]
        g1, s1 = sinks.get(w1, 1)
        if fr:
            g2, s2 = sinks.get(w2, 2)
            _K.pw_bwd(gs, w1, None, x, None, gx, g1, 0, 2, 0, 1, need_x, s1)
            _K.pw_bwd(gs, w2, None, x, None, gx, g2, Cout // 2, 2, 1, 1, need_x, s2)
        else:
            _K.pw_bwd(gs, w1, None, x, None, gx, g1, 0, 1, 0, 1, need_x, s1)
        sinks.finish(grads)
        return gx, None, None, None, None, None, grads[1], grads[2]


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
