"""DARTS CNN supernet for the CIFAR-10 search space, built for MI355X.

Behaviour matches the reference trial image
(``examples/v1beta1/trial-images/darts-cnn-cifar10/{model,operations,architect,search_space,run_trial}.py``):
same primitives (``<op>_<k>x<k>`` + ``none``), cell wiring (reduction cells at
L//3 and 2L//3 double the channels; 2-layer nets reduce at layer 1), MixedOp =
sum_k softmax(alpha)_k * op_k(x), BN(affine=False) inside ops, affine BN in the
stem, second-order architecture step (virtual step + finite-difference Hessian),
SGD(momentum, wd) + grad-clip for weights, Adam(0.5, 0.999) for alphas, and the
top-2-edges genotype parse.

MI355X-first structure (not a translation of the module tree):

* **Flat parameter storage.** All weights live in ONE fp32 buffer ``W`` (and the
  virtual weights in ``W'``); every parameter is a view. Gradients accumulate
  straight into flat gradient buffers (bucket views), so the virtual step, the
  +/-eps Hessian perturbations, the global-norm clip and SGD are whole-buffer ops
  and data parallelism is a single RCCL all-reduce per gradient
  (``katib_amd.parallel``), not one per tensor.
* **Functional network.** ``forward(x, params, alphas)`` is a pure function of a
  parameter table, so the real and the virtual model share all code and the
  Hessian passes run with weights detached (no weight-gradient kernels).
* **Fused, edge-batched kernels.** Each node (all its incoming MixedOp edges) runs
  through ``katib_amd.ops.hip_darts.mixed_node``: every kernel type is launched once
  for all edges that share a shape, with LDS-staged tiles (depthwise + pointwise on
  MFMA + BN statistics) and the softmax-weighted sums accumulated into the node
  output; the torch path (``katib_amd.ops.darts``) is the numerics oracle.
* **Graph capture.** The complete search step (5 forward + 5 backward passes,
  optimizer math, all-reduces) is captured once into a HIP graph and replayed:
  at C=4..16 channels the step is launch-bound, so removing per-kernel host
  overhead is the dominant win.
"""

from __future__ import annotations

import json
import math
from collections import namedtuple
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Genotype = namedtuple("Genotype", "normal normal_concat reduce reduce_concat")

PRIMITIVE_NAMES = ("none", "avg_pooling_3x3", "max_pooling_3x3", "skip_connection", "separable_convolution_3x3",
                   "separable_convolution_5x5", "dilated_convolution_3x3", "dilated_convolution_5x5")


class SearchSpace:
    """search_space.py:19-64 - the user primitives plus the trailing ``none``."""

    def __init__(self, primitives: Sequence[str]):
        self.primitives = list(primitives)
        if not self.primitives or self.primitives[-1] != "none":
            self.primitives.append("none")
        for p in self.primitives:
            if p not in PRIMITIVE_NAMES:
                raise ValueError("unknown DARTS primitive %r" % p)

    @staticmethod
    def from_arg(arg: str) -> "SearchSpace":
        return SearchSpace(json.loads(arg.replace("'", '"')))

    def parse(self, alphas: Sequence[torch.Tensor], k: int = 2):
        gene = []
        assert self.primitives[-1] == "none"
        for edges in alphas:
            edge_max, prim_idx = torch.topk(edges[:, :-1], 1)
            _, topk_edges = torch.topk(edge_max.view(-1), k)
            gene.append([(self.primitives[int(prim_idx[e])], int(e)) for e in topk_edges])
        return gene


# ----------------------------------------------------------------------------- layout
@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    offset: int = 0

    @property
    def numel(self):
        return int(math.prod(self.shape))


class DartsLayout:
    """Static description of the supernet: cells, edges, parameter offsets, BN slots."""

    def __init__(self, primitives: Sequence[str], init_channels=16, input_channels=3, num_classes=10,
                 num_layers=8, num_nodes=4, stem_multiplier=3):
        self.space = SearchSpace(primitives)
        self.prims = self.space.primitives
        self.C, self.L, self.N = init_channels, num_layers, num_nodes
        self.stem_mult = stem_multiplier
        self.num_classes = num_classes
        self.params: List[ParamSpec] = []
        self.bn: List[Tuple[str, int, bool]] = []  # (name, channels, affine)
        c_cur = stem_multiplier * init_channels
        self._p("stem.conv", (c_cur, input_channels, 3, 3))
        self._p("stem.bn.weight", (c_cur,))
        self._p("stem.bn.bias", (c_cur,))
        self.bn.append(("stem.bn", c_cur, True))
        cpp, cp, c_cur = c_cur, c_cur, init_channels
        self.cells = []
        red_prev = False
        for i in range(num_layers):
            if num_layers == 1:
                red = False
            elif (num_layers == 2 and i == 1) or (num_layers > 2 and i in (num_layers // 3, 2 * num_layers // 3)):
                c_cur *= 2
                red = True
            else:
                red = False
            cell = {"reduction": red, "reduction_prev": red_prev, "C": c_cur, "cpp": cpp, "cp": cp, "edges": []}
            pre = "cells.%d" % i
            if red_prev:
                self._p(pre + ".pre0.conv1", (c_cur // 2, cpp, 1, 1))
                self._p(pre + ".pre0.conv2", (c_cur // 2, cpp, 1, 1))
            else:
                self._p(pre + ".pre0.conv", (c_cur, cpp, 1, 1))
            self.bn.append((pre + ".pre0.bn", c_cur, False))
            self._p(pre + ".pre1.conv", (c_cur, cp, 1, 1))
            self.bn.append((pre + ".pre1.bn", c_cur, False))
            for n in range(num_nodes):
                for j in range(2 + n):
                    stride = 2 if red and j < 2 else 1
                    ep = "%s.n%d.e%d" % (pre, n, j)
                    edge = {"node": n, "src": j, "stride": stride, "prefix": ep}
                    cell["edges"].append(edge)
                    for prim in self.prims:
                        self._op_params(ep + "." + prim, prim, c_cur, stride)
            self.cells.append(cell)
            red_prev = red
            cpp, cp = cp, c_cur * num_nodes
        self._p("classifier.weight", (num_classes, cp))
        self._p("classifier.bias", (num_classes,))
        self.n_weights = sum(p.numel for p in self.params)
        self.by_name = {p.name: p for p in self.params}
        self.bn_index = {n: i for i, (n, _, _) in enumerate(self.bn)}
        self.n_alpha_rows = sum(2 + n for n in range(num_nodes))
        self.has_reduce = num_layers > 1
        self.n_alphas = self.n_alpha_rows * len(self.prims) * (2 if self.has_reduce else 1)

    def _p(self, name, shape):
        off = self.params[-1].offset + self.params[-1].numel if self.params else 0
        self.params.append(ParamSpec(name, tuple(shape), off))

    def _op_params(self, pre, prim, C, stride):
        if prim in ("none",):
            return
        if prim in ("avg_pooling_3x3", "max_pooling_3x3"):
            self.bn.append((pre + ".bn", C, False))
        elif prim == "skip_connection":
            if stride != 1:
                self._p(pre + ".conv1", (C // 2, C, 1, 1))
                self._p(pre + ".conv2", (C // 2, C, 1, 1))
                self.bn.append((pre + ".bn", C, False))
        elif prim.startswith("separable_convolution"):
            k = int(prim[-1])
            for s in (0, 1):
                self._p(pre + ".%d.dw" % s, (C, 1, k, k))
                self._p(pre + ".%d.pw" % s, (C, C, 1, 1))
                self.bn.append((pre + ".%d.bn" % s, C, False))
        elif prim.startswith("dilated_convolution"):
            k = int(prim[-1])
            self._p(pre + ".dw", (C, 1, k, k))
            self._p(pre + ".pw", (C, C, 1, 1))
            self.bn.append((pre + ".bn", C, False))

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {p.name: flat[p.offset:p.offset + p.numel].view(p.shape) for p in self.params}

    def alpha_views(self, flat: torch.Tensor) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
        K = len(self.prims)
        normal, reduce, off = [], [], 0
        for n in range(self.N):
            normal.append(flat[off:off + (2 + n) * K].view(2 + n, K))
            off += (2 + n) * K
        if self.has_reduce:
            for n in range(self.N):
                reduce.append(flat[off:off + (2 + n) * K].view(2 + n, K))
                off += (2 + n) * K
        return normal, reduce

    def init_weights(self, flat: torch.Tensor, gen: Optional[torch.Generator] = None):
        """PyTorch default inits (kaiming-uniform a=sqrt(5) for conv/linear, ones/zeros for BN)."""
        for p in self.params:
            v = flat[p.offset:p.offset + p.numel].view(p.shape)
            if p.name.endswith("bn.weight"):
                v.fill_(1.0)
            elif p.name.endswith("bn.bias"):
                v.zero_()
            elif p.name == "classifier.bias":
                fan_in = self.by_name["classifier.weight"].shape[1]
                bound = 1 / math.sqrt(fan_in)
                v.uniform_(-bound, bound, generator=gen)
            else:
                fan_in = int(math.prod(p.shape[1:]))
                bound = 1 / math.sqrt(fan_in)  # kaiming_uniform(a=sqrt(5)) => 1/sqrt(fan_in)
                v.uniform_(-bound, bound, generator=gen)


# ----------------------------------------------------------------------------- BN state
class BNState:
    """Running statistics of every BN layer in two flat buffers (mean, var)."""

    def __init__(self, layout: DartsLayout, device, dtype=torch.float32):
        self.offsets = []
        off = 0
        for _, c, _ in layout.bn:
            self.offsets.append((off, c))
            off += c
        # one buffer [mean | var]: a kernel can snapshot / merge all running statistics at once
        self.buf = torch.zeros(2 * off, device=device, dtype=dtype)
        self.buf[off:] = 1.0
        self.mean = self.buf[:off]
        self.var = self.buf[off:]
        self.index = layout.bn_index

    def get(self, name):
        o, c = self.offsets[self.index[name]]
        return self.mean[o:o + c], self.var[o:o + c]

    def copy_(self, other: "BNState"):
        self.buf.copy_(other.buf)


# ----------------------------------------------------------------------------- network
class DartsNetwork:
    """Functional supernet. ``ops`` is the op backend (katib_amd.ops.darts)."""

    def __init__(self, layout: DartsLayout, ops=None, momentum=0.1, eps=1e-5):
        self.layout = layout
        if ops is None:
            from ..ops import darts as ops
        self.ops = ops
        self.momentum, self.eps = momentum, eps
        self._specs = {}
        # data-parallel SyncBN (a Comm): training BN statistics over every rank's batch
        # (parallel/syncbn.py; the HIP cells use ops/hip_darts.py SyncBN under DartsSearch)
        self.sync = None
        # HIP path: the whole network as one Function (hip_darts.network_loss) instead of per-cell
        # Functions under autograd (attribute False: the per-cell path, kept for its A/B test;
        # profiles/darts_netfn_ab_r04.log)
        self.net_function = True

    def _batch_norm(self, x, rm, rv, w, b, training):
        if training and self.sync is not None and self.sync.distributed:
            from ..parallel.syncbn import sync_batch_norm

            return sync_batch_norm(x, rm, rv, w, b, self.momentum, self.eps, self.sync)
        return F.batch_norm(x, rm, rv, w, b, training, self.momentum, self.eps)

    def _bn(self, x, name, bn: BNState, training, w=None, b=None):
        rm, rv = bn.get(name)
        return self._batch_norm(x, rm, rv, w, b, training)

    def _hip(self, x, stride=1):
        hd = self.ops.hip_module() if self.ops.hip_enabled(x) else None
        return hd if hd is not None and hd.supported(x, stride) else None

    def _edge_spec(self, hd, e):
        """Static per-edge description for the fused HIP edge (parameter names relative
        to the edge prefix, BN slot indices in layout order)."""
        spec = self._specs.get(e["prefix"])
        if spec is None:
            pre = e["prefix"] + "."
            pnames = [p.name[len(pre):] for p in self.layout.params if p.name.startswith(pre)]
            bn_names = [n for n, _, _ in self.layout.bn if n.startswith(pre)]
            slots = {}
            for i, n in enumerate(bn_names):
                prim = n[len(pre):].split(".")[0]
                slots[prim] = slots.get(prim, ()) + (i,)
            spec = (hd.EdgeSpec(self.layout.prims, e["stride"], pnames, slots), pnames, bn_names)
            self._specs[e["prefix"]] = spec
        return spec

    def forward(self, x, P: Dict[str, torch.Tensor], normal, reduce, bn: BNState, training=True):
        """``normal`` / ``reduce``: per-node alpha rows (lists of [2+i, K]) or all rows of a
        cell type as one [rows, K] tensor (one softmax launch per cell type)."""
        L, ops = self.layout, self.ops
        hd = self.ops.hip_module() if self.ops.hip_enabled(x) else None
        if hd is not None and self._hip_cells(hd, x):
            return self._forward_cells(hd, x, P, normal, reduce, bn, training)
        if torch.is_tensor(normal):
            normal = self._split_rows(normal)
        if torch.is_tensor(reduce):
            reduce = self._split_rows(reduce)
        wn = [F.softmax(a, dim=-1) for a in normal]
        wr = [F.softmax(a, dim=-1) for a in reduce]
        if hd is not None and hd.stem_supported(x, P["stem.conv"]):
            s = hd.stem_conv(x, P["stem.conv"])
        else:
            s = F.conv2d(x, P["stem.conv"], padding=1)
        s = self._bn(s, "stem.bn", bn, training, P["stem.bn.weight"], P["stem.bn.bias"])
        s0 = s1 = s
        for ci, cell in enumerate(L.cells):
            pre = "cells.%d" % ci
            t0 = self.preprocess(s0, pre + ".pre0", cell["reduction_prev"], P, bn, training)
            t1 = self.preprocess(s1, pre + ".pre1", False, P, bn, training)
            weights = wr if cell["reduction"] else wn
            states = [t0, t1]
            ei = 0
            for n in range(L.N):
                edges = cell["edges"][ei:ei + 2 + n]
                ei += 2 + n
                states.append(self.mixed_node(states, edges, P, weights[n], bn, training))
            s0, s1 = s1, torch.cat(states[2:], dim=1)
        out = F.adaptive_avg_pool2d(s1, 1).flatten(1)
        return F.linear(out, P["classifier.weight"], P["classifier.bias"])

    # ------------------------------------------------------------------ cell-level HIP path
    def _split_rows(self, t):
        out, off = [], 0
        for n in range(self.layout.N):
            out.append(t[off:off + 2 + n])
            off += 2 + n
        return out

    def _hip_cells(self, hd, x) -> bool:
        """Whole-cell HIP Functions apply when every edge and preprocess shape is one the
        kernels support (hip_darts.supported / the 1x1 weight-size limit)."""
        key = ("__cells_ok__", tuple(x.shape), x.dtype)
        ok = self._specs.get(key)
        if ok is None:
            def tile_ok(C, H, stride):
                Ho = (H - 1) // stride + 1
                return C <= 256 and C * C <= 4096 and Ho <= 64 and 64 % Ho == 0 and Ho % (64 // Ho) == 0 \
                    and H == Ho * stride
            ok = hasattr(hd, "cell_forward") and x.dtype == torch.float32 and x.dim() == 4
            h = x.shape[2]
            for cell in self.layout.cells:
                C = cell["C"]
                if cell["reduction"]:
                    ok = ok and tile_ok(C, h, 2) and tile_ok(C, h // 2, 1)
                    h //= 2
                else:
                    ok = ok and tile_ok(C, h, 1)
                ok = ok and cell["cpp"] * C <= 8192 and cell["cp"] * C <= 8192
            self._specs[key] = ok
        return ok

    def _cell_spec(self, hd, ci):
        key = "__cell%d" % ci
        spec = self._specs.get(key)
        if spec is None:
            L = self.layout
            cell = L.cells[ci]
            pre = "cells.%d" % ci
            if cell["reduction_prev"]:
                pre0 = ("fr", [pre + ".pre0.conv1", pre + ".pre0.conv2"], pre + ".pre0.bn")
            else:
                pre0 = ("std", [pre + ".pre0.conv"], pre + ".pre0.bn")
            pre1 = ("std", [pre + ".pre1.conv"], pre + ".pre1.bn")
            nodes, ei, row = [], 0, 0
            for n in range(L.N):
                node = []
                for e in cell["edges"][ei:ei + 2 + n]:
                    es, pnames, bn_names = self._edge_spec(hd, e)
                    node.append((es, [e["prefix"] + "." + q for q in pnames], bn_names, e["src"], row + e["src"]))
                nodes.append(node)
                ei += 2 + n
                row += 2 + n
            spec = hd.CellSpec(pre0, pre1, nodes, cell["C"])
            self._specs[key] = spec
        return spec

    def forward_loss(self, x, y, P: Dict[str, torch.Tensor], normal, reduce, bn: BNState, training=True):
        """(cross-entropy loss, logits). On the whole-cell HIP path the head - global average
        pool, classifier, log-softmax + NLL and their backward - is one fused HIP Function
        (hip_darts.head_loss); the returned logits carry no gradient there."""
        hd = self.ops.hip_module() if self.ops.hip_enabled(x) else None
        if (hd is not None and self._hip_cells(hd, x) and hasattr(hd, "network_loss") and self.net_function
                and hd.stem_supported(x, P["stem.conv"]) and P["classifier.weight"].shape[0] <= 64
                and P["classifier.weight"].shape[1] <= 1024 and y.dtype == torch.int64 and y.dim() == 1):
            # the whole network as ONE autograd Function (hip_darts._Network): no framework launches
            L = self.layout
            an = normal if torch.is_tensor(normal) else torch.cat(list(normal), 0)
            ar = None
            if L.has_reduce:
                ar = reduce if torch.is_tensor(reduce) else torch.cat(list(reduce), 0)
            spec = self._net_spec(hd)
            return hd.network_loss(spec, x, y, [P[n] for n in spec.names], an, ar, bn.get, training, self.momentum,
                                   self.eps)
        if hd is not None and self._hip_cells(hd, x) and hasattr(hd, "head_loss"):
            s1 = self._forward_cells(hd, x, P, normal, reduce, bn, training, features=True)
            if hd.head_supported(s1, P["classifier.weight"], y):
                return hd.head_loss(s1, P["classifier.weight"], P["classifier.bias"], y)
            out = F.adaptive_avg_pool2d(s1, 1).flatten(1)
            logits = F.linear(out, P["classifier.weight"], P["classifier.bias"])
        else:
            logits = self.forward(x, P, normal, reduce, bn, training)
        return F.cross_entropy(logits, y), logits

    def _net_spec(self, hd):
        spec = self._specs.get("__net__")
        if spec is None:
            L = self.layout
            spec = hd.NetSpec(("stem.conv", "stem.bn.weight", "stem.bn.bias", "stem.bn"),
                              [self._cell_spec(hd, ci) for ci in range(len(L.cells))],
                              [c["reduction"] for c in L.cells], ("classifier.weight", "classifier.bias"))
            self._specs["__net__"] = spec
        return spec

    def _forward_cells(self, hd, x, P, normal, reduce, bn, training, features=False):
        L = self.layout
        an = normal if torch.is_tensor(normal) else torch.cat(list(normal), 0)
        wn = F.softmax(an, dim=-1)
        wr = None
        if L.has_reduce:
            ar = reduce if torch.is_tensor(reduce) else torch.cat(list(reduce), 0)
            wr = F.softmax(ar, dim=-1)
        if hd.stem_supported(x, P["stem.conv"]) and training and hasattr(hd, "stem_conv_bn"):
            rm, rv = bn.get("stem.bn")
            s = hd.stem_conv_bn(x, P["stem.conv"], P["stem.bn.weight"], P["stem.bn.bias"], rm, rv, self.momentum,
                                self.eps)
        elif hd.stem_supported(x, P["stem.conv"]) and not torch.is_grad_enabled() and hasattr(hd, "stem_bn_eval"):
            rm, rv = bn.get("stem.bn")
            s = hd.stem_bn_eval(hd.stem_conv(x, P["stem.conv"]), P["stem.bn.weight"], P["stem.bn.bias"], rm, rv,
                                self.eps)
        else:
            if hd.stem_supported(x, P["stem.conv"]):
                s = hd.stem_conv(x, P["stem.conv"])
            else:
                s = F.conv2d(x, P["stem.conv"], padding=1)
            s = self._bn(s, "stem.bn", bn, training, P["stem.bn.weight"], P["stem.bn.bias"])
        s0 = s1 = s
        for ci, cell in enumerate(L.cells):
            spec = self._cell_spec(hd, ci)
            params = [P[n] for n in spec.names]
            out = hd.cell_forward(spec, s0, s1, wr if cell["reduction"] else wn, params, bn.get, training,
                                  self.momentum, self.eps)
            s0, s1 = s1, out
        if features:
            return s1
        out = F.adaptive_avg_pool2d(s1, 1).flatten(1)
        return F.linear(out, P["classifier.weight"], P["classifier.bias"])

    def preprocess(self, x, name, reduce, P, bn, training):
        """ReLUConvBN(1x1) or FactorizedReduce (model.py cell preprocessing)."""
        ops = self.ops
        rm, rv = bn.get(name + ".bn")
        if reduce:
            w1, w2 = P[name + ".conv1"], P[name + ".conv2"]
            hd = self._hip(x, 2)
            if hd is not None and w1.shape[0] * w1.shape[1] <= 8192:
                return hd.factorized_reduce_bn(x, w1, w2, rm, rv, training, self.momentum, self.eps)
            t = ops.factorized_reduce(x, w1, w2)
        else:
            w = P[name + ".conv"]
            hd = self._hip(x, 1)
            if hd is not None and w.shape[0] * w.shape[1] <= 8192:
                return hd.relu_conv_bn(x, w, rm, rv, training, self.momentum, self.eps)
            t = ops.relu_conv1x1(x, w)
        return self._batch_norm(t, rm, rv, None, None, training)

    def mixed_node(self, states, edges, P, w, bn, training):
        """Node = sum over incoming edges of MixedOp (model.py:61-71). On the HIP backend all
        edges of the node run as one edge-batched autograd Function."""
        hd = self._hip(states[0], 1)
        if hd is not None and all(hd.supported(states[e["src"]], e["stride"]) for e in edges):
            specs, bnl, params = [], [], []
            for e in edges:
                spec, pnames, bn_names = self._edge_spec(hd, e)
                specs.append(spec)
                bnl.append([bn.get(nm) for nm in bn_names])
                params.append([P[e["prefix"] + "." + nm] for nm in pnames])
            return hd.mixed_node([states[e["src"]] for e in edges], [w[e["src"]] for e in edges], specs, bnl,
                                 params, training, self.momentum, self.eps)
        acc = None
        for e in edges:
            y = self.mixed_op(states[e["src"]], e, P, w[e["src"]], bn, training)
            acc = y if acc is None else acc + y
        return acc

    def mixed_op(self, x, e, P, w, bn, training):
        """sum_k w_k * op_k(x) (operations.py:164-180)."""
        ops, pre, stride = self.ops, e["prefix"], e["stride"]
        hd = self._hip(x, stride)
        if hd is not None:
            spec, pnames, bn_names = self._edge_spec(hd, e)
            return hd.mixed_edge(x, w, spec, [bn.get(n) for n in bn_names], [P[pre + "." + n] for n in pnames],
                                 training, self.momentum, self.eps)
        out = None
        for k, prim in enumerate(self.layout.prims):
            if prim == "none":
                continue  # contributes exactly 0 (x * 0.)
            if prim == "avg_pooling_3x3":
                y = self._bn(ops.avg_pool3x3(x, stride), pre + "." + prim + ".bn", bn, training)
            elif prim == "max_pooling_3x3":
                y = self._bn(ops.max_pool3x3(x, stride), pre + "." + prim + ".bn", bn, training)
            elif prim == "skip_connection":
                if stride == 1:
                    y = x
                else:
                    y = self._bn(ops.factorized_reduce(x, P[pre + "." + prim + ".conv1"],
                                                       P[pre + "." + prim + ".conv2"]),
                                 pre + "." + prim + ".bn", bn, training)
            elif prim.startswith("separable_convolution"):
                k_ = int(prim[-1])
                y = ops.relu_dw_pw(x, P[pre + "." + prim + ".0.dw"], P[pre + "." + prim + ".0.pw"], stride, k_ // 2, 1)
                y = self._bn(y, pre + "." + prim + ".0.bn", bn, training)
                y = ops.relu_dw_pw(y, P[pre + "." + prim + ".1.dw"], P[pre + "." + prim + ".1.pw"], 1, k_ // 2, 1)
                y = self._bn(y, pre + "." + prim + ".1.bn", bn, training)
            elif prim.startswith("dilated_convolution"):
                k_ = int(prim[-1])
                y = ops.relu_dw_pw(x, P[pre + "." + prim + ".dw"], P[pre + "." + prim + ".pw"], stride,
                                   (k_ // 2) * 2, 2)
                y = self._bn(y, pre + "." + prim + ".bn", bn, training)
            else:
                raise ValueError(prim)
            y = w[k] * y
            out = y if out is None else out + y
        return out


def accuracy(logits, target, topk=(1, 5)):
    maxk = max(topk)
    _, pred = logits.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
    return [correct[:k].reshape(-1).float().sum() / target.size(0) for k in topk]
