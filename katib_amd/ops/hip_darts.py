"""Autograd wrappers over the HIP DARTS kernels (``katib_amd._hipkern``).

:func:`mixed_node` computes one DARTS node - the sum over its incoming edges of the
MixedOp ``sum_k softmax(alpha)_k * op_k(x_j)`` (reference
``examples/v1beta1/trial-images/darts-cnn-cifar10/operations.py:164-180`` and
``model.py:61-71``) - with every kernel launched once for *all* edges of the node that
share its shape (edge batches, ``blockIdx.y`` = edge):

forward   dwpw_fwd per (kernel size, dilation, stride) [separable stage 1, dilated],
          pool_fwd (avg + max + argmax), pw_fwd x2 (stride-2 skip = FactorizedReduce),
          fold, dwpw_fwd with BN-apply prologue [separable stage 2], fold,
          combine_fwd summing every edge's weighted BN outputs into the node (+ running stats)
backward  combine_bwd_reduce (BN-backward sums + d softmax-weights), fold, then pw_bwd /
          dw_bwd / pool_bwd batches; every input gradient is written (not accumulated) by
          its first kernel, so no memsets

Cross-workgroup sums go to ``REP`` replicas of each accumulator (workgroup b adds
into replica b % REP) so that no address sees more than grid/REP atomic adds; a
``fold_f64`` launch sums the replicas of BN statistics / BN-backward reductions
into replica 0 before their consumers run (which then read one value).
Weight gradients are accumulated by the kernels directly into each weight leaf's
``.grad`` when that is a row-0 view of a buffer registered with
:func:`register_grad_replicas` (the flat gradient bucket of
:class:`katib_amd.models.darts_search.DartsSearch`, folded once per backward pass
with :func:`fold`), so no AccumulateGrad launches follow; detached weights (the
Hessian passes) skip weight-gradient work. Callers that drive autograd with
``backward(inputs=...)`` must list every weight leaf that requires grad
(DartsSearch does).

Importing this module raises if the extension is missing: the HIP path never
silently degrades to PyTorch ops.
"""

from __future__ import annotations

import contextlib
import importlib
import weakref
from collections import defaultdict
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import _hipload

try:
    _K = _hipload.hipkern()
except ImportError as e:  # pragma: no cover - machines without the build
    raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)

F64 = torch.float64
REP = int(_K.REP)
# storage of the per-op intermediates (depthwise outputs d, pre-BN op outputs z): bf16 in the
# _hipkern_zbf16 build variant (KATIB_AMD_HIPKERN), fp32 otherwise; node states, gradients, BN
# statistics and weights stay fp32 either way
ZDT = torch.bfloat16 if bool(getattr(_K, "ZBF16", False)) else torch.float32
# FOLD (module attribute, tests only): a fold_f64 launch sums the REP replicas of each cross-workgroup
# reduction before its consumers (which then read rep=1); False: consumers sum the replicas themselves
# and the fold launches disappear. Measured on MI355X (B5 step): 13.3 ms
# with the folds, 17.1 ms without - every consumer workgroup re-reading 32 replicas costs more
# than ~180 small fold launches.
FOLD = True
_R = 1 if FOLD else REP
# Self-folding producers (darts_ops.h FoldTail): with a counter ring registered for the device,
# every launch that adds into f64 replicas folds them in its last workgroup, and the fold_f64
# launches between producers and consumers disappear. Needs FOLD (consumers read replica 0).
# Off (set_selffold(True): tests and experiments): measured on MI355X, one arrival counter
# made every producer ~15-25 us slower (2000 same-address atomics serialise memory-side: B5
# step 12.1 ms), 32 sharded counters still lose to the fold launches (8.22 vs 8.05 ms),
# profiles/darts_selffold_edge_ab_r03.log.
SELFFOLD = False
_CTR: Dict[int, torch.Tensor] = {}


def set_selffold(on: bool):
    """A/B switch for tests and experiments (call between steps, never inside a capture)."""
    global SELFFOLD
    if on and _SYNC is not None:
        raise RuntimeError("self-folding producers cannot run under SyncBN (see _check_sync_fold_mode)")
    SELFFOLD = bool(on)
    _K.set_selffold(SELFFOLD)
_CTR_SIZE = 64 * 33 * 32  # 64 launch slots of (top + 32 shard) counters, 128 B apart


def _selffold(dev) -> bool:
    """Register the device's counter ring on first use (never inside a graph capture, whose
    private pool must not own it) and report whether producers on the current device fold
    their own replicas (the C++ side attaches tails under exactly this condition)."""
    if not FOLD or not SELFFOLD:
        return False
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _CTR:
        if torch.cuda.is_current_stream_capturing():
            return bool(_K.selffold_ready())
        t = torch.zeros(_CTR_SIZE, dtype=torch.int32, device=torch.device("cuda", idx))
        _K.set_fold_counters(t)
        _CTR[idx] = t
    return bool(_K.selffold_ready())


# SyncBN state of the step being built / run (set by DartsSearch through :func:`sync_scope`): BN
# statistics and BN-backward sums are folded AND summed over the ranks (one launch, the
# fold_sync kernel of parallel/xgmi.py), so every rank normalises with the global batch's
# statistics; None: per-rank BN
_SYNC = None


def _check_sync_fold_mode():
    """SyncBN sums the BN reductions over the ranks inside the fold (``_fold`` / ``SyncBN.fold``)
    and ``_bn`` then divides by count * world. Without fold launches (FOLD False) or with
    self-folding producers (SELFFOLD True) that fold never runs, and every rank would
    normalise its LOCAL sums by the global count - mean and variance off by a factor of world,
    silently. Refuse those combinations."""
    if not FOLD:
        raise RuntimeError("SyncBN needs the fold launches (hip_darts.FOLD): the cross-rank BN sum "
                           "happens inside them")
    if SELFFOLD:
        raise RuntimeError("SyncBN is incompatible with self-folding producers (hip_darts.SELFFOLD): "
                           "their replicas would never be summed over the ranks")


class SyncBN:
    """Global-batch BatchNorm for the DARTS supernet under data parallelism (reference BN over
    the whole 128-image batch, ``operations.py:62,96,117,139``). Construction is collective.

    With the one-shot xGMI path available the fold of every BN reduction becomes ONE launch that
    also sums the folded values over the ranks (``XgmiWorkspace.fold_sync``, graph-capturable, its
    own small workspace so its epochs never interleave with the gradient all-reduces'); otherwise
    the fold is followed by ONE grouped RCCL all-reduce of the synchronised segments
    (``Comm.allreduce_sum_many_``), which stays inside the captured step when the communicator
    passed ``Comm.probe_rccl_capture`` (else: host-side RCCL / gloo, step not captured)."""

    def __init__(self, comm):
        _check_sync_fold_mode()
        self.comm, self.world = comm, comm.world_size
        self.ws = None
        if comm.xgmi is not None:
            from ..parallel import xgmi

            ar = xgmi.create(comm, capacity=1 << 16, blocks=16)
            self.ws = ar.ws if ar is not None else None
        # RCCL inside the graph when the one-shot path is off or failed its self-test (collective)
        self.rccl_graph = self.ws is None and comm.probe_rccl_capture()
        self.folds = 0  # cross-rank rendezvous issued (one per fold call)

    @property
    def capturable(self) -> bool:
        return self.ws is not None or self.rccl_graph

    @property
    def path(self) -> str:
        return "xgmi-oneshot" if self.ws is not None else ("rccl-graph" if self.rccl_graph else "host")

    def fold(self, segs):
        """segs: (f64 replicas, n, rstride[, sync]); sync defaults to True (d alpha segments pass False)."""
        self.folds += 1
        if self.ws is not None:
            self.ws.fold_sync(list(segs))
            return
        _K.fold_f64([tuple(sg[:3]) for sg in segs])
        self.comm.allreduce_sum_many_([sg[0][:sg[1]] for sg in segs if len(sg) < 4 or sg[3]])


class sync_scope:
    """``with sync_scope(SyncBN or None):`` - the kernels launched inside use global-batch BN."""

    def __init__(self, sync):
        self.sync = sync

    def __enter__(self):
        global _SYNC
        if self.sync is not None:
            _check_sync_fold_mode()
        self.prev, _SYNC = _SYNC, self.sync
        return self

    def __exit__(self, *exc):
        global _SYNC
        _SYNC = self.prev
        return False


def _world() -> int:
    return _SYNC.world if _SYNC is not None else 1


def _fold(segs):
    """Fold the replicas of f64 reductions into replica 0 (under SyncBN: and sum the segments not
    marked local over the ranks)."""
    if _SYNC is not None:
        _SYNC.fold(segs)
    else:
        _K.fold_f64([tuple(sg[:3]) for sg in segs])


def _defer(dev) -> bool:
    """Consumers may sum the replicas themselves (deferred folds; never under SyncBN, whose
    cross-rank sum happens in the fold)."""
    return DEFER_FOLD and FOLD and _SYNC is None and not _selffold(dev)


def _fold64(segs, dev=None):
    """fold_f64 launch between producers and consumers, unless the producers folded themselves."""
    if FOLD and (dev is None or not _selffold(dev)):
        _fold(segs)
_CAP = {"combine_fwd": 4, "dwpw_fwd": 8, "pw_fwd": 16, "pool_fwd": 8, "combine_bwd_reduce": 4, "pw_bwd": 16,
        "dw_bwd": 20, "pool_bwd": 8}
_REPLICATED: List[Tuple[weakref.ref, int]] = []  # (buffer [REP][n], n)


class _Arena:
    """Step-scoped fp64 workspace for the BN-statistics / reduction accumulators.

    A DARTS step requests ~150 small zeroed fp64 buffers; zeroing each one was its own
    fill launch. Between :func:`arena_begin` and :func:`arena_end` they are bump-allocated
    from one buffer that is zeroed by a single launch at the start of the step (captured
    into the step's HIP graph with the rest). The first step sizes the arena; buffers that
    a captured graph may reference are never freed."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None
        self.keep: List[torch.Tensor] = []
        self.off = 0
        self.used = 0
        self.need = 0
        self.active = False
        self.pending_zero = False  # the zeroing rides on the step's first network launch (alpha softmax)


_ARENA = _Arena()


def arena_begin(device, deferred_zero: bool = False):
    """Start a step's arena. ``deferred_zero``: the zeroing is left to the step's first
    :func:`network_loss` (its alpha-softmax launch zeroes the arena too), else one fill here."""
    a = _ARENA
    if a.need and (a.buf is None or a.buf.numel() < a.need):
        if a.buf is not None:
            a.keep.append(a.buf)
        a.buf = torch.zeros(a.need, dtype=F64, device=device)
        a.pending_zero = False
    elif a.buf is not None:
        if deferred_zero:
            a.pending_zero = True
        else:
            a.buf.zero_()
    a.off, a.used, a.active = 0, 0, True


def arena_end():
    a = _ARENA
    a.need = max(a.need, a.used)
    a.active = False
    if a.pending_zero:  # nobody consumed the deferred zeroing: do it now
        a.buf.zero_()
        a.pending_zero = False


def zeros64(n: int, device) -> torch.Tensor:
    a = _ARENA
    if a.active:
        if a.pending_zero and a.buf is not None:
            # the deferred zeroing was meant for the step's network_loss launch, but a slice is
            # handed out first (a per-cell fallback step): zero the arena now, never hand out stale sums
            a.buf.zero_()
            a.pending_zero = False
        step = (n + 31) // 32 * 32  # 256-byte aligned slices
        a.used += step
        if a.buf is not None and a.off + step <= a.buf.numel() and a.buf.device == device:
            t = a.buf[a.off:a.off + n]
            a.off += step
            return t
    return torch.zeros(n, dtype=F64, device=device)


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


def _launch(name: str, calls: List, *args):
    """Run an edge-batched kernel over ``calls`` in chunks of its batch capacity."""
    cap = _CAP[name]
    fn = getattr(_K, name)
    for i in range(0, len(calls), cap):
        fn(calls[i:i + cap], *args)


MULTI = True  # mixed-variant launches (module attribute: the per-variant path stays for A/B tests)
# Deferred folds: the consumers right after a node's first reduction (the separable second stage's
# input BN in the forward, the second-stage / dilated pointwise backward after combine_bwd_reduce)
# sum the 32 replicas themselves in their prologue (workgroup-cooperative, one round trip:
# darts_ops.hip coop_pair_sums), so those fold launches merge into the node's next fold
# (False: fold before every consumer, as before; profiles/darts_defer_fold_ab_r03.log)
DEFER_FOLD = True


def _unfolded(bn):
    """The BN tuple of :func:`_bn` reading all REP replicas (its stats are not folded yet)."""
    return bn[:6] + (REP, bn[7])


# a node's stage-1 separable + dilated depthwise backward in one mixed-variant launch, each part in
# its own buffer, summed into gx by the pool-backward launch (profiles/darts_dwb_multi_ab_r03.log)
DWB_MULTI = True
# fused per-edge input gradient (edge_bwd_kernel) instead of per-family dw_bwd / pool_bwd launches.
# Off by default: measured SLOWER on MI355X (B5 step 9.22 vs 8.05 ms; its 4 conv slots run
# serially inside each workgroup, and fewer / larger bands only narrow the gap: 8.74 ms at 64 KB
# bands), profiles/darts_selffold_edge_ab_r03.log. Kept for its numerics test (module attribute).
EDGE_BWD = False


# A node's pools launched beside its stage-1 dw-pw entries (one launch instead of two per node).
# Off (module attribute, tests): measured a wash on the B5 step (6.98 vs 6.96 ms,
# profiles/darts_vec_ab_r04.log) - the pool workgroups (highest blockIdx.y) dispatch after the dw-pw
# bands anyway, so only the ~1.6 us launch boundary goes.
JOINT_POOL = False


def _dwpw_multi(entries):
    """dw-pw entries (x, dw, pw, inbn, d, z, stats, K, dil, S, pad) of one stage, mixed kernel sizes,
    dilations and strides: one launch per 20 entries (per (K, dil, S) group with MULTI off)."""
    if not entries:
        return
    if MULTI:
        for i in range(0, len(entries), 20):
            _K.dwpw_fwd_multi(entries[i:i + 20])
        return
    groups = defaultdict(list)
    for e in entries:
        groups[e[7:]].append(e[:7])
    for (K, dil, S, pad), calls in groups.items():
        _launch("dwpw_fwd", calls, K, dil, S, pad, True)


def _pool_multi(entries):
    """pool_fwd entries (x, zavg, zmax, stats_avg, stats_max, amax, S) of both strides."""
    if not entries:
        return
    if MULTI:
        for i in range(0, len(entries), _CAP["pool_fwd"]):
            _K.pool_fwd_multi(entries[i:i + _CAP["pool_fwd"]])
        return
    groups = defaultdict(list)
    for e in entries:
        groups[e[6]].append(e[:6])
    for S, calls in groups.items():
        _launch("pool_fwd", calls, S)


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
    if training:  # under SyncBN the statistics are sums over every rank's batch
        return (stats, rm, rv, 1.0 / (count * _world()), False, eps, _R, 2 * C)
    return (None, rm, rv, 1.0 / count, True, eps, 1, 2 * C)


class _Sinks:
    """Weight-gradient destinations of one backward call."""

    def __init__(self):
        self.temps = []

    def get(self, p: torch.Tensor, key):
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


class _Edge:
    """Per-call state of one edge inside a node."""

    def __init__(self, i, x, w, spec: EdgeSpec, bn, params):
        self.i, self.x, self.w, self.spec, self.bn = i, x, w, spec, bn
        self.P = dict(zip(spec.pnames, params))
        self.S = spec.stride
        self.refs = []
        self.zs, self.bns, self.widx = {}, {}, []
        self.saved = {}
        self.id_idx, self.xid = -1, None
        self.upd = []
        self.id_done = False


def _node_forward(xs, ws, specs, bns, params_list, training, momentum, eps, out=None, extra_fold=()):
    """One node's forward (all kernels of every incoming edge); ``out`` may be a preallocated
    contiguous buffer (the cell writes each node straight into its concat slot). Returns
    (out, edges) - ``edges`` is the state :func:`_node_backward` needs."""
    E = len(specs)
    xs = [t.contiguous() for t in xs]
    _selffold(xs[0].device)  # before any producer launch: registers the counter ring on first use
    N, C = xs[0].shape[:2]
    S0 = specs[0].stride
    Ho = (xs[0].shape[2] - 1) // S0 + 1
    Wo = (xs[0].shape[3] - 1) // S0 + 1
    cnt = N * Ho * Wo
    dev = xs[0].device
    slot = REP * 2 * C
    edges, off = [], 0
    for i in range(E):
        edges.append(_Edge(i, xs[i], ws[i], specs[i], bns[i], params_list[i]))
    nslots = sum(e.spec.nbn for e in edges)
    stats = zeros64(max(nslots, 1) * slot, dev) if training else None
    base = 0
    for e in edges:
        e.slot0 = base
        e.refs = [_bn(stats[(base + i) * slot:(base + i + 1) * slot] if training else None, e.bn[i][0],
                      e.bn[i][1], cnt, training, eps, C) for i in range(e.spec.nbn)]
        base += e.spec.nbn

    def st(e, i):
        return stats[(e.slot0 + i) * slot:(e.slot0 + i + 1) * slot] if training else None

    def new():  # a per-op intermediate (d or z)
        return torch.empty(N, C, Ho, Wo, device=dev, dtype=ZDT)

    # ---- stage 1: grouped by (K, dilation, stride, pad)
    dw_groups = defaultdict(list)
    pool_groups = defaultdict(list)
    fr_calls = []
    stage1, stage2 = [], []
    for e in edges:
        for k, prim in enumerate(e.spec.prims):
            if prim == "none":
                continue
            sl = e.spec.slots.get(prim, ())
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                d1, z1 = new(), new()
                dw_groups[(K, 1, e.S, K // 2)].append(
                    (e.x, e.P[prim + ".0.dw"], e.P[prim + ".0.pw"], None, d1, z1, st(e, sl[0])))
                e.saved[prim] = [d1, z1]
                stage1.append(e.slot0 + sl[0])
                stage2.append(e.slot0 + sl[1])
            elif prim.startswith("dilated_convolution"):
                K = int(prim[-1])
                d, z = new(), new()
                dw_groups[(K, 2, e.S, (K // 2) * 2)].append(
                    (e.x, e.P[prim + ".dw"], e.P[prim + ".pw"], None, d, z, st(e, sl[0])))
                e.zs[k], e.bns[k] = z, e.refs[sl[0]]
                e.saved[prim] = (d, z)
                stage1.append(e.slot0 + sl[0])
            elif prim in ("avg_pooling_3x3", "max_pooling_3x3"):
                if "pool" not in e.saved:
                    za, zm = new(), new()
                    am = torch.empty(N, C, Ho, Wo, dtype=torch.uint8, device=dev)
                    sa = e.spec.slots.get("avg_pooling_3x3")
                    sm = e.spec.slots.get("max_pooling_3x3")
                    pool_groups[e.S].append((e.x, za, zm, st(e, sa[0]) if sa else None,
                                             st(e, sm[0]) if sm else None, am))
                    e.saved["pool"] = (za, zm, am)
                e.zs[k] = e.saved["pool"][0 if prim == "avg_pooling_3x3" else 1]
                e.bns[k] = e.refs[sl[0]]
                stage1.append(e.slot0 + sl[0])
            elif prim == "skip_connection":
                if e.S == 1:
                    e.id_idx, e.xid = k, e.x
                    continue
                z = new()
                fr_calls.append((e.x, e.P[prim + ".conv1"], z, st(e, sl[0]), 0, 0))
                fr_calls.append((e.x, e.P[prim + ".conv2"], z, st(e, sl[0]), C // 2, 1))
                e.zs[k], e.bns[k] = z, e.refs[sl[0]]
                e.saved[prim] = (z,)
                stage1.append(e.slot0 + sl[0])
            else:
                raise ValueError(prim)
            e.widx.append(k)
    # all (K, dil, S) groups of the stage in ONE mixed-variant launch (and both pool strides in
    # one): independent entries overlap on the chip instead of running as 4-9 serial launches
    # (forking the groups over side streams - concurrent graph branches - measured slower on
    # MI355X: B5 step 15.4 ms vs 13.05 ms sequential)
    dw1 = [(*c, K, dil, S, pad) for (K, dil, S, pad), calls in dw_groups.items() for c in calls]
    pools = [(*c, S) for S, calls in pool_groups.items() for c in calls]
    if JOINT_POOL and MULTI and dw1 and pools and len(dw1) <= 20 and len(pools) <= _CAP["pool_fwd"]:
        # the pools beside the stage-1 dw-pw bands in one launch (both read only the node inputs;
        # the binding falls back to the two launches where the plane path does not apply)
        _K.dwpw_pool_fwd_multi(dw1, pools)
    else:
        _dwpw_multi(dw1)
        _pool_multi(pools)
    if fr_calls:
        _launch("pw_fwd", fr_calls, 2)
    defer = training and _defer(dev)
    if training and stage1 and not defer:
        _fold64([(stats[i * slot:(i + 1) * slot], 2 * C, 2 * C) for i in sorted(set(stage1))], dev)
    # ---- separable stage 2 (stride 1, input BN-apply prologue)
    s2_groups = defaultdict(list)
    for e in edges:
        for k, prim in enumerate(e.spec.prims):
            if prim.startswith("separable_convolution"):
                K = int(prim[-1])
                sl = e.spec.slots[prim]
                d1, z1 = e.saved[prim]
                d2, z2 = new(), new()
                inbn = _unfolded(e.refs[sl[0]]) if defer else e.refs[sl[0]]
                s2_groups[K].append((z1, e.P[prim + ".1.dw"], e.P[prim + ".1.pw"], inbn, d2, z2, st(e, sl[1])))
                e.upd.append(e.refs[sl[0]])
                e.zs[k], e.bns[k] = z2, e.refs[sl[1]]
                e.saved[prim] = (d1, z1, d2, z2)
    _dwpw_multi([(*c, K, 1, 1, K // 2) for K, calls in s2_groups.items() for c in calls])
    if training and (stage2 or (defer and stage1) or extra_fold):  # (deferred: the stage-1 statistics too)
        _fold64([(stats[i * slot:(i + 1) * slot], 2 * C, 2 * C)
                 for i in sorted(set(stage2 + (stage1 if defer else [])))] + list(extra_fold), dev)
    # ---- weighted sums into the node output
    if out is None:
        out = torch.empty(N, C, Ho, Wo, device=dev)
    ccalls = []
    for e in edges:
        e.zl = [e.zs[k] for k in e.widx]
        e.bl = [e.bns[k] for k in e.widx]
        ccalls.append((e.zl, e.bl, e.widx, e.w, e.id_idx, e.xid, e.upd if training else []))
    cap = _CAP["combine_fwd"]
    for i in range(0, E, cap):
        _K.combine_fwd(ccalls[i:i + cap], None, None, out, momentum, training, i > 0)
    return out, edges


def _node_backward(edges, training, C, dout, gx_of, take_first, sinks, pkey, cell_gw=None):
    """One node's backward. ``gx_of(i)`` is the input-gradient buffer of edge i (edges of
    different nodes that read the same state share one buffer); ``take_first(i)`` is True for
    the first kernel that writes it (it overwrites instead of accumulating, so no memset);
    weight gradients go through ``sinks`` under the keys ``pkey(edge, name)``. Buffers no
    kernel wrote (an edge whose only primitive is ``none``) are the caller's to zero.
    The alpha-weight gradients stay in ``edge.gw`` (f64, folded)."""
    E = len(edges)
    dout = dout.contiguous()
    dev = dout.device

    def sink(e, name):
        return sinks.get(e.P[name], pkey(e, name))

    # ---- BN-backward sums and d(alpha) for every edge, one fold
    sizes = []
    for e in edges:
        e.nred = (len(e.zl) + 1) * C + 1
        sizes.append(REP * (e.nred + e.w.numel()))
    buf = zeros64(sum(sizes), dev)
    o = 0
    calls, segs = [], []
    for e, sz in zip(edges, sizes):
        e.red = buf[o:o + REP * e.nred]
        e.gw = buf[o + REP * e.nred:o + sz]
        o += sz
        calls.append((dout, e.zl, e.bl, e.x if e.id_idx >= 0 else None, e.red, e.widx, e.id_idx, e.gw))
        segs += [(e.red, e.nred, e.nred), (e.gw, e.w.numel(), e.w.numel(), False)]  # d alpha stays per rank
    _launch("combine_bwd_reduce", calls)
    # deferred: the pointwise backward right below sums the replicas itself and this fold joins
    # the separable second stages' fold (or runs after that pointwise launch)
    defer = training and _defer(dev)
    # inside a cell every reader of this node's reductions sums the replicas itself, so the node
    # folds nothing: the d(alpha) segments go to the cell, which folds them once (if it needs them)
    nofold = defer and cell_gw is not None and not EDGE_BWD
    if nofold:
        cell_gw.extend(segs[1::2])
    if not _selffold(dev) and not defer:
        _fold(segs if FOLD else segs[1::2])  # the d(alpha) segments are always folded

    r_early = REP if defer else _R  # replicas the pointwise backward below reads
    r_late = REP if nofold else _R  # ... and the pool / stride-2 skip backward further down

    def src(e, k, z, rep=r_late):  # GradSrc of a weighted, BN'd op output
        j = e.widx.index(k)
        return (dout, z, e.red[:C], e.red[(1 + j) * C:(2 + j) * C], e.bl[j], e.w, k, rep, e.nred)

    gxs = [gx_of(e.i) for e in edges]

    # dilated convs' pointwise backward is independent of the separable chain: its entries join
    # the separable second stages' pw_bwd batch (one launch instead of two)
    dils = [(e, k, p) for e in edges for k, p in enumerate(e.spec.prims) if p.startswith("dilated_convolution")]
    pwd, dd_of = [], {}
    for e, k, prim in dils:
        d, z = e.saved[prim]
        dd = torch.empty(d.shape, device=dev)  # gradients stay fp32
        dd_of[(e.i, prim)] = dd
        g, gst = sink(e, prim + ".pw")
        pwd.append((src(e, k, z, r_early), e.P[prim + ".pw"], d, e.x, dd, None, g, 0, 0, gst))
    # ---- separable convs: both second stages, one fold, both first stages
    seps = [(e, k, p) for e in edges for k, p in enumerate(e.spec.prims) if p.startswith("separable_convolution")]
    if not seps and pwd:
        _launch("pw_bwd", pwd, 1, 0, True)
    if not seps and defer and not nofold:
        _fold(segs)
    if seps:
        red1 = zeros64(len(seps) * REP * 2 * C, dev) if training else None
        pw2, dw2 = [], defaultdict(list)
        for n, (e, k, prim) in enumerate(seps):
            K = int(prim[-1])
            d1, z1, d2, z2 = e.saved[prim]
            dd2 = torch.empty(d2.shape, device=dev)
            g, gst = sink(e, prim + ".1.pw")
            pw2.append((src(e, k, z2, r_early), e.P[prim + ".1.pw"], d2, z1, dd2, None, g, 0, 0, gst))
            g1 = torch.empty(z1.shape, device=dev)
            r1 = red1[n * REP * 2 * C:(n + 1) * REP * 2 * C] if training else None
            g, gst = sink(e, prim + ".1.dw")
            dw2[K].append((z1, e.refs[e.spec.slots[prim][0]], e.P[prim + ".1.dw"], dd2, g1, g, r1, gst, False))
            e.saved[prim + "/g1"] = (g1, r1)
        _launch("pw_bwd", pw2 + (pwd if MULTI else []), 1, 0, True)
        if not MULTI and pwd:
            _launch("pw_bwd", pwd, 1, 0, True)
        if MULTI:  # both kernel sizes in one launch (distinct g1 / red1 per entry)
            allc = [(*c, K) for K, calls in dw2.items() for c in calls]
            for i in range(0, len(allc), _CAP["dw_bwd"]):
                _K.dw_bwd_multi(allc[i:i + _CAP["dw_bwd"]])
        else:
            for K, calls in dw2.items():
                _launch("dw_bwd", calls, K, 1, 1, K // 2)
        if training and not nofold:
            _fold64([(red1[n * REP * 2 * C:(n + 1) * REP * 2 * C], 2 * C, 2 * C) for n in range(len(seps))]
                    + (segs if defer else []), dev)
        pw1 = []
        for e, k, prim in seps:
            d1, z1, d2, z2 = e.saved[prim]
            g1, r1 = e.saved[prim + "/g1"]
            b1 = e.refs[e.spec.slots[prim][0]]
            gs1 = (g1, z1, r1[:C] if training else None, r1[C:2 * C] if training else None, b1, None, 0, r_late, 2 * C)
            dd1 = torch.empty(d1.shape, device=dev)
            e.saved[prim + "/dd1"] = dd1
            g, gst = sink(e, prim + ".0.pw")
            pw1.append((gs1, e.P[prim + ".0.pw"], d1, e.x, dd1, None, g, 0, 0, gst))
        _launch("pw_bwd", pw1, 1, 0, True)

    # ---- every edge's input gradient: stage-1 separable and dilated depthwise backward, pools and
    # the identity skip in ONE fused launch (edge_bwd_kernel), else the per-family launches below
    first = {e.i: take_first(e.i) for e in edges}

    def tf(i):  # the first writer of gx_of(i) overwrites it
        f = first.get(i, False)
        first[i] = False
        return f

    def pool_srcs(e):
        za, zm, am = e.saved["pool"]
        ga = gm = None
        for k, p in enumerate(e.spec.prims):
            if p == "avg_pooling_3x3":
                ga = src(e, k, za)
            elif p == "max_pooling_3x3":
                gm = src(e, k, zm)
        return ga, gm, am

    if EDGE_BWD:
        entries = []
        for e in edges:
            convs = [None] * 4
            for k, prim in enumerate(e.spec.prims):
                if prim.startswith("separable_convolution"):
                    g, gst = sink(e, prim + ".0.dw")
                    convs[0 if prim[-1] == "3" else 1] = (e.P[prim + ".0.dw"], e.saved[prim + "/dd1"], g, gst)
                elif prim.startswith("dilated_convolution"):
                    g, gst = sink(e, prim + ".dw")
                    convs[2 if prim[-1] == "3" else 3] = (e.P[prim + ".dw"], dd_of[(e.i, prim)], g, gst)
            ga, gm, am = pool_srcs(e) if "pool" in e.saved else (None, None, None)
            entries.append((e.x, gxs[e.i], first[e.i], convs, ga, gm, am, dout if e.id_idx >= 0 else None, e.w,
                            e.id_idx, e.S))
        ok = True
        for i in range(0, len(entries), 4):
            ok = ok and bool(_K.edge_bwd(entries[i:i + 4]))
        if ok:
            for e in edges:
                first[e.i] = False
        elif len(entries) > 4:  # a partial launch cannot be undone: fail loudly
            raise RuntimeError("edge_bwd accepted part of a node's edges")
    if (not EDGE_BWD or not ok) and MULTI and DWB_MULTI:
        # every stage-1 separable and dilated depthwise backward of the node in ONE mixed-variant
        # launch, each into its own buffer (no read-modify-write of gx, so no ordering between
        # them); the pool-backward launch then forms gx = pools + identity + those parts, once
        convs, parts = [], defaultdict(list)
        for e, k, prim in seps + dils:
            sep = prim.startswith("separable_convolution")
            K = int(prim[-1])
            t = torch.empty_like(e.x)
            parts[e.i].append(t)
            name = prim + (".0.dw" if sep else ".dw")
            g, gst = sink(e, name)
            dd = e.saved[prim + "/dd1"] if sep else dd_of[(e.i, prim)]
            convs.append((e.x, None, e.P[name], dd, t, g, None, gst, True, K, 1 if sep else 2, e.S))
        for i in range(0, len(convs), _CAP["dw_bwd"]):
            _K.dw_bwd_multi(convs[i:i + _CAP["dw_bwd"]])
        sums = []
        for e in edges:
            ga, gm, am = pool_srcs(e) if "pool" in e.saved else (None, None, None)
            ex = parts.get(e.i, [])
            if ga is None and gm is None and e.id_idx < 0 and not ex:
                continue  # only a stride-2 skip (below) or 'none' writes this edge's gradient
            sums.append((ga, gm, e.x, dout if e.id_idx >= 0 else None, e.w, e.id_idx, gxs[e.i], am, tf(e.i), e.S, ex))
            e.id_done = True
        for i in range(0, len(sums), _CAP["pool_bwd"]):
            _K.pool_bwd_multi(sums[i:i + _CAP["pool_bwd"]])
    elif not EDGE_BWD or not ok:
        if seps:
            dw1 = defaultdict(list)
            for e, k, prim in seps:
                K = int(prim[-1])
                g, gst = sink(e, prim + ".0.dw")
                dw1[(K, e.S)].append((e.x, None, e.P[prim + ".0.dw"], e.saved[prim + "/dd1"], gxs[e.i], g, None, gst,
                                      tf(e.i)))
            for (K, S), calls in dw1.items():
                _launch("dw_bwd", calls, K, 1, S, K // 2)
        # ---- dilated convs (depthwise backward; the pointwise part ran above)
        if dils:
            dwd = defaultdict(list)
            for e, k, prim in dils:
                K = int(prim[-1])
                g, gst = sink(e, prim + ".dw")
                dwd[(K, e.S)].append((e.x, None, e.P[prim + ".dw"], dd_of[(e.i, prim)], gxs[e.i], g, None, gst,
                                      tf(e.i)))
            for (K, S), calls in dwd.items():
                _launch("dw_bwd", calls, K, 2, S, (K // 2) * 2)
        # ---- pools (+ the identity skip of stride-1 edges)
        pools = defaultdict(list)
        for e in edges:
            if "pool" not in e.saved:
                continue
            ga, gm, am = pool_srcs(e)
            pools[e.S].append((ga, gm, e.x, dout if e.id_idx >= 0 else None, e.w, e.id_idx, gxs[e.i], am, tf(e.i)))
            e.id_done = True
        if MULTI:  # both strides in one launch (entries are distinct edges: distinct gx buffers)
            allp = [(*c, S) for S, calls in pools.items() for c in calls]
            for i in range(0, len(allp), _CAP["pool_bwd"]):
                _K.pool_bwd_multi(allp[i:i + _CAP["pool_bwd"]])
        else:
            for S, calls in pools.items():
                _launch("pool_bwd", calls, S)
        for e in edges:
            if e.id_idx >= 0 and not e.id_done:
                if tf(e.i):
                    torch.mul(dout, e.w[e.id_idx], out=gxs[e.i])
                else:
                    gxs[e.i].add_(dout * e.w[e.id_idx])
    # ---- stride-2 skip (FactorizedReduce): scattered adds, so its gx must exist already
    frc = []
    for e in edges:
        if "skip_connection" in e.saved:
            if tf(e.i):
                gxs[e.i].zero_()
            k = e.spec.prims.index("skip_connection")
            (z,) = e.saved["skip_connection"]
            gs = src(e, k, z)
            g, gst = sink(e, "skip_connection.conv1")
            frc.append((gs, e.P["skip_connection.conv1"], None, e.x, None, gxs[e.i], g, 0, 0, gst))
            g, gst = sink(e, "skip_connection.conv2")
            frc.append((gs, e.P["skip_connection.conv2"], None, e.x, None, gxs[e.i], g, C // 2, 1, gst))
    if frc:
        _launch("pw_bwd", frc, 2, 1, True)


class _MixedNode(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, *flat):
        specs, bns, training, momentum, eps, nparams = meta
        E = len(specs)
        params, off = [], 2 * E
        for n in nparams:
            params.append(flat[off:off + n])
            off += n
        out, edges = _node_forward(flat[:E], flat[E:2 * E], specs, bns, params, training, momentum, eps)
        ctx.meta = (edges, training, out.shape[1])
        ctx.save_for_backward(*flat)
        return out

    @staticmethod
    def backward(ctx, dout):
        flat = ctx.saved_tensors
        edges, training, C = ctx.meta
        E = len(edges)
        sinks = _Sinks()
        pbase, acc = [], 2 * E
        for e in edges:
            pbase.append(acc)
            acc += len(e.spec.pnames)
        gxs = [torch.empty_like(e.x) for e in edges]
        first = [True] * E

        def take_first(i):
            f = first[i]
            first[i] = False
            return f

        _node_backward(edges, training, C, dout, lambda i: gxs[i], take_first, sinks,
                       lambda e, name: pbase[e.i] + e.spec.pidx[name])
        for i in range(E):
            if first[i]:  # an edge whose only primitive is "none"
                gxs[i].zero_()
        grads = [None] * len(flat)
        for i, e in enumerate(edges):
            grads[i] = gxs[i] if ctx.needs_input_grad[1 + i] else None
            grads[E + i] = e.gw[:e.w.numel()].to(e.w.dtype) if ctx.needs_input_grad[1 + E + i] else None
        sinks.finish(grads)
        return (None, *grads)


def mixed_node(xs: Sequence[torch.Tensor], ws: Sequence[torch.Tensor], specs: Sequence[EdgeSpec],
               bns: Sequence[List[Tuple[torch.Tensor, torch.Tensor]]], params: Sequence[Sequence[torch.Tensor]],
               training: bool, momentum: float = 0.1, eps: float = 1e-5):
    """sum over edges e of sum_k ws[e]_k * op_k(xs[e]); ``params[e]`` ordered as ``specs[e].pnames``."""
    meta = (list(specs), list(bns), training, momentum, eps, [len(p) for p in params])
    flat = list(xs) + list(ws) + [p for ps in params for p in ps]
    return _MixedNode.apply(meta, *flat)


def mixed_edge(x, w, spec: EdgeSpec, bn: List[Tuple[torch.Tensor, torch.Tensor]], params: Sequence[torch.Tensor],
               training: bool, momentum: float = 0.1, eps: float = 1e-5):
    """sum_k w_k * op_k(x) for one edge (a node with a single incoming edge)."""
    return mixed_node([x], [w], [spec], [bn], [params], training, momentum, eps)


# --------------------------------------------------------------------------------- preprocess
def _dims(x: torch.Tensor):
    """(N, C, H, W) of an [N][C][H][W] tensor or of a node-major [nodes][N][C/nodes][H][W] one."""
    if x.dim() == 5:
        return x.shape[1], x.shape[0] * x.shape[2], x.shape[3], x.shape[4]
    return tuple(x.shape)


def _stdconv_forward(x, rm, rv, training, momentum, eps, w1, w2, defer=None):
    """ReLU -> 1x1 conv (ReLUConvBN, operations.py) or FactorizedReduce (two stride-2 1x1
    convs on offset grids, channel-concatenated) -> BN(affine=False). Returns (out, state).
    ``defer`` (a list, inside a cell): the BN statistics are not folded here - the BN-apply reads
    the replicas itself and the fold segment is appended to ``defer`` for the cell's first node's
    fold; the backward then reads them folded."""
    x = x.contiguous()
    _selffold(x.device)
    N, Cin, H, W = _dims(x)
    fr = w2 is not None
    Cout = w1.shape[0] * (2 if fr else 1)
    Ho, Wo = (H // 2, W // 2) if fr else (H, W)
    cnt = N * Ho * Wo
    stats = zeros64(REP * 2 * Cout, x.device) if training else None
    z = torch.empty(N, Cout, Ho, Wo, device=x.device, dtype=ZDT)
    if fr:
        _K.pw_fwd([(x, w1, z, stats, 0, 0), (x, w2, z, stats, Cout // 2, 1)], 2)
    else:
        _K.pw_fwd([(x, w1, z, stats, 0, 0)], 1)
    bn = _bn(stats, rm, rv, cnt, training, eps, Cout)
    late = defer is not None and training and _defer(x.device)
    if training and not late:
        _fold64([(stats, 2 * Cout, 2 * Cout)], x.device)
    if late:
        defer.append((stats, 2 * Cout, 2 * Cout))
    out = torch.empty(z.shape, device=x.device)
    _K.combine_fwd([([z], [_unfolded(bn) if late else bn], [0], None, -1, None, [])], None, None, out, momentum,
                   training, False)
    return out, (x, z, w1, w2, bn, fr, Cout, training)


def _stdconv_backward(state, dout, need_x, sinks, keys, gx=None, first=True):
    """Returns the input gradient (or None); weight gradients through ``sinks``. ``gx`` (shaped
    like the input, maybe node-major): write the input gradient there - overwriting it when
    ``first``, else adding to it - instead of into a new buffer."""
    x, z, w1, w2, bn, fr, Cout, training = state
    dout = dout.contiguous()
    nred = 2 * Cout + 1
    red = zeros64(REP * nred, x.device)
    # deferred: the pointwise backward (its only consumer) sums the replicas in its prologue, and
    # nothing reads them later, so this fold goes away (the arena is re-zeroed every step)
    late = training and _defer(x.device)
    if training:
        _K.combine_bwd_reduce([(dout, [z], [bn], None, red, [0], -1, None)])
        if not late:
            _fold64([(red, nred, nred)], x.device)
    gs = (dout, z, red[:Cout], red[Cout:2 * Cout], bn, None, 0, REP if late else _R, nred)
    g1, s1 = sinks.get(w1, keys[0])
    given = gx is not None
    if fr:  # the two stride-2 grids leave 2 of 4 input pixels untouched: start from zeros
        if need_x and not given:
            gx = torch.zeros_like(x)
        elif need_x and first:
            gx.zero_()
        g2, s2 = sinks.get(w2, keys[1])
        _K.pw_bwd([(gs, w1, None, x, None, gx, g1, 0, 0, s1), (gs, w2, None, x, None, gx, g2, Cout // 2, 1, s2)],
                  2, 1, need_x)
    else:  # stride 1 covers every input pixel: the first writer overwrites gx (no fill)
        if need_x and not given:
            gx = torch.empty_like(x)
        _K.pw_bwd([(gs, w1, None, x, None, gx, g1, 0, 0, s1, first or not given)], 1, 1, need_x)
    return gx if need_x else None


class _StdConvBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rm, rv, training, momentum, eps, w1, w2):
        out, state = _stdconv_forward(x, rm, rv, training, momentum, eps, w1, w2)
        ctx.state = state
        ctx.save_for_backward(x, w1, *([w2] if w2 is not None else []))
        return out

    @staticmethod
    def backward(ctx, dout):
        sinks = _Sinks()
        grads = [None, None, None]
        gx = _stdconv_backward(ctx.state, dout, ctx.needs_input_grad[0], sinks, (1, 2))
        ctx.state = None
        sinks.finish(grads)
        return gx, None, None, None, None, None, grads[1], grads[2]


# --------------------------------------------------------------------------------- cell
class CellSpec:
    """Static description of one DARTS cell for :func:`cell_forward`: the two preprocess
    layers (``(kind, param names, bn name)``, kind ``std`` or ``fr``) and, per node, its
    edges as ``(EdgeSpec, param names, bn names, source state, alpha row)``."""

    def __init__(self, pre0, pre1, nodes, C):
        self.pre0, self.pre1, self.nodes, self.C = pre0, pre1, nodes, C
        self.names = list(pre0[1]) + list(pre1[1])
        for node in nodes:
            for _, pnames, _, _, _ in node:
                self.names += pnames
        self.index = {n: i for i, n in enumerate(self.names)}


def _cell_fwd(spec, s0, s1, wts, P, bn_of, training, momentum, eps):
    """A DARTS cell forward on the HIP kernels: preprocess(s0), preprocess(s1) (each input
    [N][C][H][W] or node-major), every node. Returns (O, state): O = the node outputs,
    node-major [nodes][N][C][H][W] - the cell output is kept as its nodes' buffers, never
    concatenated (the next cells' preprocess and the head read it node-major)."""
    late = []  # preprocess BN statistics folded by the first node's fold

    def pre(x, p):
        kind, pnames, bname = p
        rm, rv = bn_of(bname)
        if kind == "fr":
            return _stdconv_forward(x, rm, rv, training, momentum, eps, P[pnames[0]], P[pnames[1]], late)
        return _stdconv_forward(x, rm, rv, training, momentum, eps, P[pnames[0]], None, late)
    t0, st0 = pre(s0, spec.pre0)
    t1, st1 = pre(s1, spec.pre1)
    states = [t0, t1]
    N, C = t0.shape[0], spec.C
    nn_ = len(spec.nodes)
    S = [e[0].stride for e in spec.nodes[0]]
    Ho = (t0.shape[2] - 1) // max(S) + 1 if S else t0.shape[2]
    Wo = (t0.shape[3] - 1) // max(S) + 1 if S else t0.shape[3]
    O = torch.empty(nn_, N, C, Ho, Wo, device=t0.device)
    node_states = []
    for i, node in enumerate(spec.nodes):
        xs = [states[src] for _, _, _, src, _ in node]
        ws = [wts[row] for _, _, _, _, row in node]
        specs = [es for es, _, _, _, _ in node]
        bns = [[bn_of(b) for b in bnames] for _, _, bnames, _, _ in node]
        plist = [[P[n] for n in pnames] for _, pnames, _, _, _ in node]
        out, edges = _node_forward(xs, ws, specs, bns, plist, training, momentum, eps, out=O[i],
                                   extra_fold=late if i == 0 else ())
        states.append(out)
        node_states.append(edges)
    return O, (spec, training, st0, st1, node_states, states, wts)


def _cell_bwd(state, gO, sinks, pkey, gx0, first0, gx1, first1, need0, need1, alpha_rows=None):
    """The cell backward: ``gO`` = gradient of the node outputs (node-major, overwritten by the
    nodes' input-gradient kernels as scratch), nodes in reverse with one gradient buffer per cell
    state (the first kernel writing a buffer overwrites it, later ones accumulate), then both
    preprocess layers into ``gx0`` / ``gx1`` (None: new buffers) - overwriting when ``first0`` /
    ``first1``. Weight gradients through ``sinks`` under ``pkey(name)``. ``alpha_rows`` (a list):
    the edges' replicated d(softmax weight) go there as (f64 replicas, rstride, weight row) for the
    alpha-gradient kernel; otherwise they are folded and returned as a [rows, K] tensor.
    Returns (gs0, gs1, d softmax weights or None)."""
    spec, training, st0, st1, node_states, states, wts = state
    nn_ = len(spec.nodes)
    gS = [None, None] + [gO[i] for i in range(nn_)]
    first = [True, True] + [False] * nn_
    ga_rows = [None] * nn_
    cell_gw = []  # the nodes' unfolded d(alpha) replicas
    for i in reversed(range(nn_)):
        node = spec.nodes[i]
        edges = node_states[i]
        srcs = [src for _, _, _, src, _ in node]
        for src in srcs:
            if gS[src] is None:
                gS[src] = torch.empty_like(states[src])

        def take_first(k, srcs=srcs):
            f = first[srcs[k]]
            first[srcs[k]] = False
            return f

        _node_backward(edges, training, spec.C, gS[2 + i], lambda k, srcs=srcs: gS[srcs[k]], take_first, sinks,
                       lambda e, name, node=node: pkey(node[e.i][1][e.spec.pidx[name]]), cell_gw)
        if alpha_rows is not None:
            for e, (_, _, _, _, row) in zip(edges, node):
                alpha_rows.append((e.gw, e.w.numel(), wts[row], row))
        else:
            ga_rows[i] = [e.gw[:wts.shape[1]] for e in edges]
    for j in (0, 1):
        if first[j]:  # only "none" primitives read this state
            gS[j] = torch.zeros_like(states[j])
    gs0 = _stdconv_backward(st0, gS[0], need0, sinks, tuple(pkey(n) for n in spec.pre0[1]) + (None,), gx0, first0)
    gs1 = _stdconv_backward(st1, gS[1], need1, sinks, tuple(pkey(n) for n in spec.pre1[1]) + (None,), gx1, first1)
    gw = None
    if alpha_rows is None:
        if cell_gw:
            _K.fold_f64(cell_gw)  # d alpha: per rank
        gw = torch.cat([g for rows in ga_rows for g in rows]).view(wts.shape).to(torch.float32)
    return gs0, gs1, gw


class _Cell(torch.autograd.Function):
    """A whole cell - preprocess(s0), preprocess(s1), every node, the concat - as ONE autograd
    Function with a hand-scheduled backward (:func:`_cell_fwd` / :func:`_cell_bwd`); the whole
    network runs as one Function in :func:`network_loss`, which also drops this wrapper's concat
    and transpose copies."""

    @staticmethod
    def forward(ctx, meta, s0, s1, wts, *params):
        spec, bn_of, training, momentum, eps = meta
        P = dict(zip(spec.names, params))
        O, state = _cell_fwd(spec, s0, s1, wts, P, bn_of, training, momentum, eps)
        nn_, N, C, Ho, Wo = O.shape
        y = O.permute(1, 0, 2, 3, 4).reshape(N, nn_ * C, Ho, Wo)
        ctx.cell = state
        ctx.save_for_backward(s0, s1, wts, *params)
        return y

    @staticmethod
    def backward(ctx, dy):
        state = ctx.cell
        ctx.cell = None
        spec = state[0]
        saved = ctx.saved_tensors
        params = saved[3:]
        nn_ = len(spec.nodes)
        N, C = dy.shape[0], spec.C
        Ho, Wo = dy.shape[2], dy.shape[3]
        # node-major copy of the incoming gradient: one buffer per node state
        gO = dy.reshape(N, nn_, C * Ho * Wo).transpose(0, 1).contiguous().view(nn_, N, C, Ho, Wo)
        sinks = _Sinks()
        need = ctx.needs_input_grad
        grads = [None] * (4 + len(params))
        gs0, gs1, gw = _cell_bwd(state, gO, sinks, lambda n: 4 + spec.index[n], None, True, None, True, need[1],
                                 need[2])
        grads[1], grads[2] = gs0, gs1
        if need[3]:
            grads[3] = gw
        sinks.finish(grads)
        return tuple(grads)


def cell_forward(spec: CellSpec, s0, s1, wts, params: Sequence[torch.Tensor], bn_of, training: bool,
                 momentum: float = 0.1, eps: float = 1e-5):
    """A DARTS cell on the HIP kernels (see :class:`_Cell`). ``wts`` [rows, K] are the
    softmax weights of this cell type; ``params`` follow ``spec.names``; ``bn_of(name)`` gives
    the (running mean, running var) views of a BN layer."""
    return _Cell.apply((spec, bn_of, training, momentum, eps), s0, s1, wts, *params)


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


# --------------------------------------------------------------------------------- stem
class _StemConv(torch.autograd.Function):
    """Stem Conv2d(Cin, C_stem, 3, padding=1, bias=False) (reference
    ``examples/v1beta1/trial-images/darts-cnn-cifar10/model.py:90-93``) on the direct
    stem kernels: forward + weight gradient; the data gradient (never needed for the
    input image) falls back to ``torch.nn.grad.conv2d_input``."""

    @staticmethod
    def forward(ctx, x, w):
        x, w = x.contiguous(), w.contiguous()
        N, _, H, W = x.shape
        y = torch.empty(N, w.shape[0], H, W, device=x.device, dtype=x.dtype)
        _K.stem_conv_fwd(x, w, y)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        gx = gw = None
        if ctx.needs_input_grad[1]:
            chunks = stem_chunks(x, w.shape[0])
            partial = torch.empty(chunks, w.numel(), device=x.device, dtype=torch.float32)
            gw = torch.empty_like(w)
            _K.stem_conv_wgrad(x, dy, partial, gw)
        if ctx.needs_input_grad[0]:
            gx = torch.nn.grad.conv2d_input(x.shape, w, dy, padding=1)
        return gx, gw


def _stem_fwd(x, w, gamma, beta, rm, rv, momentum, eps):
    """Training-mode stem conv + affine BN (batch statistics): the conv accumulates the BN
    statistics in its epilogue, one fold + one combine_fwd apply the normalisation (running stats
    updated in the same launch). Returns (out, state)."""
    x, w = x.contiguous(), w.contiguous()
    N, _, H, W = x.shape
    C = w.shape[0]
    stats = zeros64(REP * 2 * C, x.device)
    z = torch.empty(N, C, H, W, device=x.device, dtype=x.dtype)
    _K.stem_conv_fwd_stats(x, w, z, stats)
    _fold([(stats, 2 * C, 2 * C)])  # always folded: the weight-gradient kernel reads replica 0
    bn = _bn(stats, rm, rv, N * H * W, True, eps, C)
    out = torch.empty_like(z)
    zs = z if ZDT == z.dtype else z.to(ZDT)  # the combine kernels read z in the intermediates' type
    _K.combine_fwd([([zs], [bn], [0], None, -1, None, [])], gamma, beta, out, momentum, True, False)
    return out, (x, w, gamma, beta, z, zs, bn, eps, stats)


def _stem_bwd(state, dout, sinks, keys, need):
    """The stem backward: one BN-backward reduction + fold, then the weight-gradient kernel forms
    the conv-output gradient on the fly and adds d gamma / d beta. ``keys`` = (w, gamma, beta)
    sink keys, ``need`` = (x, w, gamma, beta) flags; returns (gx or None, gw or None)."""
    x, w, gamma, beta, z, zs, bn, eps, stats = state
    dout = dout.contiguous()
    C = w.shape[0]
    nred = 2 * C + 1
    red = zeros64(REP * nred, x.device)
    _K.combine_bwd_reduce([(dout, [zs], [bn], None, red, [0], -1, None)])
    if not _selffold(x.device):
        _fold([(red, nred, nred)])
    gg, _ = sinks.get(gamma, keys[1]) if need[2] else (None, 0)
    gb, _ = sinks.get(beta, keys[2]) if need[3] else (None, 0)
    gw = gx = None
    if need[1] or need[2] or need[3]:
        chunks = stem_chunks(x, C)
        partial = torch.empty(chunks, w.numel(), device=x.device, dtype=torch.float32)
        if need[1]:  # straight into the weight's gradient row (registered replicated .grad, or a sink temp)
            gdst, _ = sinks.get(w, keys[0])
            _K.stem_conv_wgrad_bn(x, dout, z, red, stats, gamma, eps, gg, gb, partial, gdst, _world(), True)
        else:
            _K.stem_conv_wgrad_bn(x, dout, z, red, stats, gamma, eps, gg, gb, partial, torch.empty_like(w), _world())
    if need[0]:  # never for the input image; plain formula for completeness
        m = stats[:C] / z[:, 0].numel()
        var = (stats[C:2 * C] / z[:, 0].numel() - m * m).clamp_min(0)
        istd = torch.rsqrt(var.float() + eps).view(1, C, 1, 1)
        zhat = (z - m.float().view(1, C, 1, 1)) * istd
        m1 = (red[:C] / z[:, 0].numel()).float().view(1, C, 1, 1)
        m2 = (red[C:2 * C] / z[:, 0].numel()).float().view(1, C, 1, 1)
        dz = gamma.view(1, C, 1, 1) * istd * (dout - m1 - zhat * m2)
        gx = torch.nn.grad.conv2d_input(x.shape, w, dz, padding=1)
    return gx, gw


class _StemConvBN(torch.autograd.Function):
    """Stem Conv2d(Cin, C, 3, padding=1, bias=False) + BatchNorm2d(C) (affine, batch statistics)
    on the stem kernels (reference ``model.py:90-93``): :func:`_stem_fwd` / :func:`_stem_bwd`."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, rm, rv, momentum, eps):
        out, state = _stem_fwd(x, w, gamma, beta, rm, rv, momentum, eps)
        ctx.stem = state
        return out

    @staticmethod
    def backward(ctx, dout):
        state = ctx.stem
        ctx.stem = None
        need = ctx.needs_input_grad
        grads = [None] * 8
        sinks = _Sinks()
        gx, _ = _stem_bwd(state, dout, sinks, (1, 2, 3), need[:4])
        grads[0] = gx
        sinks.finish(grads)
        return tuple(grads)


def stem_conv_bn(x, w, gamma, beta, rm, rv, momentum=0.1, eps=1e-5):
    """Training-mode stem conv + BatchNorm (batch statistics, running stats updated)."""
    return _StemConvBN.apply(x, w, gamma, beta, rm, rv, momentum, eps)


@torch.no_grad()
def stem_bn_eval(z, gamma, beta, rm, rv, eps=1e-5):
    """Inference BatchNorm of the stem output with the running statistics (one combine_fwd)."""
    z = z.contiguous()
    N, C, H, W = z.shape
    out = torch.empty(z.shape, device=z.device)
    zs = z if z.dtype == ZDT else z.to(ZDT)
    _K.combine_fwd([([zs], [_bn(None, rm, rv, N * H * W, False, eps, C)], [0], None, -1, None, [])], gamma, beta, out,
                   0.0, False, False)
    return out


def stem_chunks(x: torch.Tensor, cout: int) -> int:
    """Pixel chunks of the weight-gradient grid: >= ~512 workgroups over (chunk, Cout),
    each thread covering a handful of pixels."""
    pixels = x.shape[0] * x.shape[2] * x.shape[3]
    return max(1, min(pixels // 1024, max(16, 1024 // cout)))


def stem_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 4
            and x.shape[1] in (1, 3) and tuple(w.shape[1:]) == (x.shape[1], 3, 3) and w.shape[0] <= 64
            and x.numel() < (1 << 31) // 64)


def stem_conv(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return _StemConv.apply(x, w)


# --------------------------------------------------------------------------------- head
class _Head(torch.autograd.Function):
    """Global average pool -> classifier -> cross-entropy (mean) as the fused HIP head
    (``csrc/hip/darts_head.hip``; reference ``model.py:156-161`` + ``nn.CrossEntropyLoss``):
    forward = per-sample workgroups + one loss reduction, backward = one launch writing the
    feature gradient and accumulating the classifier gradients into their replica rows."""

    @staticmethod
    def forward(ctx, x, w, b, y):
        x = x.contiguous()
        N, C = x.shape[:2]
        K = w.shape[0]
        dev = x.device
        pooled = torch.empty(N, C, device=dev)
        logits = torch.empty(N, K, device=dev)
        dl = torch.empty(N, K, device=dev)
        loss_n = torch.empty(N, device=dev)
        loss = torch.empty((), device=dev)
        _K.head_fwd(x, w, b, y, pooled, logits, dl, loss_n)
        _K.head_loss(loss_n, loss)
        ctx.save_for_backward(dl, pooled, w, b)
        ctx.xshape = x.shape
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)
        return loss, logits

    @staticmethod
    def backward(ctx, gloss, _glogits):
        dl, pooled, w, b = ctx.saved_tensors
        grads = [None, None, None, None]
        if gloss is None:
            return tuple(grads)
        need = ctx.needs_input_grad
        dev = dl.device
        x_like = torch.empty((), device=dev).expand(ctx.xshape)
        dx = torch.empty(ctx.xshape, device=dev) if need[0] else None
        sinks = _Sinks()
        gw, sw = sinks.get(w, 1) if need[1] else (None, 0)
        gb, sb = sinks.get(b, 2) if need[2] else (None, 0)
        _K.head_bwd(x_like, dl, pooled, w, gloss.reshape(()).contiguous().float(), dx, gw, sw, gb, sb)
        grads[0] = dx
        sinks.finish(grads)
        return tuple(grads)


def head_supported(x: torch.Tensor, w: torch.Tensor, y: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and w.dtype == torch.float32
            and w.dim() == 2 and w.shape[1] == x.shape[1] and x.shape[1] <= 1024 and w.shape[0] <= 64
            and y.dtype == torch.int64 and y.dim() == 1 and y.shape[0] == x.shape[0])


def head_loss(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, y: torch.Tensor):
    """(mean cross-entropy, logits) of ``linear(gap(x))`` against ``y``; logits carry no grad."""
    return _Head.apply(x, w, b, y.contiguous())


# --------------------------------------------------------------------------------- network
class NetSpec:
    """Static description of the supernet for :func:`network_loss`: the stem ``(conv, bn weight,
    bn bias, bn name)``, every cell (:class:`CellSpec`, reduction flag) and the head ``(weight,
    bias)``; ``names`` orders the parameter tensors passed to it."""

    def __init__(self, stem, cells, reduce, head):
        self.stem, self.cells, self.reduce, self.head = stem, list(cells), list(reduce), head
        names = list(stem[:3])
        for c in self.cells:
            names += c.names
        names += list(head)
        self.names = names
        self.index = {n: i for i, n in enumerate(names)}


def _alpha_grad(entries):
    """alpha_grad launches over (g replicas, rstride, weight row, destination row) entries, each
    destination row's entries in one launch (the kernel sums them per row, deterministically)."""
    groups = defaultdict(list)
    for ent in entries:
        groups[ent[3].data_ptr()].append(ent)
    chunk = []
    for rows in groups.values():
        if len(chunk) + len(rows) > 64:
            _K.alpha_grad(chunk, True)
            chunk = []
        chunk += rows
    if chunk:
        _K.alpha_grad(chunk, True)


class _Network(torch.autograd.Function):
    """The whole supernet - alpha softmax, stem conv + BN, every cell, head (gap, classifier,
    cross-entropy) - as ONE autograd Function with a hand-scheduled backward, so nothing between
    the HIP kernels is left to framework launches:

    * cell outputs stay node-major ([nodes][N][C][H][W], the nodes' own buffers): the next cells'
      preprocess and the head read them in that layout, so the forward concatenation and the
      backward transpose copies disappear (reference ``model.py:70`` torch.cat);
    * every cell state has one gradient buffer that its first consumer's kernel overwrites and later
      ones add to - the stem output's three and a cell output's two consumers need no autograd
      additions or fills;
    * the alpha softmax of both cell types is one launch (which also zeroes the step's f64 arena),
      and d(alpha) is one launch that sums the edges' replicated d(softmax weight) rows through the
      softmax Jacobian straight into the alpha leaves' gradient rows (no fold, cat, dtype copy,
      softmax backward or accumulation launches);
    * weight gradients go to the registered replicated buffers as before (:class:`_Sinks`).
    """

    @staticmethod
    def forward(ctx, meta, x, y, an, ar, *params):
        spec, bn_of, training, momentum, eps = meta
        P = dict(zip(spec.names, params))
        dev = x.device
        mats, outs = [an], [torch.empty_like(an)]
        if ar is not None:
            mats.append(ar)
            outs.append(torch.empty_like(ar))
        zero = None
        a = _ARENA
        if training and a.pending_zero and a.buf is not None and a.buf.device == dev:
            zero, a.pending_zero = a.buf, False
        _K.alpha_softmax(mats, outs, zero)
        wn, wr = outs[0], (outs[1] if ar is not None else None)
        conv, gamma, beta, bname = spec.stem
        rm, rv = bn_of(bname)
        if training:
            s, st_stem = _stem_fwd(x, P[conv], P[gamma], P[beta], rm, rv, momentum, eps)
        else:
            s, st_stem = stem_bn_eval(stem_conv(x, P[conv]), P[gamma], P[beta], rm, rv, eps), None
        tensors = [s]
        cells = []
        i0 = i1 = 0
        for cspec, red in zip(spec.cells, spec.reduce):
            O, st = _cell_fwd(cspec, tensors[i0], tensors[i1], wr if red else wn, P, bn_of, training, momentum, eps)
            tensors.append(O)
            cells.append((st, i0, i1, len(tensors) - 1, red))
            i0, i1 = i1, len(tensors) - 1
        feat = tensors[i1]
        hw, hb = spec.head
        N, C = _dims(feat)[:2]
        K = P[hw].shape[0]
        pooled = torch.empty(N, C, device=dev)
        logits = torch.empty(N, K, device=dev)
        dl = torch.empty(N, K, device=dev)
        loss_n = torch.empty(N, device=dev)
        loss = torch.empty((), device=dev)
        _K.head_fwd(feat, P[hw], P[hb], y, pooled, logits, dl, loss_n)
        _K.head_loss(loss_n, loss)
        ctx.net = (spec, P, training, st_stem, cells, tensors, i1, dl, pooled, an, ar)
        ctx.mark_non_differentiable(logits)
        ctx.set_materialize_grads(False)
        return loss, logits

    @staticmethod
    def backward(ctx, gloss, _glogits):
        spec, P, training, st_stem, cells, tensors, last, dl, pooled, an, ar = ctx.net
        ctx.net = None
        grads = [None] * (5 + len(spec.names))
        if gloss is None:
            return tuple(grads)
        need = ctx.needs_input_grad
        sinks = _Sinks()

        def key(n):
            return 5 + spec.index[n]
        g, first = {last: torch.empty_like(tensors[last])}, {last: False}
        hw, hb = spec.head
        gw, sw = sinks.get(P[hw], key(hw)) if need[key(hw)] else (None, 0)
        gb, sb = sinks.get(P[hb], key(hb)) if need[key(hb)] else (None, 0)
        _K.head_bwd(tensors[last], dl, pooled, P[hw], gloss.reshape(()).contiguous().float(), g[last], gw, sw, gb, sb)
        rows = []
        for st, i0, i1, io, red in reversed(cells):
            for i in (i0, i1):
                if i not in g:
                    g[i], first[i] = torch.empty_like(tensors[i]), True
            f0 = first[i0]
            f1 = first[i1] and i1 != i0  # the first cell's two inputs are both the stem output
            cell_rows = []
            _cell_bwd(st, g[io], sinks, key, g[i0], f0, g[i1], f1, True, True, cell_rows)
            first[i0] = first[i1] = False
            rows += [(r, red) for r in cell_rows]
        # d(alpha) straight into the leaves' gradient rows (or into returned tensors)
        dst = {}
        for red, leaf, idx in ((False, an, 3), (True, ar, 4)):
            if leaf is None or not need[idx]:
                continue
            if leaf.is_leaf and leaf.grad is not None and leaf.grad.is_contiguous() and leaf.grad.dtype == torch.float32:
                dst[red] = leaf.grad
            else:
                dst[red] = grads[idx] = torch.zeros_like(leaf)
        ents = [(gw_, rs, wrow, dst[red][row]) for (gw_, rs, wrow, row), red in rows if red in dst]
        if ents:
            _alpha_grad(ents)
        conv, gamma, beta, _ = spec.stem
        if training and st_stem is not None and 0 in g:
            flags = (False, need[key(conv)], need[key(gamma)], need[key(beta)])
            _stem_bwd(st_stem, g[0], sinks, (key(conv), key(gamma), key(beta)), flags)
        sinks.finish(grads)
        return tuple(grads)


# ------------------------------------------------------------------------- stacked passes
# Two network passes of identical structure (the +eps / -eps finite-difference Hessian passes of the
# architect step: same batch and shapes, their own weights, BN state and alpha-gradient leaves) are
# RECORDED - every launch and SyncBN fold they would issue goes to a tape instead of the device - and
# then replayed side by side: where both tapes hold the same edge-batched launch with identical
# non-entry arguments, the two entry lists go out as ONE launch (capacities in darts_ops.h are sized
# for two passes; by-value kernel arguments past 4 KB are fine on this stack); everything else is
# issued pass by pass in tape order. Each pass keeps its own stream order and no cross-pass
# dependency exists (disjoint buffers), so the result equals the two passes run one after the other.
# Under SyncBN the twin folds become one fold + cross-rank sum: one rendezvous instead of two.
# Reference: the architect's Hessian-vector product, examples/v1beta1/trial-images/darts-cnn-cifar10/
# architect.py:98-135 (two forward/backward passes at w +- eps dw').
_MERGE_CAP = {"dwpw_fwd": 16, "pw_fwd": 32, "pool_fwd": 16, "combine_bwd_reduce": 8, "pw_bwd": 32, "dw_bwd": 40,
              "pool_bwd": 16, "dw_bwd_multi": 40, "dwpw_fwd_multi": 40, "pool_fwd_multi": 16,
              "pool_bwd_multi": 16, "fold_f64": 128, "alpha_grad": 128, "__sync_fold__": 64}
_QUERIES = {"selffold_ready", "max_blocks", "stamps_compiled", "REP", "ZBF16", "OPTIM_MAX_PARTS"}


class _Recorder:
    """Stands in for the extension module (or the SyncBN object) while a pass is recorded."""

    def __init__(self, real, tape, sync=False):
        self._real, self._tape, self._sync = real, tape, sync

    def __getattr__(self, name):
        attr = getattr(self._real, name)
        if self._sync:
            if name != "fold":
                return attr
            name = "__sync_fold__"
        elif name in _QUERIES or not callable(attr):
            return attr

        def rec(*args, **kw):
            self._tape.append((name, args, kw))
            return None

        return rec


def _same(x, y) -> bool:
    if torch.is_tensor(x) or torch.is_tensor(y):
        return x is y
    if isinstance(x, (list, tuple)) and isinstance(y, (list, tuple)):
        return len(x) == len(y) and all(_same(a, b) for a, b in zip(x, y))
    return x == y


class stacked_passes:
    """``with stacked_passes() as sp: with sp.pass_(): ...; with sp.pass_(): ...`` - the launches of
    the two recorded passes are issued, merged where possible, when the outer block exits."""

    def __init__(self):
        self.tapes: List[list] = []
        self.stats = {"launches": 0, "merged": 0}

    def __enter__(self):
        return self

    @contextlib.contextmanager
    def pass_(self):
        global _K, _SYNC
        if EDGE_BWD or JOINT_POOL or SELFFOLD:
            # opt-in paths that branch on launch return values or attach per-launch fold tails:
            # the passes run live, one after the other
            yield
            return
        tape: list = []
        self.tapes.append(tape)
        real_k, real_sync = _K, _SYNC
        _K = _Recorder(real_k, tape)
        if real_sync is not None:
            _SYNC = _Recorder(real_sync, tape, sync=True)
        try:
            yield
        finally:
            _K, _SYNC = real_k, real_sync

    def _call(self, name, args, kw):
        self.stats["launches"] += 1
        if name == "__sync_fold__":
            _SYNC.fold(*args, **kw)
        else:
            getattr(_K, name)(*args, **kw)

    def __exit__(self, et, ev, tb):
        if et is not None:
            return False
        tapes = self.tapes
        if not tapes:
            return False
        if len(tapes) != 2 or len(tapes[0]) != len(tapes[1]) or any(a[0] != b[0] for a, b in zip(*tapes)):
            for t in tapes:  # not twins: replay one after the other
                for name, args, kw in t:
                    self._call(name, args, kw)
            return False
        self._replay_merged(tapes)
        return False

    def _replay_merged(self, tapes):
        for (name, aa, ka), (_, ab, kb) in zip(*tapes):
            cap = _MERGE_CAP.get(name)
            if (cap and aa and ab and isinstance(aa[0], list) and isinstance(ab[0], list)
                    and len(aa[0]) + len(ab[0]) <= cap and len(aa) == len(ab) and _same(aa[1:], ab[1:])
                    and _same(sorted(ka.items()), sorted(kb.items()))):
                self.stats["merged"] += 1
                self._call(name, (list(aa[0]) + list(ab[0]),) + tuple(aa[1:]), ka)
            else:
                self._call(name, aa, ka)
                self._call(name, ab, kb)


def network_loss(spec: NetSpec, x, y, params: Sequence[torch.Tensor], an, ar, bn_of, training: bool,
                 momentum: float = 0.1, eps: float = 1e-5):
    """(mean cross-entropy, logits) of the DARTS supernet on the HIP kernels as one Function
    (:class:`_Network`); ``an`` / ``ar``: the [rows, K] alpha matrices of the normal / reduction
    cells (``ar`` None for a one-layer net); ``params`` ordered as ``spec.names``."""
    return _Network.apply((spec, bn_of, training, momentum, eps), x, y, an, ar, *params)
