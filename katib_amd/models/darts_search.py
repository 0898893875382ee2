"""DARTS search step: second-order architect + weight step, data-parallel, graph-captured.

Per step (reference ``run_trial.py:177-222`` + ``architect.py:30-135``):

1. FWD1/BWD1  L_train(w)                 -> g1            (all-reduce)
   w' = w - xi * (mu*m + g1 + wd*w),  alpha' = alpha
2. FWD2/BWD2  L_valid(w', alpha')        -> d_alpha, d_w' (all-reduce)
3. eps = 0.01/||d_w'||; w += eps d_w';  FWD3/BWD3 L_train -> d_alpha+
   w -= 2 eps d_w';                      FWD4/BWD4 L_train -> d_alpha-
   w += eps d_w'
   alpha.grad = d_alpha - xi (d_alpha+ - d_alpha-) / (2 eps)  (all-reduce, merged)
   Adam(alpha) with L2 weight decay, betas (0.5, 0.999)
4. FWD5/BWD5  L_train(w)                 -> g5            (all-reduce)
   clip ||g5|| <= w_grad_clip;  SGD(momentum mu, weight decay wd) on w

Data parallelism is *within* the trial (the reference DARTS trial is single-GPU
only, ``run_trial.py:81-96``): each rank runs the step on its own shard of the
train/valid batches and the four gradient vectors are averaged with one RCCL
all-reduce each over flat buffers. BN statistics stay per-rank (like DDP).

With ``capture=True`` every segment between collectives is captured once as a
HIP graph (``torch.cuda.CUDAGraph``) and replayed; at world size 1, or when the
all-reduces run as the one-shot xGMI kernel (``parallel/xgmi.py``, capturable),
the whole step is a single graph. All scalars (lr, eps, Adam step) live on the device so
the replay needs no host synchronisation.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from ..parallel.comm import Comm
from .darts import BNState, DartsLayout, DartsNetwork, accuracy

# validation batches merged per captured eval forward (eval-mode BN normalises every sample with
# the running statistics, so k batches of n give the same losses and correct counts as one of k*n;
# at B5 sizes the forward is launch / latency bound: per 128-image batch 0.54 ms at k = 1, 0.31 at 4,
# 0.27 at 8, profiles/darts_eval_group_ab_r04.log; 0.252 at 16 and 32, darts_eval_group_ab_r05.log)
EVAL_GROUP = 16


def eval_groups(batches, group: int = 0):
    """(x, y) batches -> (x, y) groups of ``group`` (default EVAL_GROUP) consecutive batches
    concatenated (the last group may be shorter). Validation loss / accuracy weighted by the
    group's sample count equal the per-batch ones."""
    group = max(1, group or EVAL_GROUP)
    buf = []
    for b in batches:
        buf.append(b)
        if len(buf) == group:
            yield (buf[0][0], buf[0][1]) if group == 1 else (torch.cat([x for x, _ in buf]), torch.cat([y for _, y in buf]))
            buf = []
    if buf:
        yield (buf[0][0], buf[0][1]) if len(buf) == 1 else (torch.cat([x for x, _ in buf]), torch.cat([y for _, y in buf]))

DEFAULTS = dict(w_lr=0.025, w_lr_min=0.001, w_momentum=0.9, w_weight_decay=3e-4, w_grad_clip=5.0,
                alpha_lr=3e-4, alpha_weight_decay=1e-3)


class _Leaves:
    """Parameter leaves that are views of a flat buffer, with grads accumulating
    into a flat grad buffer (bucket views)."""

    def __init__(self, views: Dict[str, torch.Tensor], grad_views: Dict[str, torch.Tensor]):
        self.views = views
        for k, v in views.items():
            v.requires_grad_(True)
            v.grad = grad_views[k]
        self.list = list(views.values())


class DartsSearch:
    # Measurement hook, never an environment switch: True drops the two finite-difference
    # forward/backward passes (the alpha gradient is then WRONG). Only a profiling script sets it,
    # on its own instance, to bound what stacking both passes into the same edge-batched launches
    # could save (profiles/darts_hessian_stack_bound_r05.log); the step warns when it is on.
    debug_skip_hessian_passes = False

    def __init__(self, layout: DartsLayout, device, comm: Optional[Comm] = None, seed: int = 2,
                 settings: Optional[Dict] = None, capture: bool = False, ops=None, sync_bn: bool = False,
                 hessian: str = "concurrent"):
        self.layout = layout
        self.device = torch.device(device)
        self.comm = comm or Comm(device=self.device)
        if self.device.type == "cuda":
            self.comm.enable_xgmi()  # collective; RCCL stays the fallback
        self.s = dict(DEFAULTS)
        if settings:
            self.s.update({k: float(v) for k, v in settings.items() if k in DEFAULTS})
        self.capture = capture and self.device.type == "cuda"
        self.net = DartsNetwork(layout, ops=ops)
        g = torch.Generator().manual_seed(seed)
        dev, f32 = self.device, torch.float32
        nW, nA = layout.n_weights, layout.n_alphas
        W = torch.zeros(nW, dtype=f32)
        layout.init_weights(W, g)
        A = 1e-3 * torch.randn(nA, generator=g)
        # all ranks start from identical weights (rank 0's)
        self.W = W.to(dev)
        self.A = A.to(dev)
        self.comm.broadcast_(self.W)
        self.comm.broadcast_(self.A)
        self.Wv = torch.zeros_like(self.W)
        self.Av = torch.zeros_like(self.A)
        # weight-gradient buckets: [R][nW], row 0 is the gradient; with the HIP edge kernels
        # R = hip_darts.REP replica rows absorb the cross-workgroup atomics and are folded
        # into row 0 after every backward pass (_fold)
        self.hd = None
        if self.device.type == "cuda" and self.net.ops.backend() == "hip":
            self.hd = self.net.ops.hip_module()
        # SyncBN (data parallel): BN statistics over the global batch, so a W-rank step at 128/W
        # images per rank computes the single-GPU step at batch 128 (the reference's BN,
        # operations.py:62,96,117,139) instead of per-rank BN over 128/W images
        self.sync_bn = bool(sync_bn) and self.comm.distributed
        self._hsync = None
        if self.sync_bn:
            self.net.sync = self.comm
            if self.hd is not None:
                self._hsync = self.hd.SyncBN(self.comm)  # collective
                if not self._hsync.capturable:
                    self.capture = False  # its collectives sit inside the passes
            elif self.capture and not self.comm.graph_capturable([]):  # collective (RCCL capture probe)
                self.capture = False  # torch-op SyncBN all-reduces inside the passes, on the host
        R = self.hd.REP if self.hd is not None else 1
        self.gW_rep = torch.zeros(R, nW, device=dev)
        self.gWv_rep = torch.zeros(R, nW, device=dev)
        if self.hd is not None:
            self.hd.register_grad_replicas(self.gW_rep)
            self.hd.register_grad_replicas(self.gWv_rep)
        self.gW = self.gW_rep[0]  # model weight grads (BWD1 / BWD5)
        self.gWv = self.gWv_rep[0]  # virtual weight grads (BWD2)
        self.gAv = torch.zeros_like(self.A)  # virtual alpha grads (BWD2)
        self.gA = torch.zeros_like(self.A)  # alpha grads (BWD3/4/5 scratch)
        self.gAp = torch.zeros_like(self.A)
        self.alpha_grad = torch.zeros_like(self.A)
        self.mom = torch.zeros_like(self.W)
        self.adam_m = torch.zeros_like(self.A)
        self.adam_v = torch.zeros_like(self.A)
        self.adam_t = torch.zeros((), device=dev)
        self.lr = torch.full((), self.s["w_lr"], device=dev)
        self.eps = torch.zeros((), device=dev)
        self.bn = BNState(layout, dev)
        self.bn_v = BNState(layout, dev)
        self.loss_out = torch.zeros((), device=dev)
        self.logits_out = None
        # leaves: weights are views of W / W'; alphas are ONE [rows, K] leaf per cell type
        # (normal, reduce) so each forward runs one softmax per cell type
        self.Pw = _Leaves(layout.views(self.W), layout.views(self.gW))
        self.Pv = _Leaves(layout.views(self.Wv), layout.views(self.gWv))
        self.An, self.Ar = layout.alpha_views(self.A)  # per-node views (genotype)
        self.Aw, self.gAw = self._alpha_leaves(self.A, self.gA)
        self.Avw, _ = self._alpha_leaves(self.Av, self.gAv)
        self.W_detached = layout.views(self.W.detach())
        # finite-difference Hessian passes (HIP path), w + eps dw' and w - eps dw', each with its own
        # weight copy, alpha-gradient leaves and BN running statistics (merged by one kernel after both):
        # * "concurrent" (default): two branches of the captured graph (side stream fork / join); under SyncBN the
        #   side branch folds through a workspace of its own (calls of one workspace must pair up in the
        #   same order on every rank, which two concurrently running branches do not guarantee);
        # * "stacked": both passes recorded and issued as ONE pass of edge-batched launches
        #   (hip_darts.stacked_passes: both entry lists per launch, one SyncBN rendezvous per fold pair);
        #   measured 0.24 ms slower than "concurrent" on B5 (profiles/darts_hessian_stacked_ab_r06.log);
        # * "sequential": one in-place perturbation after the other (also the torch-ops path).
        if hessian not in ("stacked", "concurrent", "sequential"):
            raise ValueError("hessian must be stacked, concurrent or sequential")
        if self.device.type != "cuda" or self.hd is None:
            hessian = "sequential"
        self._hsync_side = None
        if hessian == "concurrent" and self.sync_bn:
            if self._hsync is not None and self._hsync.capturable:
                # collective, same order on every rank; on the RCCL path the side branch gets a
                # communicator of its own (two concurrently running branches must not share one)
                side = self.comm if self._hsync.ws is not None else self.comm.subgroup()
                self._hsync_side = self.hd.SyncBN(side)
            if self._hsync_side is None or not self._hsync_side.capturable:
                hessian = "sequential"
        self.hessian = hessian
        self.hess_concurrent = hessian == "concurrent"
        if hessian in ("stacked", "concurrent"):
            self.Wp = torch.empty_like(self.W)
            self.Wm = torch.empty_like(self.W)
            self.Wp_views = layout.views(self.Wp)
            self.Wm_views = layout.views(self.Wm)
            self.Aw_p, _ = self._alpha_leaves(self.A, self.gAp)
            self.bn_plus = BNState(layout, dev)
            self.bn_zero = BNState(layout, dev)
            self._one_side = torch.ones((), device=dev)  # the second pass's own unit upstream gradient
        if hessian == "concurrent":
            self._side = torch.cuda.Stream(device=dev)
        # fused optimizer kernels (csrc/hip/darts_optim.hip) on the HIP path:
        # virtual step, Hessian perturbations, Adam on alphas and clipped SGD are one launch each
        self.K = self.hd._K if self.hd is not None else None
        self._parts = (torch.zeros(self.K.OPTIM_MAX_PARTS, dtype=torch.float64, device=dev)
                       if self.K is not None else None)
        self._one = None
        self.graphs = None
        self.rendezvous_per_step = None  # cross-rank rendezvous per step (set by the first step)
        self.rendezvous_serial_per_step = None  # ... of them on the critical path (not on a concurrent branch)
        self.rendezvous_in_graph = None
        self.static = None
        self._eval_graphs = {}  # (x shape, y shape, dtypes) -> (graph, static x, static y, [loss, top1, top5])
        self.stack_stats = None  # launches issued / merged by the last stacked Hessian pair

    def _alpha_leaves(self, A, gA):
        rows, K = self.layout.n_alpha_rows, len(self.layout.prims)
        leaves, grads = [], []
        for t in range(2 if self.layout.has_reduce else 1):
            v = A[t * rows * K:(t + 1) * rows * K].view(rows, K)
            g = gA[t * rows * K:(t + 1) * rows * K].view(rows, K)
            v.requires_grad_(True)
            v.grad = g
            leaves.append(v)
            grads.append(g)
        return leaves, grads

    @staticmethod
    def _fixed(leaves):
        return [a.detach() for a in leaves]

    def _arch(self, leaves):
        return leaves[0], (leaves[1] if len(leaves) > 1 else [])

    # ------------------------------------------------------------------ pieces
    def _loss(self, x, y, P, an, ar, bn):
        return self.net.forward_loss(x, y, P, an, ar, bn, training=True)

    def _fold(self, rep):
        if self.hd is not None:
            self.hd.fold(rep)

    def _backward(self, loss, inputs):
        """loss.backward(inputs=...) with a preallocated unit upstream gradient (autograd's implicit
        ones_like would be a fill launch per pass)."""
        if self._one is None or self._one.device != loss.device:
            self._one = torch.ones((), device=loss.device)
        torch.autograd.backward(loss, grad_tensors=self._one, inputs=inputs)

    def _seg_virtual(self, tx, ty):
        """FWD1/BWD1 -> gW (not yet reduced)."""
        if self.K is None:  # the fused optimizer kernels leave gW zeroed after reading it
            self.gW.zero_()
        # weight-only pass: detached alphas, so the network Function neither computes nor writes
        # d(alpha) (backward(inputs=...) does not reach a custom Function's needs_input_grad)
        loss, _ = self._loss(tx, ty, self.Pw.views, *self._arch(self._fixed(self.Aw)), self.bn)
        self._backward(loss, self.Pw.list)
        self._fold(self.gW_rep)

    def _seg_unrolled(self, vx, vy):
        """virtual step + FWD2/BWD2 -> gAv, gWv."""
        s = self.s
        if self.K is not None:  # one launch: w', alpha' and the zeroed virtual gradients
            # ... and gW zeroed after its read: BWD5 accumulates into it next
            self.K.optim_virtual_step(self.Wv, self.W, self.mom, self.gW, self.lr, s["w_momentum"],
                                      s["w_weight_decay"], self.Av, self.A, self.gWv, self.gAv, True)
        else:
            with torch.no_grad():
                # w' = w - xi*(mu*m + g + wd*w)
                self.Wv.copy_(self.mom).mul_(s["w_momentum"]).add_(self.gW).add_(self.W, alpha=s["w_weight_decay"])
                self.Wv.mul_(-self.lr).add_(self.W)
                self.Av.copy_(self.A)
            self.gWv.zero_()
            self.gAv.zero_()
        loss, _ = self._loss(vx, vy, self.Pv.views, *self._arch(self.Avw), self.bn_v)
        self._backward(loss, self.Pv.list + self.Avw)
        self._fold(self.gWv_rep)

    def _seg_hessian(self, tx, ty):
        """+/- eps perturbations, FWD3/BWD3 and FWD4/BWD4 w.r.t. alphas only."""
        if self.K is not None and self.hessian in ("stacked", "concurrent"):
            K, args = self.K, (self.eps, self._parts)
            nparts = K.optim_sumsq(self.gWv, self._parts)
            tail = (self.gA, self.gAp, self.gAv, self.alpha_grad, self.lr, self.Wp, self.Wm, self.bn.buf,
                    self.bn_plus.buf, self.bn_zero.buf, self.net.momentum)
            # eps = 0.01/||dw'||; Wp = w + eps dw', Wm = Wp - 2 eps dw'; zeroed d(alpha)+-; BN snapshots
            K.optim_hessian_split(3, self.W, self.gWv, *args, nparts, *tail)
            if self.debug_skip_hessian_passes:  # measurement only (wrong alpha gradient): see the class attribute
                if not getattr(self, "_warned_skip", False):
                    import warnings

                    warnings.warn("DartsSearch.debug_skip_hessian_passes is set: the architecture gradient is wrong")
                    self._warned_skip = True
                K.optim_hessian_split(2, self.W, self.gWv, *args, nparts, *tail)
                return
            if self.hessian == "stacked":
                with self.hd.stacked_passes() as sp:
                    with sp.pass_():
                        loss, _ = self._loss(tx, ty, self.Wp_views, *self._arch(self.Aw_p), self.bn_plus)
                        torch.autograd.backward(loss, grad_tensors=self._one_side, inputs=self.Aw_p)
                    with sp.pass_():
                        loss, _ = self._loss(tx, ty, self.Wm_views, *self._arch(self.Aw), self.bn)
                        self._backward(loss, self.Aw)
                self.stack_stats = sp.stats
                K.optim_hessian_split(2, self.W, self.gWv, *args, nparts, *tail)
                return
            main = torch.cuda.current_stream()
            self._side.wait_stream(main)
            with torch.cuda.stream(self._side), self._scope(self._hsync_side):  # the +eps pass on its own branch
                loss, _ = self._loss(tx, ty, self.Wp_views, *self._arch(self.Aw_p), self.bn_plus)
                torch.autograd.backward(loss, grad_tensors=self._one_side, inputs=self.Aw_p)
            loss, _ = self._loss(tx, ty, self.Wm_views, *self._arch(self.Aw), self.bn)
            self._backward(loss, self.Aw)
            main.wait_stream(self._side)
            # alpha grad = d(alpha) - xi (d+ - d-) / (2 eps); BN running stats as after both sequential passes
            K.optim_hessian_split(2, self.W, self.gWv, *args, nparts, *tail)
            return
        if self.K is not None:
            K, args = self.K, (self.eps, self._parts)
            nparts = K.optim_sumsq(self.gWv, self._parts)
            tail = (self.gA, self.gAp, self.gAv, self.alpha_grad, self.lr)
            K.optim_hessian(0, self.W, self.gWv, *args, nparts, *tail)  # eps = 0.01/||dw'||; w += eps dw'
            loss, _ = self._loss(tx, ty, self.W_detached, *self._arch(self.Aw), self.bn)
            loss.backward(inputs=self.Aw)
            K.optim_hessian(1, self.W, self.gWv, *args, nparts, *tail)  # w -= 2 eps dw'; d+ saved
            loss, _ = self._loss(tx, ty, self.W_detached, *self._arch(self.Aw), self.bn)
            loss.backward(inputs=self.Aw)
            K.optim_hessian(2, self.W, self.gWv, *args, nparts, *tail)  # w += eps dw'; alpha grad
            return
        with torch.no_grad():
            self.eps.copy_(0.01 / self.gWv.norm())
            self.W.add_(self.gWv * self.eps)
        self.gA.zero_()
        loss, _ = self._loss(tx, ty, self.W_detached, *self._arch(self.Aw), self.bn)
        loss.backward(inputs=self.Aw)
        with torch.no_grad():
            self.gAp.copy_(self.gA)
            self.W.sub_(self.gWv * (2.0 * self.eps))
        self.gA.zero_()
        loss, _ = self._loss(tx, ty, self.W_detached, *self._arch(self.Aw), self.bn)
        loss.backward(inputs=self.Aw)
        with torch.no_grad():
            self.W.add_(self.gWv * self.eps)
            # alpha.grad = d_alpha - xi * (d+ - d-) / (2 eps)
            h = (self.gAp - self.gA) / (2.0 * self.eps)
            torch.sub(self.gAv, h * self.lr, out=self.alpha_grad)

    def _seg_alpha_step(self):
        """Adam(alpha_lr, betas=(0.5, 0.999), weight_decay) on alphas."""
        s = self.s
        b1, b2 = 0.5, 0.999
        if self.K is not None:  # one workgroup; also zeroes gA for the weight pass
            self.K.optim_adam(self.A, self.alpha_grad, self.adam_m, self.adam_v, self.adam_t, s["alpha_lr"], b1, b2,
                              s["alpha_weight_decay"], 1e-8, self.gA)
            return
        with torch.no_grad():
            g = self.alpha_grad + s["alpha_weight_decay"] * self.A
            self.adam_t.add_(1.0)
            self.adam_m.mul_(b1).add_(g, alpha=1 - b1)
            self.adam_v.mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1 = 1 - torch.pow(b1, self.adam_t)
            bc2 = 1 - torch.pow(b2, self.adam_t)
            denom = (self.adam_v.sqrt() / bc2.sqrt()).add_(1e-8)
            self.A.sub_(self.adam_m / denom * (s["alpha_lr"] / bc1))

    def _seg_weight(self, tx, ty):
        """FWD5/BWD5 -> gW (+ alpha grads ignored), logits/loss kept for metrics."""
        if self.K is None:
            self.gW.zero_()  # (the fused virtual step left it zeroed)
            self.gA.zero_()  # (the fused Adam launch already zeroed it)
        loss, logits = self._loss(tx, ty, self.Pw.views, *self._arch(self._fixed(self.Aw)), self.bn)
        self._backward(loss, self.Pw.list)
        self._fold(self.gW_rep)
        if self.hd is not None:
            # keep the step's own loss / logits tensors (no copies): under graph capture their
            # memory is fixed, so every replay refreshes them in place
            self.loss_out, self.logits_out = loss.detach(), logits.detach()
            return
        with torch.no_grad():
            self.loss_out.copy_(loss.detach())
            if self.logits_out is None or self.logits_out.shape != logits.shape:
                self.logits_out = torch.empty_like(logits)
            self.logits_out.copy_(logits.detach())

    def _seg_weight_update(self):
        s = self.s
        if self.K is not None:
            nparts = self.K.optim_sumsq(self.gW, self._parts)
            # gW left zeroed for the next step's BWD1 (no fill launches at the passes' starts)
            self.K.optim_sgd_clip(self.W, self.gW, self.mom, self.lr, self._parts, nparts, s["w_grad_clip"],
                                  s["w_momentum"], s["w_weight_decay"], True)
            return
        with torch.no_grad():
            total = self.gW.norm()
            coef = torch.clamp(s["w_grad_clip"] / (total + 1e-6), max=1.0)
            self.gW.mul_(coef)
            d = self.gW.add(self.W, alpha=s["w_weight_decay"])
            self.mom.mul_(s["w_momentum"]).add_(d)
            self.W.sub_(self.mom * self.lr)

    # ------------------------------------------------------------------ step
    def _segments(self):
        """List of (callable, collective-after) in order."""
        c = self.comm
        hd = None
        if self.device.type == "cuda":
            from ..ops import darts as dops

            if dops.backend() == "hip":
                from ..ops import hip_darts as hd
        begin = (lambda: hd.arena_begin(self.device, deferred_zero=self.net.net_function)) if hd else (lambda: None)
        end = hd.arena_end if hd else (lambda: None)
        return [
            (lambda: (begin(), self._seg_virtual(self.static["tx"], self.static["ty"])), [self.gW]),
            (lambda: self._seg_unrolled(self.static["vx"], self.static["vy"]), [self.gWv, self.gAv]),
            (lambda: self._seg_hessian(self.static["tx"], self.static["ty"]), [self.alpha_grad]),
            (lambda: (self._seg_alpha_step(), self._seg_weight(self.static["tx"], self.static["ty"])), [self.gW]),
            (lambda: (self._seg_weight_update(), end()), []),
        ]

    def _scope(self, sync=None):
        if self.hd is not None:
            return self.hd.sync_scope(sync if sync is not None else self._hsync)
        import contextlib

        return contextlib.nullcontext()

    def _run_eager(self):
        with self._scope():
            for fn, colls in self._segments():
                fn()
                for t in colls:
                    self.comm.allreduce_mean_(t)

    def _rendezvous(self) -> int:
        """Cross-rank rendezvous issued so far: gradient all-reduces and SyncBN folds, on every
        communicator / one-shot workspace of this search."""
        n = self.comm.calls
        for sy in (self._hsync, self._hsync_side):
            if sy is None:
                continue
            if sy.ws is not None:
                n += sy.folds  # one-shot fold + cross-rank sum: not a Comm call
            elif sy.comm is not self.comm:
                n += sy.comm.calls
        return n

    def _side_folds(self) -> int:
        sy = self._hsync_side
        if sy is None:
            return 0
        return sy.folds if sy.ws is not None else sy.comm.calls

    def _build_graphs(self):
        segs = self._segments()
        # merge segments with no host-side collective in between: all of them at world size 1
        # or when the all-reduces run as the (capturable) one-shot xGMI kernel
        whole = self.comm.graph_capturable([t for _, colls in segs for t in colls])
        groups, cur = [], []
        for fn, colls in segs:
            if whole:
                cur.append(lambda fn=fn, colls=colls: (fn(), [self.comm.allreduce_mean_(t) for t in colls]))
            else:
                cur.append(fn)
                if colls and self.comm.distributed:
                    groups.append((cur, colls))
                    cur = []
        if cur:
            groups.append((cur, []))
        # warm up on a side stream (required before capture), then capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._snapshot_state()
                self._run_eager()
                self._restore_state()
        torch.cuda.current_stream().wait_stream(s)
        graphs = []
        n0 = self._rendezvous()
        side0 = self._side_folds()
        for fns, colls in groups:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), self._scope():
                for fn in fns:
                    fn()
            graphs.append((g, colls))
        self.graphs = graphs
        # inside the graphs (captured once, replayed every step) + the host-side ones per replay
        self.rendezvous_per_step = self._rendezvous() - n0 + (
            sum(len(c) for _, c in graphs) if self.comm.distributed else 0)
        # the concurrent Hessian branch's folds run beside the main branch's: not on the critical path
        self.rendezvous_serial_per_step = self.rendezvous_per_step - (self._side_folds() - side0)
        self.rendezvous_in_graph = not any(c for _, c in graphs)

    def _state_tensors(self):
        return [self.W, self.A, self.mom, self.adam_m, self.adam_v, self.adam_t, self.bn.mean, self.bn.var,
                self.bn_v.mean, self.bn_v.var]

    def _snapshot_state(self):
        self._saved = [t.clone() for t in self._state_tensors()]

    def _restore_state(self):
        with torch.no_grad():
            for t, s in zip(self._state_tensors(), self._saved):
                t.copy_(s)
        self._saved = None

    def set_lr(self, lr: float):
        self.lr.fill_(lr)

    def sync_bn_stats(self):
        """Average the BN running statistics over the ranks (each rank tracks its own shard's
        batch statistics, like DDP without SyncBN) so that every rank validates with the same
        model. The mean of per-rank running variances ignores the spread of the per-rank
        means, a second-order term at equal shard sizes. (With SyncBN every rank already
        holds the global-batch running statistics.)"""
        if self.comm.distributed and not self.sync_bn:
            self.comm.allreduce_mean_(self.bn.mean)
            self.comm.allreduce_mean_(self.bn.var)

    def step(self, tx, ty, vx, vy):
        if self.static is None:
            self.static = {"tx": tx.clone(), "ty": ty.clone(), "vx": vx.clone(), "vy": vy.clone()}
        else:
            self.static["tx"].copy_(tx)
            self.static["ty"].copy_(ty)
            self.static["vx"].copy_(vx)
            self.static["vy"].copy_(vy)
        if self.capture:
            if self.graphs is None:
                # the first capture consumes the current batch: _build_graphs restores the state
                # after its warm-up runs, so the replay below performs this step exactly once
                self._build_graphs()
            for g, colls in self.graphs:
                g.replay()
                for t in colls:
                    self.comm.allreduce_mean_(t)
        else:
            n0, side0 = self._rendezvous(), self._side_folds()
            self._run_eager()
            self.rendezvous_per_step = self._rendezvous() - n0
            self.rendezvous_serial_per_step = self.rendezvous_per_step - (self._side_folds() - side0)
            self.rendezvous_in_graph = False
        return self.loss_out

    # ------------------------------------------------------------------ eval / genotype
    @torch.no_grad()
    def _evaluate(self, x, y):
        loss, logits = self.net.forward_loss(x, y, self.layout.views(self.W), *self._arch(self.Aw), self.bn,
                                             training=False)
        top1, top5 = accuracy(logits, y)
        return loss, top1, top5

    @torch.no_grad()
    def evaluate(self, x, y):
        """Validation forward (BN in eval mode, reference ``run_trial.py:225-255``) ->
        (loss, top1, top5) device scalars. With ``capture=True`` the forward is replayed
        from a HIP graph captured once per batch shape: the validation pass runs every
        epoch over the whole valid split, and launched eagerly its ~100 small kernels are
        host-bound (B5: 1.65 ms per batch, ~15% of the search wall clock)."""
        if not self.capture:
            return self._evaluate(x, y)
        key = (tuple(x.shape), tuple(y.shape), x.dtype, y.dtype)
        ent = self._eval_graphs.get(key)
        if ent is None:
            sx, sy = x.clone(), y.clone()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):  # warm-up before capture (allocator, kernel selection)
                    self._evaluate(sx, sy)
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = torch.stack(self._evaluate(sx, sy))
            ent = self._eval_graphs[key] = (g, sx, sy, out)
        g, sx, sy, out = ent
        sx.copy_(x)
        sy.copy_(y)
        g.replay()
        r = out.clone()  # the graph's output buffer is overwritten by the next replay
        return r[0], r[1], r[2]

    def train_metrics(self, y):
        top1, top5 = accuracy(self.logits_out, y)
        return float(self.loss_out), float(top1), float(top5)

    def genotype(self):
        from .darts import Genotype

        sp = self.layout.space
        normal = sp.parse([a.detach() for a in self.An], k=2)
        reduce = sp.parse([a.detach() for a in self.Ar], k=2) if self.Ar else []
        concat = range(2, 2 + self.layout.N)
        return Genotype(normal=normal, normal_concat=concat, reduce=reduce, reduce_concat=concat)
