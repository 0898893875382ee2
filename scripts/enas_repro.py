"""Bisect of the ENAS child training collapse seen in the enas-cifar10 experiment on MI355X:
one architecture, 3 epochs, with / without the captured train step (CapturedStep).
argv: "<capture>[:variant]" with variant in
  noeval  - no validation passes between epochs
  torchbn - nn.BatchNorm2d instead of the HIP NHWC batch norm
  noconv  - PyTorch conv instead of the HIP implicit-GEMM conv
  nodw    - PyTorch depthwise conv instead of the HIP depthwise kernels
  adamfe  - torch Adam (foreach, capturable) instead of the fused one
  probe   - captured, but every replay is checked: at the first non-finite loss the step is
            re-run eagerly from a snapshot of the state before it, with forward/backward hooks
            naming the first module whose output / input gradient is non-finite
variants combine with '+': samestream (warmup and capture on one persistent side stream),
blas (rocBLAS instead of hipBLASLt), nocache (autocast cache_enabled=False), nodrop (no dropout)"""
import functools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd.ops import batchnorm as hbn  # noqa: E402
from katib_amd.ops import conv as hconv  # noqa: E402
from katib_amd.ops import dwconv as hdw  # noqa: E402
from katib_amd.workloads import common  # noqa: E402
from katib_amd.workloads import enas_child  # noqa: E402

_orig_call = common.CapturedStep.__call__


def _closure(fn):
    return {n: c.cell_contents for n, c in zip(fn.__code__.co_freevars, fn.__closure__ or ())}


def _finite(t):
    return bool(torch.isfinite(t).all())


def _same_stream_call(self):
    """CapturedStep with one persistent side stream for the warmup runs and the capture."""
    if self.graph is None:
        if not hasattr(self, "_s"):
            self._s = torch.cuda.Stream()
        self._s.wait_stream(torch.cuda.current_stream())
        if self.calls < self.warmup:
            with torch.cuda.stream(self._s):
                out = self.fn()
            torch.cuda.current_stream().wait_stream(self._s)
            self.calls += 1
            return out
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self._s):
            self.out = self.fn()
    self.graph.replay()
    return self.out


_base = [_orig_call]


def _probe_call(self):
    if self.graph is None:
        return _base[0](self)
    env = _closure(self.fn)
    if "inner" in env:  # CapturedStep(no_miopen=True) wraps the step
        env = _closure(env["inner"])
    model, opt, acc = env["model"], env["opt"], env["acc_buf"]
    self.nstep = getattr(self, "nstep", 0) + 1
    l0 = float(acc[0])
    tens = [t for t in model.state_dict().values()] + [
        v for st in opt.state.values() for v in st.values() if torch.is_tensor(v)]
    snap = [t.detach().clone() for t in tens]
    self.graph.replay()
    l1 = float(acc[0])
    if math.isfinite(l1) or not math.isfinite(l0):
        return self.out
    print("PROBE first non-finite loss at replay %d (loss sum before %.4f)" % (self.nstep, l0), flush=True)
    bad_w = [n for n, p in model.named_parameters() if not _finite(p)]
    bad_g = [n for n, p in model.named_parameters() if p.grad is not None and not _finite(p.grad)]
    print("PROBE after replay: non-finite params %d %s, grads %d %s" % (len(bad_w), bad_w[:6], len(bad_g), bad_g[:6]))
    with torch.no_grad():
        for t, s in zip(tens, snap):
            t.copy_(s)
    acc[0].fill_(l0)
    first = []

    def fhook(name):
        def h(m, i, o):
            if torch.is_tensor(o) and not _finite(o) and not first:
                first.append("fwd " + name)
        return h

    def bhook(name):
        def h(m, gi, go):
            for g in gi:
                if g is not None and not _finite(g):
                    first.append("bwd " + name)
                    break
        return h

    hs = []
    for n, m in model.named_modules():
        hs.append(m.register_forward_hook(fhook(n)))
        hs.append(m.register_full_backward_hook(bhook(n)))
    try:
        self.fn()
    except Exception as e:  # full backward hooks can refuse views; report and go on
        print("PROBE eager rerun raised", repr(e)[:300])
    for h in hs:
        h.remove()
    torch.cuda.synchronize()
    print("PROBE eager rerun from the snapshot: loss sum %.4f, first non-finite %s" % (float(acc[0]), first[:4]))
    bad_g = [n for n, p in model.named_parameters() if p.grad is not None and not _finite(p.grad)]
    print("PROBE eager rerun grads non-finite: %d %s" % (len(bad_g), bad_g[:6]), flush=True)
    raise SystemExit(0)


import math  # noqa: E402

cfg = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "enas_repro_arch.json")))
orig = dict(bn=hbn.BatchNorm2d.forward, conv=hconv.supported, dw=hdw.supported, adam=torch.optim.Adam,
            autocast=torch.autocast, blas=torch.backends.cuda.preferred_blas_library(),
            drop=torch.nn.Dropout.forward)


class _AdamForeach(torch.optim.Adam):
    def __init__(self, params, **kw):
        kw.pop("fused", None)
        super().__init__(params, foreach=True, **kw)


for spec in sys.argv[1:] or ["1", "0"]:
    capture, _, variant = spec.partition(":")
    print("=== capture", capture, variant, flush=True)
    hbn.BatchNorm2d.forward, hconv.supported, hdw.supported = orig["bn"], orig["conv"], orig["dw"]
    enas_child.torch.optim.Adam = orig["adam"]
    parts = set(variant.split("+"))
    _base[0] = _same_stream_call if "samestream" in parts else _orig_call
    common.CapturedStep.__call__ = _probe_call if "probe" in parts else _base[0]
    torch.backends.cuda.preferred_blas_library("cublas" if "blas" in parts else orig["blas"])
    enas_child.torch.autocast = (functools.partial(orig["autocast"], cache_enabled=False) if "nocache" in parts
                                 else orig["autocast"])
    torch.nn.Dropout.forward = (lambda self, x: x) if "nodrop" in parts else orig["drop"]
    if "torchbn" in parts:
        hbn.BatchNorm2d.forward = lambda self, x, residual=None, relu=False: torch.nn.BatchNorm2d.forward(self, x)
    if "noconv" in parts:
        hconv.supported = lambda *a, **k: False
    if "nodw" in parts:
        hdw.supported = lambda *a, **k: False
    if "adamfe" in parts:
        enas_child.torch.optim.Adam = _AdamForeach
    extra = ["--num-valid=0"] if variant == "noeval" else []
    try:
        enas_child.main(extra + ["--num_epochs=3", "--num-train=20000", "--capture=" + capture,
                                 "--architecture=" + json.dumps(cfg["architecture"]), "--nn_config=" + cfg["nn_config"]])
    except SystemExit:
        pass
