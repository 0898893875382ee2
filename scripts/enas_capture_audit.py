"""Root-cause probe for the ENAS child's HIP-graph NaN (VERDICT r2 'Next round' item 2).

Two experiments on the captured ENAS child train step (scripts/enas_repro_arch.json):

1. Pointer audit. While the step is captured, every tensor argument of every HIP-kernel
   binding call (conv / depthwise / batch norm) is recorded with its op and argument index.
   After capture the caching allocator's snapshot tells, for each pointer, whether it lies in
   the graph's private pool, in a persistent tensor (parameters, gradients, optimizer state,
   module buffers, static inputs) or in an ordinary eager block - the last kind is memory the
   graph keeps using after the eager owner freed it, which eager work between replays then
   overwrites.
2. Replay variants: N replays with (a) nothing between them, (b) a host sync only, (c) eager
   allocations + writes of garbage (NaN) into fresh eager memory between replays. A NaN that
   appears only under (c) confirms that the graph reads memory outside its pool.

argv: audit | replay  (default: both)
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd.ops import batchnorm as hbn  # noqa: E402
from katib_amd.ops import conv as hconv  # noqa: E402
from katib_amd.workloads import common  # noqa: E402
from katib_amd.workloads import enas_child  # noqa: E402

RECORD = []


class _Proxy:
    """Wraps the HIP extension module: records tensor args of calls made during capture."""

    def __init__(self, k):
        self._k = k

    def __getattr__(self, name):
        f = getattr(self._k, name)
        if not callable(f):
            return f

        def call(*a, **kw):
            if torch.cuda.is_current_stream_capturing():
                for i, t in enumerate(list(a) + list(kw.values())):
                    if torch.is_tensor(t) and t.is_cuda:
                        RECORD.append((name, i, t.data_ptr(), t.untyped_storage().nbytes(), tuple(t.shape)))
            return f(*a, **kw)
        return call


def _install():
    k = hconv.kernels()
    px = _Proxy(k)
    hconv._K = px
    hbn._K = px


def _segments():
    snap = torch.cuda.memory._snapshot()
    segs = []
    for s in snap["segments"]:
        segs.append((s["address"], s["address"] + s["total_size"], s.get("segment_pool_id", (0, 0)),
                     [(b["address"], b["size"], b["state"]) for b in s["blocks"]]))
    return segs


def build(capture=True, steps=0):
    cfg = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "enas_repro_arch.json")))
    box = {}
    orig_init = common.CapturedStep.__init__

    def init(self, fn, *a, **kw):
        orig_init(self, fn, *a, **kw)
        box["step"] = self
    common.CapturedStep.__init__ = init
    try:
        enas_child.main(["--num_epochs=0", "--num-train=4096", "--num-valid=0", "--capture=%d" % int(capture),
                         "--architecture=" + json.dumps(cfg["architecture"]), "--nn_config=" + cfg["nn_config"]])
    finally:
        common.CapturedStep.__init__ = orig_init
    return box["step"]


def audit():
    _install()
    step = build()
    env = {n: c.cell_contents for n, c in zip(step.fn.__code__.co_freevars, step.fn.__closure__ or ())}
    if "inner" in env:
        env = {n: c.cell_contents for n, c in zip(env["inner"].__code__.co_freevars, env["inner"].__closure__ or ())}
    for _ in range(4):  # 3 warmups + capture
        step()
    torch.cuda.synchronize()
    model, opt = env["model"], env["opt"]
    persistent = []
    for t in list(model.parameters()) + list(model.buffers()):
        persistent.append((t.data_ptr(), t.untyped_storage().nbytes(), "param/buffer"))
        if t.grad is not None:
            persistent.append((t.grad.data_ptr(), t.grad.untyped_storage().nbytes(), "grad"))
    for st in opt.state.values():
        for v in st.values():
            if torch.is_tensor(v) and v.is_cuda:
                persistent.append((v.data_ptr(), v.untyped_storage().nbytes(), "optim"))
    for name in ("tx", "ty", "idx", "acc_buf"):
        t = env.get(name)
        if torch.is_tensor(t):
            persistent.append((t.untyped_storage().data_ptr(), t.untyped_storage().nbytes(), name))
    segs = _segments()
    pools = {}
    bad = []
    for op, i, ptr, nbytes, shape in RECORD:
        where = None
        for p0, n, kind in persistent:
            if p0 <= ptr < p0 + n:
                where = kind
                break
        if where is None:
            for a, b, pool, blocks in segs:
                if a <= ptr < b:
                    state = [st for ba, bs, st in blocks if ba <= ptr < ba + bs]
                    where = "pool%s/%s" % (tuple(pool), state[0] if state else "?")
                    break
        where = where or "unmapped"
        pools[where] = pools.get(where, 0) + 1
        if not (where.startswith("pool") and not where.startswith("pool(0, 0)")) and where not in (
                "param/buffer", "grad", "optim", "tx", "ty", "idx", "acc_buf"):
            bad.append((op, i, hex(ptr), shape, where))
    print("AUDIT %d recorded tensor args; by location: %s" % (len(RECORD), pools), flush=True)
    for b in bad[:40]:
        print("AUDIT outside the graph pool:", b, flush=True)
    print("AUDIT suspicious args: %d" % len(bad), flush=True)


def _variants(parts):
    """Swap HIP op families for PyTorch ones (same switches as scripts/enas_repro.py)."""
    from katib_amd.ops import dwconv as hdw

    if "torchbn" in parts:
        hbn.BatchNorm2d.forward = lambda self, x, residual=None, relu=False: torch.nn.BatchNorm2d.forward(self, x)
    if "noconv" in parts:
        hconv.supported = lambda *a, **k: False
    if "nodw" in parts:
        hdw.supported = lambda *a, **k: False
    if "adamfe" in parts:
        class _AdamForeach(torch.optim.Adam):
            def __init__(self, params, **kw):
                kw.pop("fused", None)
                super().__init__(params, foreach=True, **kw)
        enas_child.torch.optim.Adam = _AdamForeach


def replay(mode, n=200, capture=True, tag=""):
    step = build(capture)
    env = {n_: c.cell_contents for n_, c in zip(step.fn.__code__.co_freevars, step.fn.__closure__ or ())}
    if "inner" in env:
        env = {n_: c.cell_contents for n_, c in zip(env["inner"].__code__.co_freevars, env["inner"].__closure__ or ())}
    acc, idx = env["acc_buf"], env["idx"]
    g = torch.Generator(device=idx.device).manual_seed(0)
    first = None
    for r in range(n):
        idx.copy_(torch.randint(0, 4096, idx.shape, device=idx.device, generator=g))
        step()
        if mode == "sync":
            torch.cuda.synchronize()
        elif mode == "alloc":
            junk = [torch.full((1 << 16,), float("nan"), device=idx.device) for _ in range(64)]
            del junk
        elif mode == "allocbig":
            junk = torch.full((64 << 20,), float("nan"), device=idx.device)
            del junk
        if r % 10 == 9 or r == n - 1:
            v = float(acc[0])
            if not math.isfinite(v) and first is None:
                first = r
                break
    print("REPLAY mode=%s capture=%d %s replays=%d first_nonfinite=%s loss_sum=%s"
          % (mode, int(capture), tag, n, first, float(acc[0])), flush=True)


if __name__ == "__main__":
    what = sys.argv[1:] or ["audit", "replay"]
    if what[:1] == ["_one"]:
        what = what
    elif "audit" in what:
        audit()
    if "replay" in what:
        for mode in ("none", "sync", "alloc", "allocbig"):
            replay(mode)
    for w in (what if what[:1] != ["_one"] else []):  # "<mode>:<capture 0|1>[:variants]": one child each
        if w.count(":") >= 1:
            import subprocess

            r = subprocess.run([sys.executable, __file__, "_one", w], capture_output=True, text=True, timeout=300)
            print("\n".join(ln for ln in (r.stdout + r.stderr).splitlines() if ln.startswith("REPLAY") or
                            "Error" in ln)[-2000:] or "rc=%d" % r.returncode, flush=True)
    if what[:1] == ["_one"]:
        mode, cap, var = (what[1].split(":") + [""])[:3]
        parts = set(var.split("+")) if var else set()
        _variants(parts)
        replay(mode, capture=cap == "1", tag=var)
