"""Locate the first non-finite value inside the captured ENAS child step.

Every HIP op wrapper (conv / depthwise / batch norm, forward and backward) is wrapped so
that, while the step is being captured, a check is captured after it: one int32 flag per
(op call, tensor) set when that tensor holds a non-finite value. The flags are zeroed
before each replay (an eager memset) and read after a replay that produced a non-finite
loss, which gives the first op - in capture order - whose input or output went bad.

argv: <mode> [variants] as in scripts/enas_capture_audit.py (default: sync)
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd.ops import batchnorm as hbn  # noqa: E402
from katib_amd.ops import conv as hconv  # noqa: E402
from katib_amd.ops import dwconv as hdw  # noqa: E402
import enas_capture_audit as A  # noqa: E402

FLAGS = torch.zeros(4096, dtype=torch.int32, device="cuda")
NAMES = []
KEEP = []  # "keep" mode: references to every HIP op's tensors (inspected after a bad replay)
CFG = {"mode": "flags"}


def _check(tag, tensors):
    if not torch.cuda.is_current_stream_capturing():
        return
    if CFG["mode"] == "keep":
        for j, t in enumerate(tensors):
            if torch.is_tensor(t) and t.is_floating_point() and t.numel():
                KEEP.append(("%s[%d] %s %s" % (tag, j, tuple(t.shape), t.dtype), t))
        return
    if CFG["mode"] == "none":
        return
    for j, t in enumerate(tensors):
        if torch.is_tensor(t) and t.is_floating_point() and t.numel():
            i = len(NAMES)
            NAMES.append("%s[%d] %s %s" % (tag, j, tuple(t.shape), t.dtype))
            FLAGS[i:i + 1].copy_((~torch.isfinite(t)).any().to(torch.int32).view(1))


def _wrap(cls, name):
    fwd, bwd = cls.forward, cls.backward

    def forward(ctx, *a):
        _check(name + ".fwd.in", a)
        out = fwd(ctx, *a)
        _check(name + ".fwd.out", out if isinstance(out, (tuple, list)) else (out,))
        return out

    def backward(ctx, *g):
        _check(name + ".bwd.gin", g)
        out = bwd(ctx, *g)
        _check(name + ".bwd.gout", out if isinstance(out, (tuple, list)) else (out,))
        return out
    cls.forward = staticmethod(forward)
    cls.backward = staticmethod(backward)


def poison_pool(graph):
    """Fill every byte of the graph's private memory pool with NaN (fp32 and bf16 alike):
    a correct graph writes every temporary before reading it, so its results must not
    change; a read-before-write inside the graph now reads NaN deterministically."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    pool = tuple(graph.pool())
    torch.cuda.synchronize()
    n = 0
    for seg in torch.cuda.memory._snapshot()["segments"]:
        if tuple(seg.get("segment_pool_id", (0, 0))) != pool:
            continue
        err = hip.hipMemsetD32(ctypes.c_void_p(seg["address"]), ctypes.c_int(0x7FC07FC0),
                               ctypes.c_size_t(seg["total_size"] // 4))
        assert err == 0, err
        n += seg["total_size"]
    torch.cuda.synchronize()
    return n


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "sync"
    parts = set(sys.argv[2].split("+")) if len(sys.argv) > 2 and sys.argv[2] != "-" else set()
    CFG["mode"] = sys.argv[3] if len(sys.argv) > 3 else "flags"
    CFG["trace"] = len(sys.argv) > 4 and "trace" in sys.argv[4]
    CFG["poison"] = len(sys.argv) > 4 and "poison" in sys.argv[4]
    A._variants(parts)
    if "gapmean" in parts:  # the workload's GAP reverted to adaptive_avg_pool2d(x, 1) (= mean over H, W)
        from katib_amd.workloads import enas_child as ec
        ec.global_avg_pool = lambda x: torch.nn.functional.adaptive_avg_pool2d(x, 1).flatten(1)
    _wrap(hbn._BNFn, "bn")
    _wrap(hconv._ConvFn, "conv")
    _wrap(hdw._DwFn, "dw")
    if CFG["mode"] == "keep":  # also every module's output and the gradient flowing into it
        orig_init = torch.nn.Module.__call__

        def call(self, *a, **kw):
            out = orig_init(self, *a, **kw)
            if torch.cuda.is_current_stream_capturing() and torch.is_tensor(out) and out.is_floating_point():
                name = type(self).__name__
                KEEP.append(("mod %s.out %s %s" % (name, tuple(out.shape), out.dtype), out))
                for j, x in enumerate(a):
                    if torch.is_tensor(x) and x.is_floating_point():
                        KEEP.append(("mod %s.in[%d] %s %s" % (name, j, tuple(x.shape), x.dtype), x))
                if out.requires_grad:
                    out.register_hook(lambda g, name=name: KEEP.append(
                        ("mod %s.grad_out %s %s" % (name, tuple(g.shape), g.dtype), g)))
            return out
        torch.nn.Module.__call__ = call
    step = A.build(True)
    env = {n: c.cell_contents for n, c in zip(step.fn.__code__.co_freevars, step.fn.__closure__ or ())}
    if "inner" in env:
        env = {n: c.cell_contents for n, c in zip(env["inner"].__code__.co_freevars, env["inner"].__closure__ or ())}
    acc, idx, model, opt = env["acc_buf"], env["idx"], env["model"], env["opt"]
    g = torch.Generator(device=idx.device).manual_seed(0)
    # state snapshot into preallocated buffers (no eager allocation between replays)
    state = [t for t in model.state_dict().values() if torch.is_tensor(t)]
    snap = None
    for r in range(200):
        if r == 5:  # optimizer state exists after the warmup / capture calls
            state += [v for st in opt.state.values() for v in st.values() if torch.is_tensor(v)]
            state.append(acc)
            snap = [torch.empty_like(t) for t in state]
        if snap is not None:
            for t, s_ in zip(state, snap):
                s_.copy_(t)
        FLAGS.zero_()
        idx.copy_(torch.randint(0, 4096, idx.shape, device=idx.device, generator=g))
        if CFG.get("poison") and step.graph is not None:
            nb = poison_pool(step.graph)
            if r < 6:
                print("POISON %d bytes of the graph pool before call %d" % (nb, r), flush=True)
        step()
        if mode == "sync":
            torch.cuda.synchronize()
        after = float(acc[0])
        if r < 12 and CFG.get("trace"):
            pf = all(bool(torch.isfinite(p_).all()) for p_ in model.parameters())
            print("TRACE call %d graph=%s calls=%d loss_sum=%s params_finite=%s" % (
                r, step.graph is not None, step.calls, after, pf), flush=True)
        pbad = CFG["mode"] == "keep" and not all(bool(torch.isfinite(p_).all()) for p_ in model.parameters())
        if step.graph is not None and (not math.isfinite(after) or pbad) and CFG["mode"] == "keep":
            print("LOCATE first non-finite loss/params at call %d" % r, flush=True)
            pids = {p_.data_ptr() for p_ in model.parameters()}  # updated at the end of the replay: skip
            bad = [(i, n) for i, (n, t) in enumerate(KEEP)
                   if t.data_ptr() not in pids and not bool(torch.isfinite(t).all())]
            print("LOCATE kept %d tensors (capture order), %d non-finite; first %s" % (len(KEEP), len(bad), bad[:10]),
                  flush=True)
            for i, (n, t) in enumerate(KEEP[:bad[0][0] + 1] if bad else []):
                if t.data_ptr() not in pids:
                    print("LOCATE   #%d %s finite=%s" % (i, n, bool(torch.isfinite(t).all())), flush=True)
            return
        if step.graph is not None and not math.isfinite(after) and snap is not None:
            print("LOCATE first non-finite loss at replay %d" % r, flush=True)
            if CFG["mode"] == "flags":
                f = FLAGS[:len(NAMES)].cpu()
                bad = [NAMES[i] for i in range(len(NAMES)) if f[i]]
                print("LOCATE %d checks, %d non-finite; first %s" % (len(NAMES), len(bad), bad[:12]), flush=True)
            if CFG["mode"] == "keep":
                bad = [n for n, t in KEEP if not bool(torch.isfinite(t).all())]
                print("LOCATE kept %d tensors, %d non-finite; first %s" % (len(KEEP), len(bad), bad[:10]),
                      flush=True)
            # determinism: restore the state and replay the same batch again, three times
            outs = []
            for k in range(3):
                for t, s_ in zip(state, snap):
                    t.copy_(s_)
                torch.cuda.synchronize()
                step.graph.replay()
                torch.cuda.synchronize()
                outs.append(float(acc[0]))
            for t, s_ in zip(state, snap):
                t.copy_(s_)
            torch.cuda.synchronize()
            step.fn()  # eager, same state and batch
            torch.cuda.synchronize()
            print("LOCATE re-replays from the snapshot: %s; eager rerun: %s" % (outs, float(acc[0])), flush=True)
            return
    print("LOCATE no non-finite loss in 200 replays (%d checks, %d kept)" % (len(NAMES), len(KEEP)), flush=True)


if __name__ == "__main__":
    main()
