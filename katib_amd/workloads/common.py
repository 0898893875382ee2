"""Shared pieces of the built-in trial workloads: device selection, learnable synthetic
datasets resident in HBM, HIP-graph-captured train steps, and metric printing in the
default collector format (``name=value``).

Synthetic data (no network in the target environment): every dataset is generated
from a fixed seed by a *teacher* so that hyperparameters matter - a random linear
teacher with label noise for MNIST-shaped vectors, overlapping multi-modal
class patterns with random translations and label noise for CIFAR-shaped images, and a
sparse first-order Markov chain for token streams. None of them saturates: the earlier
single-template image teacher was fitted to >0.999 after one epoch by every ResNet trial,
so an HPO experiment could not tell its trials apart.
"""

from __future__ import annotations

import os
import time
from typing import Callable, Dict, Optional, Tuple

import torch


def device() -> torch.device:
    if torch.cuda.is_available():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def process_start_time() -> float:
    """Wall-clock time this process was created (fork), from /proc (10 ms resolution)."""
    try:
        with open("/proc/self/stat") as f:
            start_ticks = int(f.read().rsplit(")", 1)[1].split()[19])
        with open("/proc/stat") as f:
            btime = next(int(ln.split()[1]) for ln in f if ln.startswith("btime"))
        return btime + start_ticks / os.sysconf("SC_CLK_TCK")
    except (OSError, ValueError, StopIteration, IndexError):
        return float("nan")


def phase(name: str, t: Optional[float] = None):
    """Cold-trial phase breakdown (``KATIB_AMD_TRIAL_PHASES=1``): print ``katib-phase <name>
    <wall time>`` (no ``=``, so the metrics collector ignores it); bench_trials.py pairs the lines
    with the scheduler's launch and completion times."""
    if os.environ.get("KATIB_AMD_TRIAL_PHASES") == "1":
        print("katib-phase %s %.6f" % (name, time.time() if t is None else t), flush=True)


def report(**metrics):
    print(" ".join("%s=%s" % (k, _fmt(v)) for k, v in metrics.items()), flush=True)


def _fmt(v):
    if isinstance(v, float):
        return "%.6g" % v
    return str(v)


# ----------------------------------------------------------------------------- datasets
def teacher_vectors(n: int, dim: int = 784, classes: int = 10, seed: int = 0, dev=None, noise: float = 0.5,
                    label_noise: float = 0.05):
    """x ~ N(0, 1); y = argmax(x @ T + noise) for a fixed random linear teacher T, then a
    fraction ``label_noise`` of the labels replaced by random ones (accuracy caps near
    ``1 - 0.9 * label_noise``). Over the TPE example's ranges the MLP's accuracy after 3
    epochs spans ~0.15 (lr 0.3 diverges) to ~0.85, so the search has something to rank."""
    g = torch.Generator().manual_seed(seed)
    T = torch.randn(dim, classes, generator=g) / dim ** 0.5
    if dev is not None and torch.device(dev).type == "cuda":
        # drawn on the device (same seed -> same data in every trial): the host draw + 220 MB copy
        # was ~0.2 s of each cold B1 trial
        gd = torch.Generator(device=dev).manual_seed(seed + 7919)
        x = torch.randn(n, dim, generator=gd, device=dev)
        y = (x @ T.to(dev) + noise * torch.randn(n, classes, generator=gd, device=dev) / dim ** 0.5).argmax(1)
        flip = torch.rand(n, generator=gd, device=dev) < label_noise
        return x, torch.where(flip, torch.randint(0, classes, (n,), generator=gd, device=dev), y)
    x = torch.randn(n, dim, generator=g)
    y = (x @ T + noise * torch.randn(n, classes, generator=g) / dim ** 0.5).argmax(1)
    flip = torch.rand(n, generator=g) < label_noise
    y = torch.where(flip, torch.randint(0, classes, (n,), generator=g), y)
    return x.to(dev), y.to(dev)


def pattern_images(n: int, shape=(3, 32, 32), classes: int = 10, seed: int = 0, dev=None, noise: float = 1.5,
                   dtype=torch.float32, modes: int = 3, shift: int = 4, label_noise: float = 0.1):
    """CIFAR-10-shaped images that do not saturate: every class is a mixture of ``modes``
    prototypes, each prototype = a shared texture from a small common bank (so classes
    overlap) + a weaker class-specific pattern; every sample is one prototype with random
    amplitude, a random translation of up to ``shift`` pixels (so the model has to be
    translation-tolerant, not memorise pixels) and Gaussian noise; a fraction
    ``label_noise`` of the labels is random. The best attainable accuracy is below
    ``1 - 0.9 * label_noise``, and how close a trial gets depends on its learning rate,
    width and epochs - the signal HyperBand / median-stop / PBT need to rank trials."""
    g = torch.Generator().manual_seed(seed)
    C, H, W = shape
    up = lambda t: torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=False)  # noqa: E731
    bank = up(torch.randn(6, C, H // 4, W // 4, generator=g))
    own = up(torch.randn(classes * modes, C, H // 8, W // 8, generator=g))
    mix = torch.randint(0, bank.shape[0], (classes * modes,), generator=g)
    protos = bank[mix] + 0.6 * own  # [classes * modes, C, H, W]
    y = torch.randint(0, classes, (n,), generator=g)
    out = torch.empty(n, C, H, W, dtype=dtype, device=dev)
    # on a GPU the per-sample draws run on the device with their own generator (same seed -> same
    # data on every trial): generating 60k images on the host took ~4 s of each ResNet trial's
    # start-up, with 8 trials sharing the node's CPUs
    on_gpu = dev is not None and torch.device(dev).type == "cuda"
    gs = torch.Generator(device=dev).manual_seed(seed + 7919) if on_gpu else g
    sdev = dev if on_gpu else None
    protos_s, y_s = (protos.to(dev), y.to(dev)) if on_gpu else (protos, y)
    chunk = 16384 if on_gpu else 4096
    for i in range(0, n, chunk):
        yi = y_s[i:i + chunk]
        m = len(yi)
        pid = yi * modes + torch.randint(0, modes, (m,), generator=gs, device=sdev)
        xi = protos_s[pid] * (0.5 + torch.rand(m, 1, 1, 1, generator=gs, device=sdev))
        if shift:
            dy = torch.randint(-shift, shift + 1, (m,), generator=gs, device=sdev)
            dx = torch.randint(-shift, shift + 1, (m,), generator=gs, device=sdev)
            rows = (torch.arange(H, device=sdev).view(1, H) - dy.view(m, 1)) % H  # [m, H]
            cols = (torch.arange(W, device=sdev).view(1, W) - dx.view(m, 1)) % W
            xi = xi[torch.arange(m, device=sdev).view(m, 1, 1, 1), torch.arange(C, device=sdev).view(1, C, 1, 1),
                    rows.view(m, 1, H, 1), cols.view(m, 1, 1, W)]
        xi = xi + noise * torch.randn(m, C, H, W, generator=gs, device=sdev)
        out[i:i + chunk] = xi.to(device=dev, dtype=dtype)
    flip = torch.rand(n, generator=g) < label_noise
    y = torch.where(flip, torch.randint(0, classes, (n,), generator=g), y)
    return out, y.to(dev)


def markov_tokens(n_tokens: int, vocab: int = 50257, seed: int = 0, dev=None, fanout: int = 8):
    """Token stream from a sparse first-order Markov chain (each token has ``fanout``
    successors): learnable, with entropy ~log(fanout)."""
    g = torch.Generator().manual_seed(seed)
    succ = torch.randint(0, vocab, (vocab, fanout), generator=g)
    chains = 1024
    steps = (n_tokens + chains - 1) // chains
    toks = torch.empty(chains, steps, dtype=torch.long)
    state = torch.randint(0, vocab, (chains,), generator=g)
    for i in range(steps):  # 1024 independent chains walked in lock-step
        toks[:, i] = state
        state = succ[state, torch.randint(0, fanout, (chains,), generator=g)]
    return toks.reshape(-1)[:n_tokens].to(dev)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] -> [N, C] average as ONE pooling window (``avg_pool2d`` with the whole plane
    as the kernel), not ``adaptive_avg_pool2d(x, 1)``: for output 1x1 PyTorch lowers that to
    ``mean`` over (H, W), and on a channels-last bf16 activation the mean is a strided
    reduction whose cross-workgroup path (a global staging buffer plus semaphores reset by a
    memset before the kernel) reads its staging buffer before it is written when replayed
    from a HIP graph on this ROCm stack: with the graph's memory pool poisoned with NaN
    before a replay, that ``mean`` is the first op with a non-finite output
    (scripts/enas_nan_locate.py, profiles/enas_child_capture_rootcause_r03.log). That was
    the captured ENAS child step's NaN: stale staging data from earlier replays usually
    averages to finite garbage, occasionally to NaN/Inf, and the eager validation between
    epochs (or a host sync between replays) changed what the stale memory held."""
    return torch.nn.functional.avg_pool2d(x, (x.shape[2], x.shape[3])).flatten(1)


# ----------------------------------------------------------------------------- graphs
class CapturedStep:
    """Capture ``fn()`` (a full train step reading static input buffers) into a HIP
    graph after ``warmup`` eager runs on a side stream; replay afterwards. Falls back
    to eager execution on CPU or when ``enabled`` is False.

    ``no_miopen``: run the step (warmup, capture and eager) with MIOpen disabled, so a
    convolution / batch-norm fallback takes PyTorch's native kernels instead of MIOpen
    solvers inside a captured graph."""

    def __init__(self, fn: Callable[[], torch.Tensor], enabled: bool = True, warmup: int = 3,
                 no_miopen: bool = False):
        if no_miopen:
            inner = fn

            def fn():
                with torch.backends.cudnn.flags(enabled=False):
                    return inner()
        self.fn = fn
        self.enabled = enabled and torch.cuda.is_available()
        self.warmup = warmup
        self.graph = None
        self.out = None
        self.calls = 0

    def __call__(self):
        if not self.enabled:
            return self.fn()
        if self.graph is None:
            if self.calls < self.warmup:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    out = self.fn()
                torch.cuda.current_stream().wait_stream(s)
                self.calls += 1
                return out
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self.fn()
        self.graph.replay()
        return self.out


class Timer:
    def __init__(self):
        self.t0 = time.time()

    def elapsed(self) -> float:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        return time.time() - self.t0
