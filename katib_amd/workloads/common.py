"""Shared pieces of the built-in trial workloads: device selection, learnable synthetic
datasets resident in HBM, HIP-graph-captured train steps, and metric printing in the
default collector format (``name=value``).

Synthetic data (no network in the target environment): every dataset is generated
from a fixed seed by a *teacher* so that hyperparameters matter - a random linear
teacher for MNIST-shaped vectors, class-conditional spatial patterns for
CIFAR-shaped images, and a sparse first-order Markov chain for token streams.
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


def report(**metrics):
    print(" ".join("%s=%s" % (k, _fmt(v)) for k, v in metrics.items()), flush=True)


def _fmt(v):
    if isinstance(v, float):
        return "%.6g" % v
    return str(v)


# ----------------------------------------------------------------------------- datasets
def teacher_vectors(n: int, dim: int = 784, classes: int = 10, seed: int = 0, dev=None, noise: float = 0.5):
    """x ~ N(0, 1); y = argmax(x @ T + noise) for a fixed random teacher T."""
    g = torch.Generator().manual_seed(seed)
    T = torch.randn(dim, classes, generator=g) / dim ** 0.5
    x = torch.randn(n, dim, generator=g)
    y = (x @ T + noise * torch.randn(n, classes, generator=g) / dim ** 0.5).argmax(1)
    return x.to(dev), y.to(dev)


def pattern_images(n: int, shape=(3, 32, 32), classes: int = 10, seed: int = 0, dev=None, noise: float = 1.0,
                   dtype=torch.float32):
    """Per-class smooth spatial template + Gaussian noise (CIFAR-10 shaped)."""
    g = torch.Generator().manual_seed(seed)
    C, H, W = shape
    base = torch.randn(classes, C, H // 4, W // 4, generator=g)
    tmpl = torch.nn.functional.interpolate(base, size=(H, W), mode="bilinear", align_corners=False)
    y = torch.randint(0, classes, (n,), generator=g)
    out = torch.empty(n, C, H, W, dtype=dtype, device=dev)
    chunk = 4096
    for i in range(0, n, chunk):
        yi = y[i:i + chunk]
        xi = tmpl[yi] + noise * torch.randn(len(yi), C, H, W, generator=g)
        out[i:i + chunk] = xi.to(device=dev, dtype=dtype)
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
