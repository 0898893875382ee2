"""HIP-graph hygiene checks.

A captured graph owns a private memory pool for its temporaries. A correct graph writes
every temporary before reading it within one replay, so the values left in the pool by
earlier replays (or by anything else) must not matter. :func:`poison_graph_pool` fills the
whole pool with NaN (0x7FC07FC0: NaN as fp32 and as two bf16) so that any read-before-write
inside the graph turns the next replay's results non-finite deterministically, instead of
once in a while when stale data happens to be bad. This is how the round-2 ENAS child NaN was
root-caused (scripts/enas_nan_locate.py): PyTorch's cross-workgroup reductions (``mean`` /
``sum`` over the non-innermost dims of channels-last bf16 tensors) read their staging buffer
before writing it when replayed from a graph on this ROCm stack.
"""

from __future__ import annotations

import ctypes

import torch

_HIP = None
POISON_WORD = 0x7FC07FC0


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    return _HIP


def poison_graph_pool(graph: "torch.cuda.CUDAGraph") -> int:
    """Fill every segment of ``graph``'s private memory pool with NaN; returns the bytes filled."""
    pool = tuple(graph.pool())
    torch.cuda.synchronize()
    n = 0
    for seg in torch.cuda.memory._snapshot()["segments"]:
        if tuple(seg.get("segment_pool_id", (0, 0))) != pool:
            continue
        err = _hip().hipMemsetD32(ctypes.c_void_p(seg["address"]), ctypes.c_int(POISON_WORD),
                                  ctypes.c_size_t(seg["total_size"] // 4))
        if err != 0:
            raise RuntimeError("hipMemsetD32 failed: %d" % err)
        n += seg["total_size"]
    torch.cuda.synchronize()
    return n
