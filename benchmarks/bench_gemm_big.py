#!/usr/bin/env python3
"""GPT-2 forward projections at the PBT member's 16k tokens: the 256 x 256-tile MFMA GEMM
(gemm_bf16.hip gemm_nt_big_kernel, 128 x 128 per wave; variant 0 plain K loop, 1 software-pipelined)
against the 128 x 128-tile kernel and hipBLASLt (torch.addmm), bf16, interleaved rounds, median of
per-round means. Checks each output against the fp32 product first. One JSON line per shape."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from katib_amd import _hipload  # noqa: E402

SHAPES = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072)]


def timeit(fn, iters=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    k = _hipload.hipkern()
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("TOKENS", "16384"))
    for name, N, K in SHAPES:
        g = torch.Generator(device=dev).manual_seed(N + K)
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g).to(torch.bfloat16)
        ref = x.float() @ w.float().t() + b.float()
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        err = {}
        for v in (-1, 0, 1):
            c.zero_()
            k.gemm_nt(x, w, b, c, None, v)
            torch.cuda.synchronize()
            err[v] = float((c.float() - ref).abs().max() / ref.abs().max())
        fns = {"tile128": lambda: k.gemm_nt(x, w, b, c, None, -1), "big0": lambda: k.gemm_nt(x, w, b, c, None, 0),
               "big1": lambda: k.gemm_nt(x, w, b, c, None, 1), "hipblaslt": lambda: torch.addmm(b, x, w.t())}
        ts = {n: [] for n in fns}
        for _ in range(5):
            for n, f in fns.items():
                ts[n].append(timeit(f))
        flop = 2.0 * M * N * K
        r = {"shape": name, "M": M, "N": N, "K": K, "rel_err": {str(v): round(e, 5) for v, e in err.items()}}
        for n in fns:
            t = statistics.median(ts[n])
            r[n + "_us"] = round(t, 2)
            r[n + "_tflops"] = round(flop / t / 1e6, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
