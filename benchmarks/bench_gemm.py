#!/usr/bin/env python3
"""GPT-2-small forward projections (M = 8 x 1024 tokens): the hand-written MFMA GEMM
(gemm_bf16.hip, bias / GELU fused) against hipBLASLt through torch.addmm (+ the separate GELU
kernel for fc), interleaved rounds in one process, median of per-round means. Prints a table and
one JSON line per shape."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from katib_amd import _hipload

SHAPES = [("qkv", 2304, 768, False), ("proj", 768, 768, False), ("fc+gelu", 3072, 768, True),
          ("fc2", 768, 3072, False), ("lm_head", 50304, 768, False)]


def timeit(fn, iters=50):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters  # us


def main(M=8192, rounds=5):
    k = _hipload.hipkern()
    from katib_amd.ops.transformer import HipOps

    ops = HipOps()
    dev = torch.device("cuda", 0)
    rows = []
    for name, N, K, gelu in SHAPES:
        g = torch.Generator(device=dev).manual_seed(N + K)
        A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        b = None if name == "lm_head" else (torch.randn(N, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        G = torch.empty_like(C) if gelu else None

        def ours():
            k.gemm_nt(A, W, b, C, G)

        def lib():
            u = torch.addmm(b, A, W.t()) if b is not None else torch.mm(A, W.t())
            if gelu:
                ops.gelu_fwd(u)

        for f in (ours, lib):
            timeit(f, 5)
        t_ours, t_lib = [], []
        for _ in range(rounds):
            t_ours.append(timeit(ours))
            t_lib.append(timeit(lib))
        flop = 2.0 * M * N * K
        r = {"shape": name, "M": M, "N": N, "K": K, "fused_gelu": gelu,
             "katib_hip_us": round(statistics.median(t_ours), 2), "hipblaslt_us": round(statistics.median(t_lib), 2)}
        r["katib_hip_tflops"] = round(flop / r["katib_hip_us"] / 1e6, 1)
        r["hipblaslt_tflops"] = round(flop / r["hipblaslt_us"] / 1e6, 1)
        r["speedup"] = round(r["hipblaslt_us"] / r["katib_hip_us"], 3)
        rows.append(r)
        print(json.dumps(r), flush=True)
    print("%-8s %6s %6s %6s %12s %12s %8s" % ("shape", "M", "N", "K", "katib_hip us", "hipBLASLt us", "speedup"))
    for r in rows:
        print("%-8s %6d %6d %6d %12.1f %12.1f %8.3f" % (r["shape"], r["M"], r["N"], r["K"], r["katib_hip_us"],
                                                       r["hipblaslt_us"], r["speedup"]))


if __name__ == "__main__":
    main()
