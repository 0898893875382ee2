#!/usr/bin/env python3
"""GPT-2-small projections (M = 8 x 1024 tokens): the hand-written MFMA GEMM (gemm_bf16.hip, bias /
GELU fused) against hipBLASLt through torch.addmm (+ the separate GELU kernel for fc), interleaved
rounds in one process, median of per-round means. Prints a table and one JSON line per shape.

``--backward`` adds the two backward GEMMs of every projection (VERDICT r03 "next" #8: the
per-shape table that decides each hipBLASLt choice):
  dgrad  dX[M, K] = dY[M, N] W[N, K]   (NN)  ours = gemm_nt(dY, W^T shadow); the W^T transpose
         (one per step per weight) is timed separately and added in ``katib_hip_total_us``
  wgrad  dW[N, K] = dY^T[N, M] X[M, K] (TN)  ours = gemm_nt(dY^T, X^T); both activation transposes
         (M x N and M x K, every step) are timed and added the same way
hipBLASLt runs the same products on the strided views (torch.mm(dY, W), torch.mm(dY.t(), X)),
which is what the autograd path of the GPT-2 step calls."""
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


def _row(name, kind, M, N, K, t_ours, t_lib, t_tr=0.0):
    flop = 2.0 * M * N * K
    r = {"shape": name, "kind": kind, "M": M, "N": N, "K": K,
         "katib_hip_us": round(t_ours, 2), "transpose_us": round(t_tr, 2),
         "katib_hip_total_us": round(t_ours + t_tr, 2), "hipblaslt_us": round(t_lib, 2)}
    r["katib_hip_tflops"] = round(flop / t_ours / 1e6, 1)
    r["hipblaslt_tflops"] = round(flop / t_lib / 1e6, 1)
    r["speedup"] = round(t_lib / (t_ours + t_tr), 3)
    r["choice"] = "katib_hip" if r["speedup"] > 1.0 else "hipBLASLt"
    print(json.dumps(r), flush=True)
    return r


def backward(M=8192, rounds=5):
    """dgrad / wgrad of every forward projection (module docstring)."""
    k = _hipload.hipkern()
    dev = torch.device("cuda", 0)
    rows = []
    for name, N, K, _ in SHAPES:
        g = torch.Generator(device=dev).manual_seed(N * 7 + K)
        X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dY = (torch.randn(M, N, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        Wt, dYt, Xt = W.t().contiguous(), dY.t().contiguous(), X.t().contiguous()
        dX = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        # numerics of the NT formulations before timing them
        k.gemm_nt(dY, Wt, None, dX, None)
        ref = dY.float() @ W.float()
        assert (dX.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3, name
        k.gemm_nt(dYt, Xt, None, dW, None)
        ref = dY.float().t() @ X.float()
        assert (dW.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3, name
        fns = {
            "d_ours": lambda: k.gemm_nt(dY, Wt, None, dX, None),
            "d_tr": lambda: Wt.copy_(W.t()),
            "d_lib": lambda: torch.mm(dY, W, out=dX),
            "w_ours": lambda: k.gemm_nt(dYt, Xt, None, dW, None),
            "w_tr": lambda: (dYt.copy_(dY.t()), Xt.copy_(X.t())),
            "w_lib": lambda: torch.mm(dY.t(), X, out=dW),
        }
        for f in fns.values():
            timeit(f, 5)
        t = {key: [] for key in fns}
        for _ in range(rounds):
            for key, f in fns.items():
                t[key].append(timeit(f, 20))
        med = {key: statistics.median(v) for key, v in t.items()}
        rows.append(_row(name, "dgrad", M, K, N, med["d_ours"], med["d_lib"], med["d_tr"]))
        rows.append(_row(name, "wgrad", N, K, M, med["w_ours"], med["w_lib"], med["w_tr"]))
    print("%-8s %-6s %6s %6s %6s %10s %10s %10s %12s %8s %s" % (
        "shape", "kind", "M", "N", "K", "ours us", "transp us", "ours tot", "hipBLASLt us", "speedup", "choice"))
    for r in rows:
        print("%-8s %-6s %6d %6d %6d %10.1f %10.1f %10.1f %12.1f %8.3f %s" % (
            r["shape"], r["kind"], r["M"], r["N"], r["K"], r["katib_hip_us"], r["transpose_us"],
            r["katib_hip_total_us"], r["hipblaslt_us"], r["speedup"], r["choice"]))
    return rows


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
    if "--backward" in sys.argv:
        backward()
