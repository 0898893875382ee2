#!/usr/bin/env python3
"""GPT-2-small projections (M = 8 x 1024 tokens): the hand-written MFMA GEMM (gemm_bf16.hip, bias /
GELU fused) against hipBLASLt through torch.addmm (+ the separate GELU kernel for fc), interleaved
rounds in one process, median of per-round means. Prints a table and one JSON line per shape.

``--backward`` adds the two backward GEMMs of every projection on the layout-native kernel
(gemm_lt, no transposed copies):
  dgrad  dX[M, K] = dY[M, N] W[N, K]   (NN: W read as [k][n] through ds_read_b64_tr_b16)
  wgrad  dW[N, K] = dY^T[N, M] X[M, K] (TN: both operands MN-contiguous, split-K fp32 slabs)
hipBLASLt runs the same products on the strided views (torch.mm(dY, W), torch.mm(dY.t(), X)),
which is what the autograd path of the GPT-2 step calls. ``--tokens T`` sets M (default 8192;
the PBT member runs 16 x 1024)."""
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
    """dgrad / wgrad of every forward projection on the layout-native kernel (gemm_lt: NN dgrad,
    TN wgrad with split-K fp32 slabs + one row-sum launch, the split chosen per shape by timing)
    against hipBLASLt on the same strided views (torch.mm(dY, W), torch.mm(dY.t(), X)) - no
    transposed copies on either side."""
    k = _hipload.hipkern()
    dev = torch.device("cuda", 0)
    rows = []
    for name, N, K, _ in SHAPES:
        g = torch.Generator(device=dev).manual_seed(N * 7 + K)
        X = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dY = (torch.randn(M, N, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        dX = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        k.gemm_lt(dY, False, W, True, None, dX)
        ref = dY.float() @ W.float()
        assert (dX.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3, name
        splits = [s_ for s_ in (1, 2, 4, 8, 16) if M % (64 * s_) == 0]
        parts = {s_: torch.empty(s_, N, K, device=dev, dtype=torch.float32) for s_ in splits if s_ > 1}

        def wg(s_):
            if s_ == 1:
                return lambda: k.gemm_lt(dY, True, X, True, None, dW)
            p_ = parts[s_]
            return lambda: (k.gemm_lt(dY, True, X, True, None, p_, s_), k.reduce_rows(p_.view(s_, N * K), dW.view(-1)))

        for s_ in splits:
            wg(s_)()
            ref = dY.float().t() @ X.float()
            assert (dW.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-3, (name, s_)
        # hipBLASLt baselines: the plain strided mm, and the split-K batched mm with fp32 output + the
        # same row-sum launch (what HipOps.wgrad ran before gemm_lt) - the better of the two counts
        ls = 1
        while (N // 128) * (K // 128) * ls < 512 and M % (2 * ls) == 0 and M // (2 * ls) >= 1024:
            ls *= 2
        lpart = torch.empty(ls, N, K, device=dev, dtype=torch.float32)

        def w_lib_split():
            torch.bmm(dY.view(ls, M // ls, N).transpose(1, 2), X.view(ls, M // ls, K), out_dtype=torch.float32,
                      out=lpart)
            k.reduce_rows(lpart.view(ls, N * K), dW.view(-1))

        fns = {"d_ours": lambda: k.gemm_lt(dY, False, W, True, None, dX), "d_lib": lambda: torch.mm(dY, W, out=dX),
               "w_lib": lambda: torch.mm(dY.t(), X, out=dW), "w_lib_split": w_lib_split}
        for s_ in splits:
            fns["w_ours%d" % s_] = wg(s_)
        for f in fns.values():
            timeit(f, 5)
        t = {key: [] for key in fns}
        for _ in range(rounds):
            for key, f in fns.items():
                t[key].append(timeit(f, 20))
        med = {key: statistics.median(v) for key, v in t.items()}
        best = min(splits, key=lambda s_: med["w_ours%d" % s_])
        rows.append(_row(name, "dgrad", M, K, N, med["d_ours"], med["d_lib"]))
        r = _row(name, "wgrad", N, K, M, med["w_ours%d" % best], min(med["w_lib"], med["w_lib_split"]))
        r["splitk"] = best
        r["hipblaslt_plain_us"], r["hipblaslt_splitk_us"] = round(med["w_lib"], 2), round(med["w_lib_split"], 2)
        rows.append(r)
    print("%-8s %-6s %6s %6s %6s %10s %8s %8s %12s %8s %s" % (
        "shape", "kind", "M", "N", "K", "ours us", "TF/s", "splitk", "hipBLASLt us", "speedup", "choice"))
    for r in rows:
        print("%-8s %-6s %6d %6d %6d %10.1f %8.1f %8s %12.1f %8.3f %s" % (
            r["shape"], r["kind"], r["M"], r["N"], r["K"], r["katib_hip_us"], r["katib_hip_tflops"],
            r.get("splitk", "-"), r["hipblaslt_us"], r["speedup"], r["choice"]))
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
    tokens = int(sys.argv[sys.argv.index("--tokens") + 1]) if "--tokens" in sys.argv else 8192
    if "--backward-only" not in sys.argv:
        main(tokens)
    if "--backward" in sys.argv or "--backward-only" in sys.argv:
        backward(tokens)
