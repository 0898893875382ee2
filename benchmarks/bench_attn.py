"""Causal flash attention for GPT-2 small (head dim 64) on the HIP kernels (csrc/hip/transformer.hip)
vs PyTorch's scaled_dot_product_attention on the same node, bf16, graph-captured timing.

Shape: the PBT member's batch (B=16, T=1024, H=12, d=64). FLOPs counted for the causal half:
forward 4 B H T^2 d / 2, backward 2.5x the forward (dQ, dK, dV + the recomputed scores).
Prints one JSON line per pass."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit_graph(fn, it=10, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (it * reps)


def timeit_eager(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    from katib_amd.ops.transformer import HipOps

    B, T, H, d = (int(v) for v in os.environ.get("ATTN_SHAPE", "16,1024,12,64").split(","))
    dev = torch.device("cuda", 0)
    ops = HipOps()
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(B * T, 3 * H * d, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    dout = torch.randn(B * T, H * d, device=dev, generator=g).to(torch.bfloat16)
    o, lse = ops.attn_fwd(qkv, B, T, H)
    fwd_flops = 4.0 * B * H * T * T * d / 2
    res = {}
    res["hip_fwd_ms"] = timeit_graph(lambda: ops.attn_fwd(qkv, B, T, H))
    res["hip_bwd_ms"] = timeit_graph(lambda: ops.attn_bwd(qkv, o, dout, lse, B, T, H))
    print(json.dumps({"shape": [B, T, H, d], **{k_: round(v_, 4) for k_, v_ in res.items()}}), flush=True)
    q, k, v = qkv.view(B, T, 3, H, d).permute(2, 0, 3, 1, 4)
    q, k, v = (t.contiguous().requires_grad_(True) for t in (q, k, v))
    do = dout.view(B, T, H, d).permute(0, 2, 1, 3).contiguous()
    # PyTorch SDPA (same node): forward captured; forward + backward timed eagerly (its autograd
    # backward aborted inside graph capture on this stack), GPU-bound at this size
    res["sdpa_fwd_ms"] = timeit_graph(lambda: F.scaled_dot_product_attention(q.detach(), k.detach(), v.detach(),
                                                                             is_causal=True))

    def fb():
        yy = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        torch.autograd.grad(yy, (q, k, v), do)

    res["sdpa_fwdbwd_eager_ms"] = timeit_eager(fb)
    res["sdpa_bwd_ms"] = res["sdpa_fwdbwd_eager_ms"] - res["sdpa_fwd_ms"]
    out = {"shape": [B, T, H, d]}
    for k_, val in res.items():
        if k_.endswith("_ms"):
            out[k_] = round(val, 4)
            mult = 1.0 if "fwd_ms" in k_ and "fwdbwd" not in k_ else (2.5 if "bwd_ms" in k_ and "fwdbwd" not in k_ else 3.5)
            out[k_.replace("_ms", "_tflops")] = round(mult * fwd_flops / val / 1e9, 1)
        else:
            out[k_] = val
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
