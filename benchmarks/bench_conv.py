"""Per-layer timing of the implicit-GEMM HIP convolutions vs MIOpen (torch) on the
ResNet-18 CIFAR shapes, batch 256, bf16 channels-last: forward, input grad, weight grad.
Prints one JSON line per layer with ms and TFLOP/s.

``--graph``: every timed region is captured into a HIP graph (10 calls) and replayed, so
both sides are measured without Python / launch overhead - kernel quality only. The HIP
side times the three kernels on prepared operands (bf16 [K][R][S][C] and [C][R][S][K]
filters, a pre-zeroed fp32 weight-gradient accumulator: in the fused ResNet step the
optimizer kernel writes those), the MIOpen side F.conv2d and its autograd backward."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from katib_amd.ops import conv as hc  # noqa: E402

LAYERS = [  # name, C, H, K, R, stride
    ("stem", 3, 32, 64, 3, 1), ("l1", 64, 32, 64, 3, 1), ("l2a", 64, 32, 128, 3, 2), ("l2s", 64, 32, 128, 1, 2),
    ("l2", 128, 16, 128, 3, 1), ("l3a", 128, 16, 256, 3, 2), ("l3", 256, 8, 256, 3, 1),
    ("l4a", 256, 8, 512, 3, 2), ("l4", 512, 4, 512, 3, 1)]


def timeit(fn, it=20):
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


def main_graph(B):
    dev = torch.device("cuda", 0)
    k = hc.kernels()
    tot = {"hip": 0.0, "torch": 0.0}
    for name, C, H, K, R, s in LAYERS:
        pad = R // 2
        C8 = (C + 7) // 8 * 8
        OH = (H + 2 * pad - R) // s + 1
        flops = 2.0 * B * OH * OH * K * C * R * R
        geom = [B, H, H, C8, K, R, R, OH, OH, s, s, pad, pad, 1, 1]
        xn = torch.randn(B, H, H, C8, device=dev).to(torch.bfloat16)
        if C8 != C:
            xn[..., C:] = 0
        wk = (torch.randn(K, R, R, C8, device=dev) * 0.05).to(torch.bfloat16)
        wt = wk.permute(3, 1, 2, 0).contiguous()
        gy = torch.randn(B, OH, OH, K, device=dev).to(torch.bfloat16)
        y = torch.empty(B, OH, OH, K, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(B, H, H, C8, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(K, R * R * C8, device=dev)
        res = {"hip_fwd": timeit_graph(lambda: k.conv_fwd(xn, wk, y, geom)),
               "hip_wgrad": timeit_graph(lambda: k.conv_wgrad(xn, gy, dw, geom))}
        if name != "stem":
            res["hip_dgrad"] = timeit_graph(lambda: k.conv_dgrad(gy, wt, dx, geom))
        res["hip_fwdbwd"] = res["hip_fwd"] + res["hip_wgrad"] + res.get("hip_dgrad", 0.0)
        if "--hip-only" in sys.argv:
            print(json.dumps({"layer": name, **{k_ + "_ms": round(v, 4) for k_, v in res.items()}}), flush=True)
            tot["hip"] += res["hip_fwdbwd"]
            continue
        x = xn[..., :C].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        wb = wk[..., :C].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        gyt = gy.permute(0, 3, 1, 2)
        xt = x.clone().requires_grad_(name != "stem")
        wt_ = wb.clone().requires_grad_(True)
        res["torch_fwd"] = timeit_graph(lambda: F.conv2d(xt.detach(), wt_.detach(), stride=s, padding=pad))
        ins = (xt, wt_) if name != "stem" else (wt_,)
        res["torch_fwdbwd"] = timeit_graph(
            lambda: torch.autograd.grad(F.conv2d(xt, wt_, stride=s, padding=pad), ins, gyt))
        out = {"layer": name, "shape": [B, C, H, K, R, s]}
        for k_, v in res.items():
            out[k_ + "_ms"] = round(v, 4)
            mult = (3.0 if name != "stem" else 2.0) if "fwdbwd" in k_ else 1.0
            out[k_ + "_tflops"] = round(mult * flops / v / 1e9, 1)
        out["speedup_fwdbwd"] = round(res["torch_fwdbwd"] / res["hip_fwdbwd"], 2)
        tot["hip"] += res["hip_fwdbwd"]
        tot["torch"] += res["torch_fwdbwd"]
        print(json.dumps(out), flush=True)
    print(json.dumps({"graph_total_fwdbwd_ms": {k_: round(v, 3) for k_, v in tot.items()},
                      "speedup": round(tot["torch"] / tot["hip"], 3) if tot["torch"] else None}), flush=True)


def main():
    B = int(os.environ.get("BATCH", "256"))
    if "--graph" in sys.argv:
        return main_graph(B)
    dev = torch.device("cuda", 0)
    tot = {"hip": 0.0, "torch": 0.0}
    for name, C, H, K, R, s in LAYERS:
        pad = R // 2
        x = torch.randn(B, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(K, C, R, R, device=dev) * 0.05
        OH = (H + 2 * pad - R) // s + 1
        flops = 2.0 * B * OH * OH * K * C * R * R
        gy = torch.randn(B, K, OH, OH, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        res = {}
        # hip
        xh = x.clone().requires_grad_(True)
        wh = w.clone().requires_grad_(True)
        res["hip_fwd"] = timeit(lambda: hc.conv2d(xh.detach(), wh.detach(), stride=s, padding=pad))
        y = hc.conv2d(xh, wh, stride=s, padding=pad)
        res["hip_fwdbwd"] = timeit(lambda: torch.autograd.grad(hc.conv2d(xh, wh, stride=s, padding=pad), (xh, wh), gy))
        # torch / MIOpen
        wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        xt = x.clone().requires_grad_(True)
        res["torch_fwd"] = timeit(lambda: F.conv2d(xt.detach(), wb.detach(), stride=s, padding=pad))
        res["torch_fwdbwd"] = timeit(lambda: torch.autograd.grad(F.conv2d(xt, wb, stride=s, padding=pad), (xt, wb), gy))
        del y
        out = {"layer": name, "shape": [B, C, H, K, R, s]}
        for k_, v in res.items():
            out[k_ + "_ms"] = round(v, 4)
            mult = 3.0 if "bwd" in k_ else 1.0
            out[k_ + "_tflops"] = round(mult * flops / v / 1e9, 1)
        tot["hip"] += res["hip_fwdbwd"]
        tot["torch"] += res["torch_fwdbwd"]
        print(json.dumps(out), flush=True)
    print(json.dumps({"total_fwdbwd_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
