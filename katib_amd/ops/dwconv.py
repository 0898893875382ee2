"""Depthwise convolution on the hand-written NHWC HIP kernels (``csrc/hip/dwconv.hip``).

The ENAS child networks' ``depthwise_convolution`` op and the depthwise half of
``separable_convolution`` (reference ``examples/v1beta1/trial-images/enas-cnn-cifar10/
op_library.py:22-155``: Keras ``DepthwiseConv2D`` / ``SeparableConv2D`` with
``padding='same'``) - kernel 3/5/7, stride 1/2, depth multiplier 1/2. Activations are bf16
channels-last like the rest of the child network, weights are the fp32 master parameters
(``[C*DM, 1, K, K]``, output channel ``o`` reads input channel ``o // DM`` as in Keras and
``groups=C`` in PyTorch), accumulation is fp32. The weight gradient is summed from
per-workgroup partials without atomics (deterministic). Channel counts that are not a
multiple of 8 (the 3-channel image input of a child whose first op is a (separable)
depthwise convolution) are zero-padded to 8 channels around the kernels, so no child op
falls back to MIOpen's grouped convolution (whose solvers, measured on MI355X, corrupt
the HIP-graph-captured train step: ``profiles/enas_child_capture_bisect_r02.log``).
"""

from __future__ import annotations

import torch

from .conv import kernels


def _same(size: int, k: int, s: int):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, out


def supported(x: torch.Tensor, weight: torch.Tensor, groups: int, stride: int) -> bool:
    C = x.shape[1]
    K = weight.shape[-1]
    dm = weight.shape[0] // max(C, 1)
    return (x.is_cuda and x.dim() == 4 and groups == C and weight.shape[0] == C * dm
            and dm in (1, 2) and K in (3, 5, 7) and weight.shape[-2] == K and stride in (1, 2))


class _DwFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride):
        k = kernels()
        N, C, H, W = x.shape
        Co, _, K, _ = w.shape
        dm = Co // C
        pt, OH = _same(H, K, stride)
        pl, OW = _same(W, K, stride)
        geom = [N, H, W, C, dm, K, stride, pt, pl, OH, OW]
        xn = x.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        wt = w.detach().float().reshape(Co, K * K).t().contiguous()  # [K*K][Co] tap-major
        y = torch.empty((N, OH, OW, Co), device=x.device, dtype=torch.bfloat16)
        k.dw_fwd(xn, wt, b.detach().float().contiguous() if b is not None else None, y, geom)
        ctx.save_for_backward(xn, wt)
        ctx.geom, ctx.wshape, ctx.wdtype, ctx.has_b = geom, w.shape, w.dtype, b is not None
        return y.permute(0, 3, 1, 2)  # NCHW view, channels_last memory

    @staticmethod
    def backward(ctx, gy):
        k = kernels()
        xn, wt = ctx.saved_tensors
        N, H, W, C, dm, K, S, pt, pl, OH, OW = ctx.geom
        gyn = gy.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((N, H, W, C), device=gy.device, dtype=torch.bfloat16)
            k.dw_dgrad(gyn, wt, dx, ctx.geom)
            gx = dx.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            rows = k.dw_wgrad_rows(ctx.geom)
            part = torch.empty((rows, C * dm, K * K), device=gy.device, dtype=torch.float32)
            k.dw_wgrad(xn, gyn, part, ctx.geom)
            gw = part.sum(0).view(ctx.wshape).to(ctx.wdtype)
        if ctx.has_b and ctx.needs_input_grad[2]:  # HIP channel sum: no PyTorch reduction under capture
            gb = torch.empty(C * dm, device=gy.device, dtype=torch.float32)
            k.channel_sum(gyn.view(-1, C * dm), gb)
        return gx, gw, gb, None


def depthwise_same(x: torch.Tensor, weight: torch.Tensor, bias, stride: int) -> torch.Tensor:
    """Keras ``padding='same'`` depthwise convolution (bf16 NHWC in / out)."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    C = x.shape[1]
    if C % 8 == 0:
        return _DwFn.apply(x, weight, bias, int(stride))
    # zero channels C..C8-1: output channel o = c*DM + j, so the real outputs are the first C*DM
    c8, dm = (C + 7) // 8 * 8, weight.shape[0] // C
    xp = torch.nn.functional.pad(x, (0, 0, 0, 0, 0, c8 - C))
    wp = torch.nn.functional.pad(weight, (0, 0, 0, 0, 0, 0, 0, (c8 - C) * dm))
    bp = torch.nn.functional.pad(bias, (0, (c8 - C) * dm)) if bias is not None else None
    return _DwFn.apply(xp, wp, bp, int(stride))[:, :C * dm]
