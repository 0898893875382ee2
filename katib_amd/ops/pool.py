"""Max / average pooling on the hand-written NHWC bf16 HIP kernels (``csrc/hip/pool_nhwc.hip``).

The ENAS child network's ``reduction`` op (reference ``examples/v1beta1/trial-images/
enas-cnn-cifar10/op_library.py:127-150``: Keras ``MaxPooling2D`` / ``AveragePooling2D`` with
``padding='valid'``). Activations are bf16 channels-last like the rest of the child network;
channel counts that are not a multiple of 8 are zero-padded around the kernels. The backward
gathers (every input element written once, no atomics), so the op is deterministic and safe
inside the child's HIP-graph-captured train step.
"""

from __future__ import annotations

import torch

from .conv import kernels


def supported(x: torch.Tensor, pool: int, stride: int) -> bool:
    return (x.is_cuda and x.dim() == 4 and 1 <= pool <= 16 and stride >= 1
            and pool <= x.shape[2] and pool <= x.shape[3])


class _PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pool, stride, is_max):
        k = kernels()
        N, C, H, W = x.shape
        geom = [N, H, W, C, pool, stride]
        xn = x.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        OH, OW = (H - pool) // stride + 1, (W - pool) // stride + 1
        y = torch.empty((N, OH, OW, C), device=x.device, dtype=torch.bfloat16)
        arg = torch.empty((N, OH, OW, C), device=x.device, dtype=torch.uint8) if is_max else None
        k.pool_nhwc_fwd(xn, y, arg, is_max, geom)
        ctx.save_for_backward(*([arg] if is_max else []))
        ctx.geom, ctx.is_max = geom, is_max
        return y.permute(0, 3, 1, 2)  # NCHW view, channels_last memory

    @staticmethod
    def backward(ctx, gy):
        k = kernels()
        N, H, W, C, _, _ = ctx.geom
        arg = ctx.saved_tensors[0] if ctx.is_max else None
        gyn = gy.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        gx = torch.empty((N, H, W, C), device=gy.device, dtype=torch.bfloat16)
        k.pool_nhwc_bwd(gyn, arg, gx, ctx.is_max, ctx.geom)
        return gx.permute(0, 3, 1, 2), None, None, None


def pool2d(x: torch.Tensor, pool: int, stride: int, is_max: bool) -> torch.Tensor:
    """``max_pool2d`` / ``avg_pool2d`` (``padding=0``, ``ceil_mode=False``) with bf16 NHWC kernels."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    C = x.shape[1]
    if C % 8 == 0:
        return _PoolFn.apply(x, int(pool), int(stride), bool(is_max))
    xp = torch.nn.functional.pad(x, (0, 0, 0, 0, 0, (C + 7) // 8 * 8 - C))
    return _PoolFn.apply(xp, int(pool), int(stride), bool(is_max))[:, :C]
