"""2-D convolution on the hand-written implicit-GEMM HIP kernels (``csrc/hip/conv_igemm.hip``).

Activations are bf16 NHWC (``torch.channels_last``), weights are the fp32 master
parameters ([K, C, R, S]); the forward casts them to a bf16 [K][R][S][C] matrix, the
backward returns an fp32 weight gradient (accumulated by the kernel in fp32) and a bf16
input gradient. Channel counts that are not a multiple of 8 (the 3-channel image stem)
are zero-padded to 8 on the fly.

Used by the ResNet-18 trial (reference BASELINE config 3; the reference's own trial
images delegate convolutions to cuDNN, e.g. ``examples/v1beta1/trial-images/
pytorch-mnist/mnist.py:32-48``) and the ENAS child CNNs (reference
``examples/v1beta1/trial-images/enas-cnn-cifar10/op_library.py:22-155``).

:class:`Conv2d` is a drop-in ``nn.Conv2d``: on a GPU it runs the HIP kernels (inputs
cast to bf16 like autocast does), on CPU it is the stock module.
"""

from __future__ import annotations

import importlib

import torch

from .. import _hipload
import torch.nn as nn
import torch.nn.functional as F

_K = None


def kernels():
    global _K
    if _K is None:
        try:
            _K = _hipload.hipkern()
        except ImportError as e:
            raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)
    return _K


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (any memory format) -> contiguous NHWC view/copy."""
    return t.permute(0, 2, 3, 1).contiguous()


def _pad_c(t: torch.Tensor, c8: int) -> torch.Tensor:
    return t if t.shape[-1] == c8 else F.pad(t, (0, c8 - t.shape[-1]))


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding, dilation, out_hw):
        k = kernels()
        N, C, H, W = x.shape
        K, _, R, S = w.shape
        sh, sw = stride
        ph, pw = padding
        dh, dw = dilation
        if out_hw is None:
            OH = (H + 2 * ph - dh * (R - 1) - 1) // sh + 1
            OW = (W + 2 * pw - dw * (S - 1) - 1) // sw + 1
        else:  # asymmetric ('same') padding: (ph, pw) top/left, the rest implied by the output size
            OH, OW = out_hw
        C8 = (C + 7) // 8 * 8
        xn = _pad_c(_nhwc(x.to(torch.bfloat16)), C8)
        wk = _pad_c(w.detach().permute(0, 2, 3, 1).to(torch.bfloat16), C8).contiguous()  # [K][R][S][C8]
        y = torch.empty((N, OH, OW, K), device=x.device, dtype=torch.bfloat16)
        geom = [N, H, W, C8, K, R, S, OH, OW, sh, sw, ph, pw, dh, dw]
        k.conv_fwd(xn, wk, y, geom)
        ctx.save_for_backward(xn, wk)
        ctx.geom, ctx.C, ctx.wdtype = geom, C, w.dtype
        return y.permute(0, 3, 1, 2)  # NCHW view with channels_last memory

    @staticmethod
    def backward(ctx, gy):
        k = kernels()
        xn, wk = ctx.saved_tensors
        N, H, W, C8, K, R, S, OH, OW = ctx.geom[:9]
        gyn = _nhwc(gy.to(torch.bfloat16))
        gx = gw = None
        if K % 8:
            raise ValueError("HIP conv backward needs K % 8 == 0")
        if ctx.needs_input_grad[0]:
            wt = wk.permute(3, 1, 2, 0).contiguous()  # [C8][R][S][K]
            dx = torch.empty((N, H, W, C8), device=gy.device, dtype=torch.bfloat16)
            k.conv_dgrad(gyn, wt, dx, ctx.geom)
            gx = dx[..., :ctx.C].permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            dw32 = torch.zeros((K, R * S * C8), device=gy.device, dtype=torch.float32)
            k.conv_wgrad(xn, gyn, dw32, ctx.geom)
            gw = dw32.view(K, R, S, C8)[..., :ctx.C].permute(0, 3, 1, 2).to(ctx.wdtype)
        return gx, gw, None, None, None, None


def channel_sum_nhwc(g: torch.Tensor) -> torch.Tensor:
    """Sum of an [N, C, H, W] gradient over (N, H, W) -> fp32 [C] on the HIP channel-sum kernel
    (C % 8 == 0), never through PyTorch's cross-workgroup reduction: on this ROCm stack that
    reduction (global staging buffer + semaphores) reads its staging memory before writing it
    when replayed from a HIP graph, which turned the captured ENAS child step NaN
    (profiles/enas_child_capture_rootcause_r03.log)."""
    N, C, H, W = g.shape
    rows = g.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous().view(-1, C)
    out = torch.empty(C, device=g.device, dtype=torch.float32)
    kernels().channel_sum(rows, out)
    return out


class _BiasAddFn(torch.autograd.Function):
    """y + bias[c]; the bias gradient is the HIP channel sum (see :func:`channel_sum_nhwc`)."""

    @staticmethod
    def forward(ctx, y, bias):
        ctx.bdtype = bias.dtype
        return y + bias.to(y.dtype).view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, gy):
        gb = channel_sum_nhwc(gy).to(ctx.bdtype) if ctx.needs_input_grad[1] else None
        return gy, gb


def bias_add(y: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    if y.is_cuda and y.shape[1] % 8 == 0:
        return _BiasAddFn.apply(y, bias)
    return y + bias.to(y.dtype).view(1, -1, 1, 1)


def conv2d(x: torch.Tensor, w: torch.Tensor, bias=None, stride=1, padding=0, dilation=1,
           out_hw=None) -> torch.Tensor:
    """bf16 NHWC implicit-GEMM convolution (groups=1) with an fp32 weight master.
    ``out_hw`` overrides the output size for asymmetric padding (``padding`` = top/left)."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)  # like autocast; keeps the Function's input grad bf16
    y = _ConvFn.apply(x, w, _pair(stride), _pair(padding), _pair(dilation), out_hw)
    if bias is not None:
        y = bias_add(y, bias)
    return y


def supported(x: torch.Tensor, w: torch.Tensor, groups: int = 1) -> bool:
    return x.is_cuda and groups == 1 and w.shape[0] % 8 == 0 and x.dim() == 4


def same_conv2d(x, w, bias, stride: int):
    """TF/Keras ``padding='same'`` (bottom/right-heavy when the total padding is odd)."""
    k = w.shape[2]
    outs, tops = [], []
    for size in x.shape[2:]:
        out = -(-size // stride)
        total = max((out - 1) * stride + k - size, 0)
        outs.append(out)
        tops.append(total // 2)
    return conv2d(x, w, bias, stride, tuple(tops), 1, tuple(outs))


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` whose GPU path is the HIP implicit-GEMM kernels (bf16 compute)."""

    def forward(self, x):
        if (supported(x, self.weight, self.groups) and self.padding_mode == "zeros"
                and isinstance(self.padding, tuple)):
            return conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation)
        return super().forward(x)
