"""BatchNorm2d with fused residual add + ReLU on the NHWC bf16 HIP kernels
(``csrc/hip/batchnorm.hip``).

Training forward: batch statistics in fp32 (two streaming passes over the
channels-last activation), running statistics updated in place (unbiased variance,
``momentum`` like ``nn.BatchNorm2d``), ``y = relu(x * scale + shift + residual)``
written once. Backward: the ReLU mask comes from the saved output, so the residual
branch gets its gradient from the same kernel. Eval mode folds the running statistics
into one scale/shift pass.

Used by the ResNet-18 trial (BASELINE config 3); the reference's trial images leave
batch norm to cuDNN/MIOpen (e.g. ``examples/v1beta1/trial-images/enas-cnn-cifar10/
op_library.py:22-155`` via Keras). :class:`BatchNorm2d` is a drop-in ``nn.BatchNorm2d``
whose ``forward(x, residual=None, relu=False)`` takes the fused epilogue; on CPU (or
for channel counts that are not a multiple of 8) it is the stock module plus the
residual add and ReLU.
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


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (channels-last memory or not) -> contiguous [N*H*W, C] bf16."""
    t = t.to(torch.bfloat16)
    return t.permute(0, 2, 3, 1).contiguous().view(-1, t.shape[1])


class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, rmean, rvar, training, momentum, eps, relu, counter=None):
        k = kernels()
        N, C, H, W = x.shape
        xr = _rows(x)
        rr = _rows(res) if res is not None else None
        y = torch.empty((N, H, W, C), device=x.device, dtype=torch.bfloat16)
        w = weight.detach().float().contiguous()
        b = bias.detach().float().contiguous()
        if training:
            mean = torch.empty(C, device=x.device, dtype=torch.float32)
            invstd = torch.empty_like(mean)
            k.bn_fwd_train(xr, rr, y.view(-1, C), w, b, rmean, rvar, mean, invstd, eps, momentum, relu, counter)
            ctx.save_for_backward(xr, y if relu else None, w, mean, invstd)
        else:
            k.bn_fwd_eval(xr, rr, y.view(-1, C), w, b, rmean, rvar, eps, relu)
        ctx.training, ctx.has_res, ctx.shape = training, res is not None, (N, C, H, W)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        if not ctx.training:
            raise RuntimeError("HIP batch norm backward needs training-mode statistics")
        k = kernels()
        xr, y, w, mean, invstd = ctx.saved_tensors
        N, C, H, W = ctx.shape
        gr = _rows(gy)
        dx = torch.empty((N, H, W, C), device=gy.device, dtype=torch.bfloat16)
        dres = torch.empty_like(dx) if ctx.has_res and ctx.needs_input_grad[1] else None
        dgamma = torch.empty(C, device=gy.device, dtype=torch.float32)
        dbeta = torch.empty_like(dgamma)
        k.bn_bwd(gr, None if y is None else y.view(-1, C), xr, w, mean, invstd, dx.view(-1, C),
                 None if dres is None else dres.view(-1, C), dgamma, dbeta)
        return (dx.permute(0, 3, 1, 2), None if dres is None else dres.permute(0, 3, 1, 2), dgamma, dbeta,
                None, None, None, None, None, None, None)


class BatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with a fused ``(+ residual) -> ReLU`` epilogue on the HIP kernels."""

    def forward(self, x, residual=None, relu: bool = False):
        if x.is_cuda and self.num_features % 8 == 0 and self.affine and self.track_running_stats:
            training = self.training
            mom = self.momentum if self.momentum is not None else 0.1
            # num_batches_tracked is bumped by the finalize kernel (one launch fewer per layer)
            return _BNFn.apply(x, residual, self.weight, self.bias, self.running_mean, self.running_var, training,
                               mom, self.eps, relu, self.num_batches_tracked if training else None)
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
