"""Global-batch BatchNorm over data-parallel ranks for the functional (PyTorch-op) DARTS path.

The reference DARTS trial normalises every BN layer over its whole 128-image batch
(``examples/v1beta1/trial-images/darts-cnn-cifar10/operations.py:62,96,117,139``) on one GPU.
When the supernet step is split over W ranks (strong scaling: 128/W images each), per-rank
statistics would change the forward and every gradient. :func:`sync_batch_norm` sums the
per-channel (sum, sum of squares, count) over the ranks in the forward and (sum dy, sum dy*xhat)
in the backward, so a W-rank step computes the single-rank step's numbers: the input gradient
is that of the sum of all ranks' losses, the affine-parameter gradients stay per rank (the
gradient all-reduce averages them), exactly as ``torch.nn.SyncBatchNorm`` + DDP. Works over
gloo (CPU, the tests) and RCCL; the HIP kernels have their own fused version
(``ops/hip_darts.py`` ``SyncBN``).
"""

from __future__ import annotations

import torch


class _SyncBatchNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, running_mean, running_var, weight, bias, momentum, eps, comm):
        C = x.shape[1]
        dims = [d for d in range(x.dim()) if d != 1]
        xd = x.double()
        buf = torch.cat([xd.sum(dims), (xd * xd).sum(dims),
                         torch.tensor([x.numel() // C], dtype=torch.float64, device=x.device)])
        comm.allreduce_sum_(buf)
        n = buf[-1]
        mean = buf[:C] / n
        var = (buf[C:2 * C] / n - mean * mean).clamp_min(0.0)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1.0 - momentum).add_(momentum * mean.to(running_mean.dtype))
                running_var.mul_(1.0 - momentum).add_(momentum * (var * n / (n - 1).clamp_min(1.0)).to(running_var.dtype))
        shape = [1, C] + [1] * (x.dim() - 2)
        invstd = torch.rsqrt(var + eps).to(x.dtype)
        xhat = (x - mean.to(x.dtype).view(shape)) * invstd.view(shape)
        y = xhat
        if weight is not None:
            y = y * weight.view(shape) + bias.view(shape)
        ctx.save_for_backward(xhat, invstd, weight)
        ctx.comm, ctx.n, ctx.dims = comm, n, dims
        return y

    @staticmethod
    def backward(ctx, dy):
        xhat, invstd, weight = ctx.saved_tensors
        C = xhat.shape[1]
        dims = ctx.dims
        shape = [1, C] + [1] * (xhat.dim() - 2)
        sdy = dy.sum(dims)
        sdyx = (dy * xhat).sum(dims)
        buf = torch.cat([sdy, sdyx]).double()
        ctx.comm.allreduce_sum_(buf)
        n = ctx.n
        m1 = (buf[:C] / n).to(dy.dtype).view(shape)
        m2 = (buf[C:] / n).to(dy.dtype).view(shape)
        k = invstd.view(shape) if weight is None else (weight * invstd).view(shape)
        dx = k * (dy - m1 - xhat * m2)
        gw = sdyx if weight is not None and ctx.needs_input_grad[3] else None
        gb = sdy if weight is not None and ctx.needs_input_grad[4] else None
        return dx, None, None, gw, gb, None, None, None


def sync_batch_norm(x, running_mean, running_var, weight, bias, momentum: float, eps: float, comm):
    """Training-mode BatchNorm with statistics over every rank's batch (see module docstring)."""
    return _SyncBatchNorm.apply(x, running_mean, running_var, weight, bias, momentum, eps, comm)
