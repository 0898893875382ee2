"""DARTS edge operators with two backends.

* ``torch`` - composition of PyTorch ops; the numerics oracle (and the CPU path).
* ``hip``   - hand-written CDNA4 kernels from ``katib_amd._hipkern``
  (``csrc/hip/darts_ops.hip`` via :mod:`katib_amd.ops.hip_darts`): a whole
  MixedOp edge (all primitives + their BatchNorms + the weighted sum) and the
  ReLU-conv-BN / FactorizedReduce-BN preprocess layers are single autograd
  Functions whose forward and backward are HIP kernels.

The backend is chosen per process with :func:`set_backend` (``KATIB_AMD_DARTS_OPS``
env var). With backend ``hip`` on a GPU tensor a missing extension raises
(``hip_darts`` import error) instead of silently falling back.
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F

_BACKEND = os.environ.get("KATIB_AMD_DARTS_OPS", "torch")


def set_backend(name: str):
    global _BACKEND
    if name not in ("torch", "hip"):
        raise ValueError(name)
    _BACKEND = name


def backend() -> str:
    return _BACKEND


def hip_enabled(x: torch.Tensor) -> bool:
    return _BACKEND == "hip" and x.is_cuda


def hip_module():
    from . import hip_darts

    return hip_darts


# ------------------------------------------------------------------------- torch path
def relu_conv1x1(x, w):
    return F.conv2d(F.relu(x), w)


def factorized_reduce(x, w1, w2):
    x = F.relu(x)
    return torch.cat([F.conv2d(x, w1, stride=2), F.conv2d(x[:, :, 1:, 1:], w2, stride=2)], dim=1)


def relu_dw_pw(x, dw, pw, stride, padding, dilation):
    y = F.conv2d(F.relu(x), dw, stride=stride, padding=padding, dilation=dilation, groups=x.shape[1])
    return F.conv2d(y, pw)


def avg_pool3x3(x, stride):
    return F.avg_pool2d(x, 3, stride, 1, count_include_pad=False)


def max_pool3x3(x, stride):
    return F.max_pool2d(x, 3, stride, 1)
