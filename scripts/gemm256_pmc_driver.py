#!/usr/bin/env python3
"""A few launches of gemm256 (NT, 8192^3 and the GPT-2 fc shape) and hipBLASLt on the same operands,
for rocprofv3 --pmc passes (scripts/gpu_r06b.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd import _hipload  # noqa: E402

k = _hipload.hipkern()
dev = torch.device("cuda", 0)
for M, N, K in ((8192, 8192, 8192),):
    g = torch.Generator(device=dev).manual_seed(M)
    A = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        k.gemm256(A, False, B, False, None, C)
        torch.mm(A, B.t(), out=C)
torch.cuda.synchronize()
