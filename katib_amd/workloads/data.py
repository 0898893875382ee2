"""Synthetic datasets resident in device memory.

There is no network access for CIFAR-10 / MNIST downloads, so workloads train on
synthetic tensors of the real shapes (documented as ``data: synthetic`` in every
benchmark line). The MI355X-first data path keeps the *whole* dataset in HBM
(CIFAR-10 train: 50k x 3 x 32 x 32 fp32 = 614 MB, trivial against 288 GB) and
draws batches with an on-device gather of a per-epoch permutation - no host
loader, no H2D copy per step. The labels are a fixed random linear function of
the images so that training makes measurable progress.
"""

from __future__ import annotations

import math
from typing import Iterator, Optional, Tuple

import torch


class DeviceDataset:
    def __init__(self, n: int, shape: Tuple[int, ...], num_classes: int, device, seed: int = 0,
                 dtype=torch.float32, learnable: bool = True):
        g = torch.Generator(device="cpu").manual_seed(seed)
        x = torch.randn((n,) + tuple(shape), generator=g, dtype=torch.float32)
        if learnable:
            proj = torch.randn(int(math.prod(shape)), num_classes, generator=g)
            y = (x.flatten(1) @ proj).argmax(1)
        else:
            y = torch.randint(0, num_classes, (n,), generator=g)
        self.x = x.to(device=device, dtype=dtype)
        self.y = y.to(device)
        self.n = n
        self.device = torch.device(device)
        self.num_classes = num_classes

    def subset(self, start: int, end: int) -> "DeviceSubset":
        return DeviceSubset(self, start, end)


class DeviceSubset:
    def __init__(self, ds: DeviceDataset, start: int, end: int):
        self.ds, self.start, self.end = ds, start, end

    def __len__(self):
        return self.end - self.start

    def batches(self, batch_size: int, seed: int = 0, shard: int = 0, num_shards: int = 1,
                drop_last: bool = False) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        """Random permutation each epoch (SubsetRandomSampler); each rank takes its own
        ``batch_size`` slice of every global batch of ``batch_size * num_shards``."""
        g = torch.Generator(device="cpu").manual_seed(seed)
        perm = (torch.randperm(len(self), generator=g) + self.start).to(self.ds.device)
        gb = batch_size * num_shards
        n = len(self)
        steps = n // gb if drop_last else math.ceil(n / gb)
        for s in range(steps):
            idx = perm[s * gb + shard * batch_size: s * gb + (shard + 1) * batch_size]
            if idx.numel() == 0:
                idx = perm[:batch_size]
            yield self.ds.x.index_select(0, idx), self.ds.y.index_select(0, idx)

    def steps_per_epoch(self, batch_size: int, num_shards: int = 1) -> int:
        return math.ceil(len(self) / (batch_size * num_shards))


def cifar10(device, n: int = 50000, seed: int = 0) -> DeviceDataset:
    return DeviceDataset(n, (3, 32, 32), 10, device, seed)


def mnist(device, n: int = 60000, seed: int = 0) -> DeviceDataset:
    return DeviceDataset(n, (1, 28, 28), 10, device, seed)
