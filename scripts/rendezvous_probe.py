#!/usr/bin/env python3
"""Per-rendezvous cost of the one-shot xGMI all-reduce (parallel/xgmi.py) - the SyncBN fold and the
gradient buckets of the DARTS DP step - run under torchrun with N ranks. On a one-GPU box every rank
maps device 0 (cross-process HIP IPC: same kernel, same flag protocol, same-device memory), so the
figure is the launch + flag-handshake floor, not the cost over real xGMI links. Times R back-to-back
all-reduces of each size inside one captured HIP graph (the way the DP step issues them)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from katib_amd.parallel.xgmi import XgmiAllReduce  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("gloo", rank=rank, world_size=world)
R = 50
for blocks in (1, 4, 16):  # workgroups of the fixed grid: each exchanges one flag with every peer
    ar = XgmiAllReduce(rank, world, dev, capacity=1 << 20, blocks=blocks)
    assert ar.ok, "one-shot all-reduce unavailable"
    for n in (64, 2048, 9472, 65536):  # BN-fold segments .. the B5 gradient vector (~37 KB) .. 256 KB
        x = torch.ones(n, device=dev)
        for _ in range(3):
            ar.allreduce_(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(R):
                ar.allreduce_(x)
        g.replay()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6 / (5 * R)
        if rank == 0:
            print("world %d blocks %2d floats %7d: %.2f us per rendezvous (captured, back to back)" % (world, blocks, n, us),
                  flush=True)
    assert ar.error() == 0
dist.destroy_process_group()
