"""Process-group plumbing for multi-GPU trials: one process per GPU, ``torch.distributed``
with the ``nccl`` backend (= RCCL on ROCm, over xGMI) or ``gloo`` on CPU.

Everything the DARTS / PBT / DP workloads exchange is laid out as *flat* buffers,
so a gradient synchronisation is one collective per buffer - the right shape for
xGMI, where every collective pays a fixed latency and small messages are
latency-bound (0.9-1.8 MB per DARTS step).
"""

from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank: int = 0, world_size: int = 1, local_rank: int = 0, backend: Optional[str] = None,
                 device: Optional[torch.device] = None):
        self.rank, self.world_size, self.local_rank = rank, world_size, local_rank
        self.backend = backend
        self.device = device or torch.device("cpu")
        self.xgmi = None  # one-shot xGMI all-reduce (parallel/xgmi.py), see enable_xgmi()

    @staticmethod
    def from_env(device_type: Optional[str] = None, backend: Optional[str] = None) -> "Comm":
        """torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE / MASTER_ADDR /
        MASTER_PORT), as set by ``torch.distributed.run`` or by the scheduler's rank plans
        (``controller/jobs.py``).

        Rank r drives visible device ``LOCAL_RANK % device_count``: every rank of a trial sees
        the trial's whole device list. When there are more local ranks than devices (a 2-rank
        trial placed on a 1-GPU box with ``slots_per_device: 2``) the ranks share a GPU, which
        RCCL refuses, so the process group is gloo and the gradient all-reduce runs as the
        one-shot IPC kernel (``parallel/xgmi.py``; host copies through gloo if that is off).
        ``backend`` (a trial's ``--backend`` flag) or ``KATIB_AMD_DIST_BACKEND`` overrides the
        choice, except that ``nccl`` on ranks sharing a device becomes gloo."""
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        lrank = int(os.environ.get("LOCAL_RANK", str(rank)))
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
        if device_type is None:
            device_type = "cuda" if torch.cuda.is_available() else "cpu"
        shared = False
        if device_type == "cuda":
            ndev = max(1, torch.cuda.device_count())
            idx = lrank % ndev
            shared = lws > ndev
            torch.cuda.set_device(idx)
            device = torch.device("cuda", idx)
        else:
            device = torch.device("cpu")
        want = backend
        backend = None
        if ws > 1:
            backend = want or os.environ.get("KATIB_AMD_DIST_BACKEND") or (
                "nccl" if device_type == "cuda" and not shared else "gloo")
            if backend == "nccl" and (shared or device_type != "cuda"):
                backend = "gloo"
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                kw = {}
                if backend == "nccl":
                    kw["device_id"] = device
                dist.init_process_group(backend, rank=rank, world_size=ws,
                                        timeout=datetime.timedelta(seconds=600), **kw)
        return Comm(rank, ws, lrank, backend, device)

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    def enable_xgmi(self) -> bool:
        """Collective: set up the one-shot xGMI all-reduce for small float32 messages
        (falls back to RCCL when unavailable, disabled or failing its self-test)."""
        if self.xgmi is None and self.world_size > 1 and self.device.type == "cuda":
            from . import xgmi

            self.xgmi = xgmi.create(self)
        return self.xgmi is not None

    def graph_capturable(self, tensors) -> bool:
        """True when all-reducing ``tensors`` can be captured inside a HIP graph."""
        return self.world_size == 1 or (self.xgmi is not None and all(self.xgmi.fits(t) for t in tensors))

    def _coll(self, fn, t: torch.Tensor, *a, **kw) -> torch.Tensor:
        """Run a torch.distributed collective; gloo gets a host copy of device tensors."""
        if self.backend == "gloo" and t.is_cuda:
            h = t.cpu()
            fn(h, *a, **kw)
            t.copy_(h)
        else:
            fn(t, *a, **kw)
        return t

    def allreduce_mean_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size > 1:
            if self.xgmi is not None and self.xgmi.fits(t):
                self.xgmi.allreduce_(t, average=True)
            elif self.backend == "nccl":
                dist.all_reduce(t, op=dist.ReduceOp.AVG)
            else:
                self._coll(dist.all_reduce, t)
                t.div_(self.world_size)
        return t

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size > 1:
            if self.xgmi is not None and self.xgmi.fits(t):
                self.xgmi.allreduce_(t)
            else:
                self._coll(dist.all_reduce, t)
        return t

    def allreduce_max(self, x: float) -> float:
        if self.world_size <= 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self._coll(dist.all_reduce, t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size > 1:
            self._coll(dist.broadcast, t, src)
        return t

    def barrier(self):
        if self.world_size > 1:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def destroy(self):
        if self.world_size > 1 and dist.is_initialized():
            dist.destroy_process_group()
