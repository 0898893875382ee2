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
                 device: Optional[torch.device] = None, group=None):
        self.rank, self.world_size, self.local_rank = rank, world_size, local_rank
        self.backend = backend
        self.device = device or torch.device("cpu")
        self.group = group  # None: the default process group
        self.xgmi = None  # one-shot xGMI all-reduce (parallel/xgmi.py), see enable_xgmi()
        self._rccl_capture = None  # verdict of probe_rccl_capture() (collective, run once)
        self.calls = 0  # collectives issued (eager calls + captured ones at capture time)
        self.xgmi_status = None  # one-shot xGMI self-test verdict (enable_xgmi)

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
            if self.xgmi is not None:
                # a self-test between ranks that share one GPU exercises IPC mappings, not an xGMI link
                self.xgmi_status = "passed" if self.distinct_devices() == self.world_size else "passed (same device)"
            elif os.environ.get("KATIB_AMD_XGMI", "1") == "0":
                self.xgmi_status = "disabled"
            elif int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world_size))) != self.world_size \
                    or self.world_size > 8:
                self.xgmi_status = "not applicable (ranks span nodes or > 8)"
            else:
                self.xgmi_status = "failed"  # mapping or self-test failed on some rank: RCCL fallback
        return self.xgmi is not None

    def device_identity(self) -> str:
        """Host + physical identity of this rank's device (UUID / PCI location, not the visible
        index, which every rank of a shared-GPU rehearsal reports as 0)."""
        import socket

        if self.device.type != "cuda":
            return "%s/cpu" % socket.gethostname()
        p = torch.cuda.get_device_properties(self.device)
        ident = str(getattr(p, "uuid", "") or "")
        pci = tuple(getattr(p, k, -1) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        if not ident or ident.strip("0-") == "":
            ident = "pci%s" % (pci,)
        return "%s/%s" % (socket.gethostname(), ident)

    def distinct_devices(self) -> int:
        """Collective: how many distinct physical devices the ranks drive (1 per rank on a real
        multi-GPU node; 1 in total when every rank shares one GPU). Cached after the first call."""
        if getattr(self, "_distinct", None) is None:
            if self.world_size <= 1:
                self._distinct = 1
            else:
                ids = [None] * self.world_size
                dist.all_gather_object(ids, self.device_identity(), group=self.group)
                self._distinct = len(set(ids))
        return self._distinct

    def subgroup(self) -> "Comm":
        """Collective: the same ranks on a communicator of their own (a new process group of this
        backend). Two graph branches that run concurrently must not share a communicator: RCCL
        serialises a communicator's kernels, and two branches interleaving their collectives
        differently on different ranks deadlock."""
        if self.world_size <= 1:
            return Comm(self.rank, 1, self.local_rank, self.backend, self.device)
        g = dist.new_group(backend=self.backend)
        c = Comm(self.rank, self.world_size, self.local_rank, self.backend, self.device, group=g)
        t = torch.zeros(1, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, group=g)  # set the communicator up now, never inside a graph capture
        return c

    def probe_rccl_capture(self) -> bool:
        """Collective (every rank must call it at the same point): can RCCL all-reduces on this
        communicator be captured inside a HIP graph (``torch.cuda.graph``) and replayed?

        Capturing records the collective without running it, so the ranks agree on "captured"
        before any replay (a rank whose capture raised would otherwise leave its peers waiting in
        a replayed all-reduce), then replay twice, check the sums and agree again. Off with
        ``KATIB_AMD_RCCL_CAPTURE=0``; only the ``nccl`` backend (RCCL) qualifies - gloo runs on
        the host."""
        if self._rccl_capture is not None:
            return self._rccl_capture
        ok = (self.world_size > 1 or dist.is_initialized()) and self.backend == "nccl" and \
            self.device.type == "cuda" and os.environ.get("KATIB_AMD_RCCL_CAPTURE", "1") != "0"
        if not ok or self.backend != "nccl":
            self._rccl_capture = False
            return False
        g = None
        x = torch.zeros(64, device=self.device, dtype=torch.float64)
        try:
            dist.all_reduce(x, group=self.group)  # communicator set up outside the capture
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                dist.all_reduce(x, group=self.group)
        except Exception:  # noqa: BLE001 - any failure keeps the collectives on the host
            ok, g = False, None
        ok = self._agree(ok)
        if ok:
            try:
                for _ in range(2):
                    x.fill_(float(self.rank + 1))
                    g.replay()
                torch.cuda.synchronize(self.device)
                ok = bool((x == self.world_size * (self.world_size + 1) / 2.0).all())
            except Exception:  # noqa: BLE001
                ok = False
            ok = self._agree(ok)
        self._rccl_capture = ok
        return ok

    def _agree(self, ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))

    @property
    def rccl_capturable(self) -> bool:
        """The verdict of :meth:`probe_rccl_capture` (False until it ran)."""
        return bool(self._rccl_capture)

    def graph_capturable(self, tensors) -> bool:
        """True when all-reducing ``tensors`` can be captured inside a HIP graph: world size 1, the
        one-shot xGMI kernel (every tensor fits its workspace), or RCCL collectives that passed
        :meth:`probe_rccl_capture`. Collective when the probe has not run yet."""
        if self.world_size == 1:
            return True
        if self.xgmi is not None and all(self.xgmi.fits(t) for t in tensors):
            return True
        return self.probe_rccl_capture()

    def _coll(self, fn, t: torch.Tensor, *a, **kw) -> torch.Tensor:
        """Run a torch.distributed collective; gloo gets a host copy of device tensors."""
        self.calls += 1
        if self.group is not None:
            kw["group"] = self.group
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
                self.calls += 1
                self.xgmi.allreduce_(t, average=True)
            elif self.backend == "nccl":
                self._coll(dist.all_reduce, t, op=dist.ReduceOp.AVG)
            else:
                self._coll(dist.all_reduce, t)
                t.div_(self.world_size)
        return t

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size > 1:
            if self.xgmi is not None and self.xgmi.fits(t):
                self.calls += 1
                self.xgmi.allreduce_(t)
            else:
                self._coll(dist.all_reduce, t)
        return t

    def allreduce_sum_many_(self, ts) -> None:
        """Sum each tensor of ``ts`` over the ranks, in place. On RCCL the all-reduces are one
        grouped call (``ncclGroupStart/End``: one kernel for all of them, capturable like a
        single all-reduce) - the per-fold BN segments of SyncBN are a few hundred bytes each."""
        ts = list(ts)
        if self.world_size <= 1 or not ts:
            return
        if self.backend == "nccl" and len(ts) > 1:
            from torch.distributed.distributed_c10d import _coalescing_manager

            self.calls += 1
            with _coalescing_manager(group=self.group, device=self.device):
                for t in ts:
                    dist.all_reduce(t, group=self.group)
            return
        for t in ts:
            self.allreduce_sum_(t)

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
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def destroy(self):
        if self.world_size > 1 and dist.is_initialized():
            dist.destroy_process_group()
