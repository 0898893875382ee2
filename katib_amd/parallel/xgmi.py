"""One-shot all-reduce over xGMI (inventory K23).

Reference: the reference never calls a collective itself; its trials reduce gradients
with DDP / MirroredStrategy over NCCL (``examples/v1beta1/trial-images/pytorch-mnist/
mnist.py:164-166``). The DARTS supernet trial here is data-parallel on every GPU of a
node, and its per-step gradient vectors are small (37 KB for the B5 config, 1.8 MB for
``darts-gpu.yaml``), where a ring all-reduce is latency-bound and walks one xGMI link at
a time. :class:`XgmiAllReduce` maps every rank's staging buffer into every other rank
(HIP IPC) and sums with one kernel that reads all W-1 peers over their dedicated links
in parallel (``csrc/hip/xgmi_allreduce.hip``). It is HIP-graph capturable, so the DARTS
step can be captured whole at any world size.

Safety: the kernel bounds every wait by a wall-clock timeout and raises an error word
instead of hanging; the constructor runs a self-test whose verdict all ranks agree on
(``ok``), and callers fall back to RCCL when it fails or a message does not fit.
"""

from __future__ import annotations

import importlib
import os
from typing import Optional

import torch

from .. import _hipload
import torch.distributed as dist


def _kern():
    try:
        return _hipload.hipkern()
    except ImportError as e:  # pragma: no cover - GPU boxes always carry the in-tree build
        raise ImportError("katib_amd._hipkern is not built (run __graft_entry__.build()): %s" % e)


def _env_int(name: str, default: int) -> int:
    return int(os.environ.get(name, str(default)))


class XgmiAllReduce:
    """Sum / mean of a float32 GPU tensor over the ranks of one node, in place."""

    def __init__(self, rank: int, world: int, device: torch.device, group=None,
                 capacity: Optional[int] = None, blocks: Optional[int] = None,
                 timeout_s: Optional[float] = None, self_test: bool = True):
        k = _kern()
        if world > k.XGMI_MAX_RANKS:
            raise ValueError("one-shot all-reduce supports up to %d ranks" % k.XGMI_MAX_RANKS)
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.group = group
        cap = capacity if capacity is not None else _env_int("KATIB_AMD_XGMI_CAP", 4 << 20)  # floats
        nb = blocks if blocks is not None else _env_int("KATIB_AMD_XGMI_BLOCKS", 128)
        tmo = timeout_s if timeout_s is not None else float(os.environ.get("KATIB_AMD_XGMI_TIMEOUT", "20"))
        # every step is collective: a rank that fails still takes part, with None / False
        try:
            self.ws = k.XgmiWorkspace(self.device.index, int(cap), int(nb))
            mine = self.ws.handles()
        except RuntimeError:
            self.ws, mine = None, None
        handles = [None] * world
        dist.all_gather_object(handles, mine, group=group)
        opened = False
        if all(h is not None for h in handles):
            try:
                self.ws.open(rank, world, handles, tmo)
                opened = True
            except RuntimeError:
                pass
        self.capacity = self.ws.capacity if self.ws is not None else 0
        self.ok = self._agree(opened)
        if self.ok and self_test:
            self.ok = self._self_test()

    # ------------------------------------------------------------------ api
    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.device == self.device and t.dtype == torch.float32 and t.is_contiguous()
                and t.numel() <= self.capacity)

    def allreduce_(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        self.ws.allreduce(t, t, (1.0 / self.world) if average else 1.0)
        return t

    def allreduce(self, t: torch.Tensor, out: torch.Tensor, average: bool = False) -> torch.Tensor:
        self.ws.allreduce(t, out, (1.0 / self.world) if average else 1.0)
        return out

    def error(self) -> int:
        """Non-zero once any wait timed out (a peer never arrived)."""
        return self.ws.error()

    def check(self):
        if self.ws.error():
            raise RuntimeError("xGMI all-reduce: a peer wait timed out (results invalid)")

    # ------------------------------------------------------------------ self test
    def _agree(self, ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        backend = dist.get_backend(self.group)
        if backend != "gloo":
            t = t.to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return bool(int(t.item()))

    def _self_test(self) -> bool:
        ok = True
        try:
            tri = self.world * (self.world + 1) / 2.0
            x = torch.ones(64, device=self.device)
            self.allreduce_(x)
            torch.cuda.synchronize(self.device)
            if self.ws.error():
                return self._agree(False)  # a peer never arrived: do not wait again
            for n in (5, 4099, min(self.capacity, 1 << 20) - 3):
                x = torch.full((n,), float(self.rank + 1), device=self.device)
                self.allreduce_(x)
                y = torch.empty(n, device=self.device)
                self.allreduce(torch.arange(n, device=self.device, dtype=torch.float32), y, average=True)
                torch.cuda.synchronize(self.device)
                ok = ok and bool((x == tri).all()) and bool(
                    torch.allclose(y, torch.arange(n, device=self.device, dtype=torch.float32), rtol=1e-6))
            ok = ok and self.ws.error() == 0
        except Exception:  # noqa: BLE001 - any failure disables the fast path on every rank
            ok = False
        return self._agree(ok)


def create(comm, group=None, capacity: Optional[int] = None, blocks: Optional[int] = None) -> Optional[XgmiAllReduce]:
    """The fast path for a :class:`~katib_amd.parallel.comm.Comm`, or None (RCCL only).

    Enabled for multi-rank jobs on GPUs of one node (``LOCAL_WORLD_SIZE == WORLD_SIZE``,
    at most 8 ranks) unless ``KATIB_AMD_XGMI=0``. ``capacity`` (floats) / ``blocks`` size a
    workspace of its own (e.g. the SyncBN fold of ``ops/hip_darts.py``)."""
    if os.environ.get("KATIB_AMD_XGMI", "1") == "0" or comm.world_size < 2 or comm.device.type != "cuda":
        return None
    if int(os.environ.get("LOCAL_WORLD_SIZE", str(comm.world_size))) != comm.world_size or comm.world_size > 8:
        return None
    if group is None:
        group = dist.new_group(backend="gloo")
    ar = XgmiAllReduce(comm.rank, comm.world_size, comm.device, group=group, capacity=capacity, blocks=blocks)
    return ar if ar.ok else None
