"""GPU-resident checkpoint hand-off between trial processes (PBT exploit over xGMI).

Reference PBT copies the parent's checkpoint *directory* on a shared volume
(``pkg/suggestion/v1beta1/pbt/service.py:260-268``, ``shutil.copytree``). On an
MI355X node the parent's weights are still in HBM of the warm worker that trained
it, so the child reads them straight from that GPU:

* :func:`publish` (producer, end of a trial) packs the checkpoint's tensors into one
  flat buffer per dtype on the trial's GPU (one allocation, one copy), keeps it in a
  small per-process LRU cache, exports a HIP IPC handle per buffer and writes it
  with the layout to ``<ckpt_dir>/gpu_checkpoint.ipc`` (the PBT service's copytree
  carries the file into the child's directory).
* :func:`fetch` (consumer, start of the child trial, another process and usually
  another GPU) maps the producer's buffers and copies each with one device-to-device
  transfer (peer-to-peer over xGMI, ~1.7 GB GPT-2-small + Adam state in ~11 ms on one
  link), then rebuilds the checkpoint as views of the local flat buffers.

The files written by :func:`torch.save` stay the durable copy (FromVolume resume,
crash of the producer): :func:`fetch` returns ``None`` whenever the producer is
gone or the handle cannot be mapped, and the caller falls back to the files.
The handle file is JSON: plain integers and hex strings for the IPC handles, and names
from a fixed whitelist for the tensor / storage classes and dtypes. The checkpoint
directory is writable by the trial (user code), so nothing in it is ever unpickled.
"""

from __future__ import annotations

import collections
import json
import os
import socket
from typing import Any, Dict, List, Optional, Tuple

import torch

HANDLE_FILE = "gpu_checkpoint.ipc"
_CACHE: "collections.OrderedDict[str, List[torch.Tensor]]" = collections.OrderedDict()


def _cache_size() -> int:
    return int(os.environ.get("KATIB_AMD_P2P_CACHE", "4"))


def _flatten(obj, tensors: List[torch.Tensor]):
    if isinstance(obj, torch.Tensor):
        tensors.append(obj)
        return {"__tensor__": len(tensors) - 1}
    if isinstance(obj, dict):
        if all(isinstance(k, str) for k in obj) and not ({"__tensor__", "__tuple__", "__items__"} & set(obj)):
            return {k: _flatten(v, tensors) for k, v in obj.items()}
        # non-string keys (an optimizer state_dict's parameter ids) survive JSON as pairs
        return {"__items__": [[k, _flatten(v, tensors)] for k, v in obj.items()]}
    if isinstance(obj, (list, tuple)):
        out = [_flatten(v, tensors) for v in obj]
        return out if isinstance(obj, list) else {"__tuple__": out}
    return obj


def _unflatten(obj, tensors: List[torch.Tensor]):
    if isinstance(obj, dict):
        if set(obj) == {"__tensor__"}:
            return tensors[obj["__tensor__"]]
        if set(obj) == {"__tuple__"}:
            return tuple(_unflatten(v, tensors) for v in obj["__tuple__"])
        if set(obj) == {"__items__"}:
            return {(k if not isinstance(k, list) else tuple(k)): _unflatten(v, tensors) for k, v in obj["__items__"]}
        return {k: _unflatten(v, tensors) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_unflatten(v, tensors) for v in obj]
    return obj


_DTYPES = {str(d): d for d in (torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32,
                                torch.int16, torch.int8, torch.uint8, torch.bool)}


def _storage_classes():
    return {c.__name__: c for c in (torch.UntypedStorage, torch.storage.TypedStorage)}


def _encode_handle(args) -> List:
    """The rebuild_cuda_tensor argument tuple of ``reduce_tensor`` as JSON values."""
    (tensor_cls, size, stride, toff, storage_cls, dtype, device, handle, sbytes, soff, req, rc_handle, rc_off,
     ev_handle, ev_sync) = args
    if tensor_cls is not torch.Tensor or storage_cls.__name__ not in _storage_classes():
        raise TypeError("unsupported tensor/storage class for a P2P checkpoint")
    hx = lambda b: b.hex() if isinstance(b, (bytes, bytearray)) else None  # noqa: E731
    return [list(size), list(stride), int(toff), storage_cls.__name__, str(dtype), int(device), hx(handle),
            int(sbytes), int(soff), bool(req), hx(rc_handle), int(rc_off), hx(ev_handle), bool(ev_sync)]


def _decode_handle(v: List):
    """Inverse of :func:`_encode_handle`; only whitelisted classes and dtypes are accepted."""
    (size, stride, toff, sname, dname, device, handle, sbytes, soff, req, rc_handle, rc_off, ev_handle,
     ev_sync) = v
    scls = _storage_classes()[str(sname)]
    dtype = _DTYPES[str(dname)]
    fb = lambda h: bytes.fromhex(h) if isinstance(h, str) else None  # noqa: E731
    return (torch.Tensor, torch.Size([int(x) for x in size]), tuple(int(x) for x in stride), int(toff), scls, dtype,
            int(device), fb(handle), int(sbytes), int(soff), bool(req), fb(rc_handle), int(rc_off), fb(ev_handle),
            bool(ev_sync))


def publish(state: Any, ckpt_dir: str, key: Optional[str] = None) -> bool:
    """Export ``state`` (nested dicts/lists of tensors and plain values) for :func:`fetch`.
    Returns False (and writes nothing) when the tensors are not on a GPU."""
    from torch.multiprocessing.reductions import reduce_tensor

    tensors: List[torch.Tensor] = []
    try:
        skeleton = _flatten(state, tensors)
        json.dumps(skeleton)  # the handle file is data-only JSON: check before touching the cache / files
    except (TypeError, ValueError):
        return False  # e.g. numpy scalars, dtypes, sets: the caller falls back to torch.save files
    if not tensors or not all(t.is_cuda for t in tensors):
        return False
    dev = tensors[0].device
    groups: Dict[torch.dtype, List[int]] = collections.defaultdict(list)
    for i, t in enumerate(tensors):
        groups[t.dtype].append(i)
    layout: List[Tuple[str, int, Tuple[int, ...], int]] = [None] * len(tensors)  # (dtype, offset, shape, numel)
    bufs, handles = [], {}
    with torch.no_grad():
        for dt, idx in groups.items():
            total = sum(tensors[i].numel() for i in idx)
            buf = torch.empty(total, dtype=dt, device=dev)
            off = 0
            for i in idx:
                n = tensors[i].numel()
                buf[off:off + n].copy_(tensors[i].detach().reshape(-1))
                layout[i] = (str(dt), off, tuple(tensors[i].shape), n)
                off += n
            bufs.append(buf)
            handles[str(dt)] = _encode_handle(reduce_tensor(buf)[1])
    torch.cuda.current_stream(dev).synchronize()
    key = key or os.path.abspath(ckpt_dir)
    _CACHE[key] = bufs
    _CACHE.move_to_end(key)
    while len(_CACHE) > _cache_size():
        _CACHE.popitem(last=False)
    os.makedirs(ckpt_dir, exist_ok=True)
    tmp = os.path.join(ckpt_dir, HANDLE_FILE + ".tmp")
    with open(tmp, "w") as f:
        json.dump({"pid": os.getpid(), "host": socket.gethostname(), "device": dev.index, "key": key,
                   "skeleton": skeleton, "layout": layout, "handles": handles}, f)
    os.replace(tmp, os.path.join(ckpt_dir, HANDLE_FILE))
    return True


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except OSError:
        return False


def fetch(ckpt_dir: str, device: Optional[torch.device] = None) -> Optional[Any]:
    """Copy a published checkpoint onto ``device`` (peer-to-peer); None if unavailable."""
    from torch.multiprocessing.reductions import rebuild_cuda_tensor

    path = os.path.join(ckpt_dir, HANDLE_FILE)
    if not torch.cuda.is_available() or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            meta = json.load(f)  # data only: classes/dtypes are resolved through whitelists
    except (OSError, ValueError):
        return None
    if meta.get("host") != socket.gethostname() or not _alive(int(meta["pid"])):
        return None
    device = device or torch.device("cuda", torch.cuda.current_device())
    local: Dict[str, torch.Tensor] = {}
    if meta["pid"] == os.getpid() and meta.get("key") in _CACHE:
        # same process (the child landed on the producer's worker): no IPC mapping needed
        for b in _CACHE[meta["key"]]:
            local[str(b.dtype)] = b.to(device, copy=True)
    if not local:
        try:
            for dt, enc in meta["handles"].items():
                src = rebuild_cuda_tensor(*_decode_handle(enc))
                dst = torch.empty(src.numel(), dtype=src.dtype, device=device)
                dst.copy_(src)  # device-to-device: xGMI peer copy across GPUs
                torch.cuda.synchronize(device)
                local[dt] = dst
                del src
        except Exception:
            return None
    tensors = []
    for dt, off, shape, n in meta["layout"]:
        tensors.append(local[dt][off:off + n].view(shape))
    return _unflatten(meta["skeleton"], tensors)


def drop(ckpt_dir: str):
    """Release this process's cached copy of a published checkpoint."""
    _CACHE.pop(os.path.abspath(ckpt_dir), None)
