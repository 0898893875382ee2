"""TensorFlow event-file metrics collector (reference
``pkg/metricscollector/v1beta1/tfevent-metricscollector/tfevent_loader.py:35-114``).

TensorFlow/TensorBoard are not needed: TFRecord framing and the few Event /
Summary / TensorProto fields involved are decoded directly from the protobuf
wire format. Both TF2 tensor summaries (what the reference's TENSORS
EventAccumulator reads) and TF1 ``simple_value`` scalars are accepted.
Metric-name matching follows the reference: a metric ``dir/tag`` matches tag
``tag*`` in event files whose directory ends with ``dir``; a bare ``tag`` matches
in any directory.
"""

from __future__ import annotations

import datetime as _dt
import os
import struct
from typing import Iterator, List, Optional, Tuple

import numpy as np

from ..api import constants as C


def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _fields(buf: bytes) -> Iterator[Tuple[int, int, object]]:
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        else:
            raise ValueError("unsupported wire type %d" % wt)
        yield fno, wt, v


def read_records(path: str) -> Iterator[bytes]:
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                return
            (length,) = struct.unpack("<Q", hdr[:8])
            data = f.read(length)
            f.read(4)  # data crc (not verified, like a tolerant reader)
            if len(data) < length:
                return
            yield data


_DT_FLOAT, _DT_DOUBLE, _DT_INT32, _DT_INT64 = 1, 2, 3, 9


def _tensor_value(buf: bytes) -> Optional[str]:
    dtype, content, fvals, dvals, ivals, i64vals = 0, None, [], [], [], []
    for fno, wt, v in _fields(buf):
        if fno == 1:
            dtype = v
        elif fno == 4:
            content = v
        elif fno == 5:
            if wt == 2:
                fvals += list(struct.unpack("<%df" % (len(v) // 4), v))
            else:
                fvals.append(struct.unpack("<f", v)[0])
        elif fno == 6:
            if wt == 2:
                dvals += list(struct.unpack("<%dd" % (len(v) // 8), v))
            else:
                dvals.append(struct.unpack("<d", v)[0])
        elif fno == 7:
            ivals.append(v)
        elif fno == 10:
            i64vals.append(v)
    if content:
        fmt = {_DT_FLOAT: "<f4", _DT_DOUBLE: "<f8", _DT_INT32: "<i4", _DT_INT64: "<i8"}.get(dtype)
        if fmt is None:
            return None
        arr = np.frombuffer(content, dtype=fmt)
        return str(arr[0]) if arr.size == 1 else str(arr)
    if fvals:
        return str(np.float32(fvals[0]))
    if dvals:
        return str(np.float64(dvals[0]))
    if ivals:
        return str(ivals[0])
    if i64vals:
        return str(i64vals[0])
    return None


def parse_event(buf: bytes):
    """-> (wall_time, step, [(tag, value_str)])"""
    wall, step, vals = 0.0, 0, []
    for fno, wt, v in _fields(buf):
        if fno == 1 and wt == 1:
            wall = struct.unpack("<d", v)[0]
        elif fno == 2:
            step = v
        elif fno == 5 and wt == 2:  # Summary
            for sf, swt, sv in _fields(v):
                if sf != 1 or swt != 2:
                    continue
                tag, value = "", None
                for vf, vwt, vv in _fields(sv):
                    if vf == 1:
                        tag = vv.decode("utf-8", "replace")
                    elif vf == 2 and vwt == 5:
                        value = str(np.float32(struct.unpack("<f", vv)[0]))
                    elif vf == 8 and vwt == 2:
                        value = _tensor_value(vv)
                if value is not None:
                    vals.append((tag, value))
    return wall, step, vals


def _rfc3339(ts: float) -> str:
    return _dt.datetime.fromtimestamp(ts, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def collect(directory: str, metric_names: List[str]) -> List[Tuple[str, str, str]]:
    logs = []
    for root, _, files in os.walk(directory):
        for fn in sorted(files):
            path = os.path.join(root, fn)
            try:
                for rec in read_records(path):
                    wall, _, vals = parse_event(rec)
                    for tag, value in vals:
                        for m in metric_names:
                            parent = os.path.dirname(m) if len(m.split("/")) >= 2 else os.path.dirname(path)
                            if not tag.startswith(m.split("/")[-1]) or not os.path.dirname(path).endswith(parent):
                                continue
                            logs.append((_rfc3339(wall), m, value))
            except Exception:
                continue
    if metric_names and not any(l[1] == metric_names[0] for l in logs):
        now = _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")
        logs = [(now, metric_names[0], C.UNAVAILABLE_METRIC_VALUE)]
    return logs


# ---------------------------------------------------------------- writer (tests/examples)
def _enc_varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fno, wt):
    return _enc_varint((fno << 3) | wt)


def _ld(fno, payload: bytes) -> bytes:
    return _key(fno, 2) + _enc_varint(len(payload)) + payload


def _masked_crc(data: bytes) -> int:
    # crc32c masked as in TFRecord; readers here do not verify, value kept well-formed anyway
    import zlib

    crc = zlib.crc32(data) & 0xFFFFFFFF
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


class EventWriter:
    """Minimal TFRecord event writer producing TF2-style tensor scalar summaries."""

    def __init__(self, logdir: str, filename: str = "events.out.tfevents.katib-amd"):
        os.makedirs(logdir, exist_ok=True)
        self.f = open(os.path.join(logdir, filename), "ab")

    def scalar(self, tag: str, value: float, step: int, wall_time: Optional[float] = None):
        import time

        tensor = _key(1, 0) + _enc_varint(_DT_FLOAT) + _ld(4, struct.pack("<f", float(value)))
        val = _ld(1, tag.encode()) + _ld(8, tensor)
        summary = _ld(1, val)
        ev = _key(1, 1) + struct.pack("<d", wall_time if wall_time is not None else time.time()) + \
            _key(2, 0) + _enc_varint(step) + _ld(5, summary)
        hdr = struct.pack("<Q", len(ev))
        self.f.write(hdr + struct.pack("<I", _masked_crc(hdr)) + ev + struct.pack("<I", _masked_crc(ev)))
        self.f.flush()

    def add_scalar(self, tag: str, scalar_value: float, global_step: int = 0, walltime: Optional[float] = None):
        """``torch.utils.tensorboard.SummaryWriter.add_scalar`` signature."""
        self.scalar(tag, scalar_value, global_step, walltime)

    def close(self):
        self.f.close()
