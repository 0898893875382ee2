"""Timeline tracing: control-plane spans for trials and suggestion calls, plus roctx
ranges around GPU phases.

The reference has no tracing at all (observability is K8s events,
logs and Prometheus counters; e.g. ``pkg/controller.v1beta1/trial/trial_controller.go:
188-191,290-291``). Here every trial leaves a timeline - created (queued), launched on
its device slot, running, first metric, completed with its phase - and every
``GetSuggestions`` call a span with its request size, so the per-trial overhead that
bounds trials/hour is visible. ``Tracer.chrome_trace()`` emits the Chrome/Perfetto
``traceEvents`` JSON (one track per GPU slot, one for the controller); the same events
stream to a JSON-lines file when ``KATIB_AMD_TRACE_FILE`` (or ``path``) is set.

:func:`gpu_range` wraps a GPU phase in a roctx range (``torch.cuda.nvtx`` maps to roctx
on ROCm) when ``KATIB_AMD_ROCTX=1``, so ``rocprofv3 --marker-trace`` shows kernels under
their training phase; it is a no-op otherwise.
"""

from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from collections import deque
from typing import Deque, Dict, List, Optional

CONTROLLER_TRACK = "controller"


class Tracer:
    def __init__(self, capacity: int = 200_000, path: Optional[str] = None, enabled: bool = True):
        self.enabled = enabled
        self.events: Deque[Dict] = deque(maxlen=capacity)
        self._open: Dict[str, Dict] = {}
        self._lock = threading.Lock()
        self._t0 = time.time()
        path = path or os.environ.get("KATIB_AMD_TRACE_FILE") or None
        self._file = open(path, "a", buffering=1) if (path and enabled) else None

    # ------------------------------------------------------------------ recording
    def _emit(self, ev: Dict):
        with self._lock:
            self.events.append(ev)
            if self._file is not None:
                self._file.write(json.dumps(ev, default=str) + "\n")

    def instant(self, name: str, track: str = CONTROLLER_TRACK, **args):
        if self.enabled:
            self._emit({"ph": "i", "name": name, "ts": time.time(), "track": track, "args": args})

    def begin(self, key: str, name: str, track: str = CONTROLLER_TRACK, **args):
        """Open an asynchronous span identified by ``key`` (e.g. a trial name)."""
        if not self.enabled:
            return
        ev = {"ph": "B", "name": name, "ts": time.time(), "track": track, "key": key, "args": args}
        with self._lock:
            self._open[key] = ev
        self._emit(ev)

    def end(self, key: str, **args):
        if not self.enabled:
            return
        with self._lock:
            b = self._open.pop(key, None)
        if b is None:
            return
        self._emit({"ph": "E", "name": b["name"], "ts": time.time(), "track": b["track"], "key": key,
                    "dur": time.time() - b["ts"], "args": args})

    @contextlib.contextmanager
    def span(self, name: str, track: str = CONTROLLER_TRACK, **args):
        if not self.enabled:
            yield
            return
        t = time.time()
        try:
            yield
        finally:
            self._emit({"ph": "X", "name": name, "ts": t, "dur": time.time() - t, "track": track, "args": args})

    # ------------------------------------------------------------------ queries
    def trial_timeline(self, trial: str) -> List[Dict]:
        with self._lock:
            return [e for e in self.events if e.get("key") == trial or e.get("args", {}).get("trial") == trial]

    def phase_latencies(self) -> Dict[str, float]:
        """Mean seconds from trial creation to launch, launch to first metric, launch to done."""
        firsts: Dict[str, Dict[str, float]] = {}
        with self._lock:
            for e in self.events:
                tr = e.get("args", {}).get("trial") or (e.get("key") if e["name"] == "trial" else None)
                if not tr:
                    continue
                tag = {"trial.created": "created", "trial.first_metric": "first_metric"}.get(e["name"])
                if e["name"] == "trial" and e["ph"] == "B":
                    tag = "launched"
                elif e["name"] == "trial" and e["ph"] == "E":
                    tag = "done"
                if tag:
                    firsts.setdefault(tr, {}).setdefault(tag, e["ts"])
        out: Dict[str, List[float]] = {"queue_s": [], "first_metric_s": [], "run_s": []}
        for d in firsts.values():
            if "created" in d and "launched" in d:
                out["queue_s"].append(d["launched"] - d["created"])
            if "launched" in d and "first_metric" in d:
                out["first_metric_s"].append(d["first_metric"] - d["launched"])
            if "launched" in d and "done" in d:
                out["run_s"].append(d["done"] - d["launched"])
        return {k: (sum(v) / len(v) if v else float("nan")) for k, v in out.items()}

    def chrome_trace(self) -> Dict:
        """Chrome / Perfetto ``traceEvents`` (microseconds; one thread track per GPU slot)."""
        tids: Dict[str, int] = {CONTROLLER_TRACK: 0}
        out = []
        with self._lock:
            evs = list(self.events)
        for e in evs:
            tid = tids.setdefault(e["track"], len(tids))
            ts = (e["ts"] - self._t0) * 1e6
            if e["ph"] == "X":
                out.append({"name": e["name"], "ph": "X", "ts": ts, "dur": e["dur"] * 1e6, "pid": 1, "tid": tid,
                            "args": e.get("args", {})})
            elif e["ph"] in ("B", "E"):
                out.append({"name": e["name"], "ph": "b" if e["ph"] == "B" else "e", "cat": "trial",
                            "id": e["key"], "ts": ts, "pid": 1, "tid": tid, "args": e.get("args", {})})
            else:
                out.append({"name": e["name"], "ph": "i", "s": "t", "ts": ts, "pid": 1, "tid": tid,
                            "args": e.get("args", {})})
        meta = [{"name": "thread_name", "ph": "M", "pid": 1, "tid": t, "args": {"name": n}} for n, t in tids.items()]
        return {"traceEvents": meta + out, "displayTimeUnit": "ms"}

    def export(self, path: str):
        with open(path, "w") as f:
            json.dump(self.chrome_trace(), f)

    def close(self):
        if self._file is not None:
            self._file.close()
            self._file = None


_ROCTX = os.environ.get("KATIB_AMD_ROCTX", "0") == "1"


@contextlib.contextmanager
def gpu_range(name: str):
    """roctx range around a GPU phase (``KATIB_AMD_ROCTX=1``), else a no-op."""
    if not _ROCTX:
        yield
        return
    import torch

    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
