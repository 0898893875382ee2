"""PrometheusMetric collector: scrape a trial's ``/metrics`` endpoint.

The reference accepts ``collector.kind: PrometheusMetric`` (defaults: port 8080, path
``/metrics``; ``experiment_defaults.go:135-147``, validation ``validator.go:460-467``) but
ships no collector for it. Here the scheduler scrapes the endpoint while the trial runs:
samples in the Prometheus text exposition format whose metric name is one of the
experiment's metrics become observation-log entries (a new entry when a value or its
sample timestamp changes), so the objective / best trial / early-stopping machinery works
as for the other collectors.

Concurrent trials on one node cannot all listen on the spec's port: each trial gets its
own port in ``KATIB_PROMETHEUS_PORT`` (and the path in ``KATIB_PROMETHEUS_PATH``); a
trial that serves on the spec's port works when it is the only one running. The port is
chosen free by the scheduler just before the launch; another process can still take it
in between (the trial then fails to bind and fails, and is retried only under its Job
``backoffLimit``) - a window of microseconds on a node whose only listeners are trials.

Scrapes run outside the scheduler's lock (``Manager.step``) with a short timeout. A value
published right before the trial exits can fall between two scrapes; trials close that
gap by writing their last exposition to ``KATIB_PROMETHEUS_FINAL`` (:class:`TrialExporter`
does it on ``close()`` / at exit), which the scheduler reads when the trial exits.

Labels: one series per metric name is followed. An unlabelled sample wins; otherwise the
first label set seen for that name is pinned and the others are ignored, so samples of
different label sets never interleave in one observation log.
"""

from __future__ import annotations

import atexit
import math
import os
import re
import threading
import time
import urllib.request
from typing import Dict, Iterable, List, Optional, Tuple

_SAMPLE = re.compile(r"^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{[^}]*\})?\s+(\S+)(?:\s+(-?\d+))?\s*$")


def _rfc3339(t: float) -> str:
    sec = int(math.floor(t))
    ns = int(round((t - sec) * 1e9))
    if ns >= 1_000_000_000:
        sec, ns = sec + 1, ns - 1_000_000_000
    frac = ("%09d" % ns).rstrip("0")
    return time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(sec)) + ("." + frac if frac else "") + "Z"


def parse_exposition(text: str, names: Iterable[str]) -> List[Tuple[str, str, Optional[int]]]:
    """(metric name, value, timestamp ms or None) for every sample line of a wanted metric;
    ``# HELP`` / ``# TYPE`` comments and other metrics are skipped."""
    return [(n, v, ts) for n, _, v, ts in parse_exposition_labeled(text, names)]


def parse_exposition_labeled(text: str, names: Iterable[str]) -> List[Tuple[str, str, str, Optional[int]]]:
    """(metric name, label set text ('' if none), value, timestamp ms or None) per sample."""
    want = set(names)
    out = []
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        m = _SAMPLE.match(line)
        if not m or m.group(1) not in want:
            continue
        value = m.group(3)
        try:
            float(value)  # Prometheus spells NaN / +Inf / -Inf the way float() reads them
        except ValueError:
            continue
        out.append((m.group(1), m.group(2) or "", value, int(m.group(4)) if m.group(4) else None))
    return out


class Scraper:
    """Per-trial scrape state: last value (and sample timestamp) seen per metric."""

    def __init__(self, port: int, path: str, names: List[str], interval: float = 0.25, timeout: float = 0.2,
                 host: str = "127.0.0.1"):
        self.url = "http://%s:%d%s" % (host, int(port), path if path.startswith("/") else "/" + path)
        self.names = list(names)
        self.interval = interval
        self.timeout = timeout
        self.next_at = 0.0
        self.last: Dict[str, Tuple[str, Optional[int]]] = {}
        self.series: Dict[str, str] = {}  # metric name -> the label set followed
        self.scrapes = 0

    def due(self, now: float) -> bool:
        return now >= self.next_at

    def scrape(self, now: Optional[float] = None) -> List[Tuple[str, str, str]]:
        """One scrape; returns new (timestamp, name, value) observations (empty when the
        endpoint is not up yet or gone)."""
        now = time.time() if now is None else now
        self.next_at = now + self.interval
        try:
            with urllib.request.urlopen(self.url, timeout=self.timeout) as r:
                text = r.read().decode("utf-8", "replace")
        except (OSError, ValueError):
            return []
        self.scrapes += 1
        return self.observe(text, now)

    def read_final(self, path: str, now: Optional[float] = None) -> List[Tuple[str, str, str]]:
        """The trial's last exposition (``KATIB_PROMETHEUS_FINAL``), read once it has exited."""
        try:
            with open(path) as f:
                text = f.read()
        except OSError:
            return []
        return self.observe(text, time.time() if now is None else now)

    def observe(self, text: str, now: float) -> List[Tuple[str, str, str]]:
        logs = []
        samples = parse_exposition_labeled(text, self.names)
        for name, labels, _, _ in samples:  # an unlabelled series takes precedence
            if labels == "" and self.series.get(name) != "":
                self.series[name] = ""
        for name, labels, value, ts_ms in samples:
            pinned = self.series.setdefault(name, labels)
            if labels != pinned:
                continue
            key = (value, ts_ms)
            if self.last.get(name) == key:
                continue
            self.last[name] = key
            logs.append((_rfc3339(ts_ms / 1000.0 if ts_ms is not None else now), name, value))
        return logs


class TrialExporter:
    """Trial-side helper: serves ``name value`` gauges on ``KATIB_PROMETHEUS_PORT`` /
    ``KATIB_PROMETHEUS_PATH`` and writes the last exposition to ``KATIB_PROMETHEUS_FINAL``
    on :meth:`close` (and at interpreter exit), so the final objective survives a trial that
    exits right after publishing it."""

    def __init__(self, port: Optional[int] = None, path: Optional[str] = None):
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        self.values: Dict[str, float] = {}
        self.path = path or os.environ.get("KATIB_PROMETHEUS_PATH", "/metrics")
        self.final = os.environ.get("KATIB_PROMETHEUS_FINAL", "")
        self._lock = threading.Lock()
        exporter = self

        class _H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_GET(self):
                if self.path != exporter.path:
                    self.send_response(404)
                    self.end_headers()
                    return
                body = exporter.exposition().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        port = int(port if port is not None else os.environ.get("KATIB_PROMETHEUS_PORT", "8080"))
        self.server = ThreadingHTTPServer(("127.0.0.1", port), _H)
        threading.Thread(target=self.server.serve_forever, daemon=True).start()
        self._closed = False
        atexit.register(self.close)

    def set(self, name: str, value: float):
        with self._lock:
            self.values[name] = float(value)

    def exposition(self) -> str:
        with self._lock:
            return "".join("# TYPE %s gauge\n%s %r\n" % (k, k, v) for k, v in self.values.items())

    def close(self):
        if self._closed:
            return
        self._closed = True
        if self.final:
            tmp = self.final + ".tmp"
            with open(tmp, "w") as f:
                f.write(self.exposition())
            os.replace(tmp, self.final)
        self.server.shutdown()
        self.server.server_close()
