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
trial that serves on the spec's port works when it is the only one running.
"""

from __future__ import annotations

import math
import re
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
        out.append((m.group(1), value, int(m.group(4)) if m.group(4) else None))
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

    def observe(self, text: str, now: float) -> List[Tuple[str, str, str]]:
        logs = []
        for name, value, ts_ms in parse_exposition(text, self.names):
            key = (value, ts_ms)
            if self.last.get(name) == key:
                continue
            self.last[name] = key
            logs.append((_rfc3339(ts_ms / 1000.0 if ts_ms is not None else now), name, value))
        return logs
