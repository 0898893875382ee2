"""Prometheus collectors with the reference metric names
(``pkg/controller.v1beta1/experiment/util/prometheus_metrics.go:27-136``,
``trial/util/prometheus_metrics.go:27-148``) plus MI355X-node gauges
(trials/hour, GPU slot utilisation). Text exposition format 0.0.4."""

from __future__ import annotations

import threading
from collections import defaultdict
from typing import Dict, Tuple

_HELP = {
    "katib_experiment_created_total": "The total number of experiments created",
    "katib_experiment_deleted_total": "The total number of experiments deleted",
    "katib_experiment_succeeded_total": "The total number of experiments succeeded",
    "katib_experiment_failed_total": "The total number of experiments failed",
    "katib_experiments_current": "The number of current katib experiments in cluster",
    "katib_trial_created_total": "The total number of trials created",
    "katib_trial_deleted_total": "The total number of trials deleted",
    "katib_trial_succeeded_total": "The total number of trials succeeded",
    "katib_trial_failed_total": "The total number of trials failed",
    "katib_trial_metrics_unavailable_total": "The total number of trials which metrics are unavailable",
    "katib_trials_current": "The number of current katib trials in cluster",
    "katib_amd_trials_per_hour": "Completed trials per hour since the scheduler started",
    "katib_amd_gpu_slots_busy": "GPU slots currently held by trials",
    "katib_amd_gpu_slots_total": "GPU slots available to trials",
}


class Registry:
    def __init__(self):
        self._lock = threading.Lock()
        self._counters: Dict[str, Dict[Tuple, float]] = defaultdict(lambda: defaultdict(float))
        self._gauges: Dict[str, Dict[Tuple, float]] = defaultdict(dict)

    def inc(self, name: str, **labels):
        with self._lock:
            self._counters[name][tuple(sorted(labels.items()))] += 1

    def set(self, name: str, value: float, **labels):
        with self._lock:
            self._gauges[name][tuple(sorted(labels.items()))] = float(value)

    def get(self, name: str, **labels) -> float:
        key = tuple(sorted(labels.items()))
        with self._lock:
            if name in self._counters:
                return self._counters[name].get(key, 0.0)
            return self._gauges.get(name, {}).get(key, 0.0)

    def expose(self) -> str:
        lines = []
        with self._lock:
            for kind, table in (("counter", self._counters), ("gauge", self._gauges)):
                for name in sorted(table):
                    lines.append("# HELP %s %s" % (name, _HELP.get(name, name)))
                    lines.append("# TYPE %s %s" % (name, kind))
                    for key, v in sorted(table[name].items()):
                        lab = ",".join('%s="%s"' % (k, val) for k, val in key)
                        lines.append("%s{%s} %s" % (name, lab, repr(float(v))) if lab else "%s %s" % (name, v))
        return "\n".join(lines) + "\n"
