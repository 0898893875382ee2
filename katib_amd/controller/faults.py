"""Deterministic fault injection for the scheduler.

The reference has no fault injection; its failure paths (GJSON ``failureCondition`` ->
Failed, succeeded-without-metrics -> MetricsUnavailable, ``maxFailedTrialCount``, Job
``backoffLimit`` retries; ``trial_controller_util.go:42-122``,
``experiment/util/status_util.go:191-212``) are only reached by real crashes. A
:class:`FaultPlan` installed as ``Manager.fault_injector`` reaches each of them on
purpose, reproducibly:

=================  =========================================================================
point / action     effect
=================  =========================================================================
launch / fail      the launch raises -> trial Failed (reason ``LaunchError``)
exit / crash       the primary's exit is rewritten to exit code 1 -> retried while the
                   Job's ``backoffLimit`` allows, then Failed
exit / drop_metrics the trial's observation logs are dropped -> MetricsUnavailable
exit / gpu_fault   the exit becomes SIGSEGV and each of the trial's devices records a GPU
                   fault -> devices quarantined at ``fault_quarantine_threshold``
=================  =========================================================================

Rules select trials by creation order within the experiment (``index``, 0-based), by
name, or all trials (``index=None``), and fire ``times`` times (``None`` = always).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

Key = Tuple[str, str]


@dataclass
class FaultRule:
    point: str  # launch | exit
    action: str  # fail | crash | drop_metrics | gpu_fault
    index: Optional[int] = None
    trial: Optional[str] = None
    times: Optional[int] = 1
    fired: int = 0


@dataclass
class FaultPlan:
    rules: List[FaultRule] = field(default_factory=list)
    log: List[Tuple[str, str, str]] = field(default_factory=list)  # (point, trial, action)
    _order: Dict[str, int] = field(default_factory=dict)

    def add(self, point: str, action: str, index: Optional[int] = None, trial: Optional[str] = None,
            times: Optional[int] = 1) -> "FaultPlan":
        self.rules.append(FaultRule(point, action, index, trial, times))
        return self

    def _index(self, name: str) -> int:
        if name not in self._order:
            self._order[name] = len(self._order)
        return self._order[name]

    def __call__(self, point: str, tkey: Key):
        """Returns the action to inject at ``point`` for trial ``tkey`` (or ``None``); the
        launch point is called first for every trial, which fixes the creation order."""
        name = tkey[1]
        idx = self._index(name)
        for r in self.rules:
            if r.point != point or (r.times is not None and r.fired >= r.times):
                continue
            if r.trial is not None and r.trial != name:
                continue
            if r.index is not None and r.index != idx:
                continue
            r.fired += 1
            self.log.append((point, name, r.action))
            return r.action
        return None
