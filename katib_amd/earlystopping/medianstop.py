"""Median-stop early stopping (reference ``pkg/earlystopping/v1beta1/medianstop/service.py:38-238``).

Settings ``min_trials_required`` (default 3, > 0) and ``start_step`` (default 4, >= 1).
For every newly *succeeded* trial the first ``start_step`` objective values are
averaged; once ``min_trials_required`` trials are recorded the rule
``{objective, value=<mean of averages>, comparison=LESS (maximise) | GREATER
(minimise), start_step}`` is emitted. Parity quirk kept: despite the name the
statistic is the arithmetic *mean* of the per-trial averages (service.py:175).

Observation logs come from the in-process observation store (or any object with
``get_observation_log(trial, metric)``), ``SetTrialStatus`` calls a callback that
marks the trial EarlyStopped in the scheduler instead of patching a K8s object.
A gRPC ``db_manager_address`` is honoured when no in-process source is given.
"""

from __future__ import annotations

import logging
from typing import Callable, Dict, List, Optional

from ..rpc import api_pb2 as api

logger = logging.getLogger(__name__)


class MedianStopService:
    algorithm_names = ("medianstop",)

    def __init__(self, log_source=None, set_trial_status: Optional[Callable[[str], None]] = None):
        self.is_first_run = True
        self.min_trials_required = 3
        self.start_step = 4
        self.trials_avg_history: Dict[str, float] = {}
        self.log_source = log_source
        self.set_trial_status_cb = set_trial_status
        self.comparison = None
        self.objective_metric = None
        self.db_manager_address = None

    # ---------------------------------------------------------------- validation
    @staticmethod
    def validate_medianstop_setting(settings):
        for s in settings:
            try:
                if s.name == "min_trials_required":
                    if not int(s.value) > 0:
                        return False, "min_trials_required must be greater than zero (>0)"
                elif s.name == "start_step":
                    if not int(s.value) >= 1:
                        return False, "start_step must be greater or equal than one (>=1)"
                else:
                    return False, "unknown setting {} for algorithm medianstop".format(s.name)
            except Exception as e:
                return False, "failed to validate {}({}): {}".format(s.name, s.value, e)
        return True, ""

    def validate_early_stopping_spec(self, spec):
        if spec.algorithm_name == "medianstop":
            return self.validate_medianstop_setting(spec.algorithm_settings)
        return False, "unknown algorithm name {}".format(spec.algorithm_name)

    def ValidateEarlyStoppingSettings(self, request, context=None):
        ok, msg = self.validate_early_stopping_spec(request.early_stopping)
        if not ok:
            from ..algorithms.internal import abort

            abort(context, "INVALID_ARGUMENT", msg)
        return api.ValidateEarlyStoppingSettingsReply()

    # ---------------------------------------------------------------- rules
    def GetEarlyStoppingRules(self, request, context=None):
        if self.is_first_run:
            self.is_first_run = False
            for s in request.experiment.spec.early_stopping.algorithm_settings:
                if s.name == "min_trials_required":
                    self.min_trials_required = int(s.value)
                elif s.name == "start_step":
                    self.start_step = int(s.value)
            self.comparison = api.LESS if request.experiment.spec.objective.type == api.MAXIMIZE else api.GREATER
            self.objective_metric = request.experiment.spec.objective.objective_metric_name
            if request.db_manager_address:
                parts = request.db_manager_address.split(":")
                if len(parts) != 2:
                    raise ValueError("Invalid Katib DB manager service address: {}".format(parts))
                self.db_manager_address = request.db_manager_address
        rules = []
        median = self.get_median_value(request.trials)
        if median is not None:
            rules.append(api.EarlyStoppingRule(name=self.objective_metric, value=str(median),
                                               comparison=self.comparison, start_step=self.start_step))
        return api.GetEarlyStoppingRulesReply(early_stopping_rules=rules)

    def _logs(self, trial_name) -> List[str]:
        if self.log_source is not None:
            return [v for _, _, v in self.log_source.get_observation_log(trial_name, self.objective_metric)]
        import grpc

        from ..rpc.client import DBManagerStub

        with grpc.insecure_channel(self.db_manager_address) as ch:
            rep = DBManagerStub(ch).GetObservationLog(
                api.GetObservationLogRequest(trial_name=trial_name, metric_name=self.objective_metric), timeout=60)
        return [m.metric.value for m in rep.observation_log.metric_logs]

    def get_median_value(self, trials) -> Optional[float]:
        for t in trials:
            if t.name in self.trials_avg_history or t.status.condition != api.TrialStatus.SUCCEEDED:
                continue
            vals = self._logs(t.name)[: self.start_step]
            nums = []
            for v in vals:
                try:
                    nums.append(float(v))
                except ValueError:
                    continue
            if not nums:
                continue
            self.trials_avg_history[t.name] = sum(nums) / len(nums)
        if len(self.trials_avg_history) >= self.min_trials_required:
            return sum(self.trials_avg_history.values()) / len(self.trials_avg_history)
        return None

    def SetTrialStatus(self, request, context=None):
        if self.set_trial_status_cb is not None:
            self.set_trial_status_cb(request.trial_name)
        return api.SetTrialStatusReply()
