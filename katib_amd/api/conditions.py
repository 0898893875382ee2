"""Condition state machines for Experiment, Trial and Suggestion.

Same semantics as the reference helpers:
``pkg/apis/controller/experiments/v1beta1/util.go:26-160``,
``pkg/apis/controller/trials/v1beta1/util.go:68-181``,
``pkg/apis/controller/suggestions/v1beta1/util.go:26-167``:

* ``set_condition`` is a no-op when type, status and reason are unchanged, keeps
  ``lastTransitionTime`` when only the reason changes, and moves the condition to
  the end of the list (so "last condition" == latest transition).
* Succeeded/Failed/Killed/... flip an existing Running condition to False.
"""

from __future__ import annotations

from typing import List, Optional

from . import constants as C
from .models import (V1beta1ExperimentCondition, V1beta1SuggestionCondition, V1beta1TrialCondition,
                     V1beta1ExperimentStatus, V1beta1TrialStatus, V1beta1SuggestionStatus, now)


def _status_obj(obj, status_cls):
    if obj.status is None:
        obj.status = status_cls()
    if obj.status.conditions is None:
        obj.status.conditions = []
    return obj.status


def get_condition(obj, ctype: str):
    st = obj.status
    if st is None or not st.conditions:
        return None
    for c in st.conditions:
        if c.type == ctype:
            return c
    return None


def has_condition(obj, ctype: str) -> bool:
    c = get_condition(obj, ctype)
    return c is not None and c.status == C.CONDITION_TRUE


def remove_condition(obj, ctype: str):
    if obj.status is None or not obj.status.conditions:
        return
    obj.status.conditions = [c for c in obj.status.conditions if c.type != ctype]


def _cond_cls(obj):
    k = type(obj).__name__
    if "Experiment" in k:
        return V1beta1ExperimentCondition, V1beta1ExperimentStatus
    if "Trial" in k:
        return V1beta1TrialCondition, V1beta1TrialStatus
    return V1beta1SuggestionCondition, V1beta1SuggestionStatus


def set_condition(obj, ctype: str, status: str, reason: str, message: str):
    cond_cls, st_cls = _cond_cls(obj)
    st = _status_obj(obj, st_cls)
    t = now()
    new = cond_cls(type=ctype, status=status, reason=reason, message=message,
                   last_update_time=t, last_transition_time=t)
    cur = get_condition(obj, ctype)
    if cur is not None and cur.status == status and cur.reason == reason:
        return
    if cur is not None and cur.status == status:
        new.last_transition_time = cur.last_transition_time
    remove_condition(obj, ctype)
    st.conditions.append(new)


def last_condition_type(obj) -> Optional[str]:
    if obj.status is None or not obj.status.conditions:
        return None
    return obj.status.conditions[-1].type


def _flip_running(obj, running_type: str):
    cur = get_condition(obj, running_type)
    if cur is not None:
        set_condition(obj, running_type, C.CONDITION_FALSE, cur.reason, cur.message)


# ---------------------------------------------------------------- Experiment -------------
class ExperimentConditions:
    @staticmethod
    def is_created(e): return has_condition(e, C.EXPERIMENT_CREATED)

    @staticmethod
    def is_running(e): return has_condition(e, C.EXPERIMENT_RUNNING)

    @staticmethod
    def is_restarting(e): return has_condition(e, C.EXPERIMENT_RESTARTING)

    @staticmethod
    def is_succeeded(e): return has_condition(e, C.EXPERIMENT_SUCCEEDED)

    @staticmethod
    def is_failed(e): return has_condition(e, C.EXPERIMENT_FAILED)

    @staticmethod
    def is_completed(e):
        return has_condition(e, C.EXPERIMENT_SUCCEEDED) or has_condition(e, C.EXPERIMENT_FAILED)

    @staticmethod
    def is_completed_reason(e, reason):
        c = get_condition(e, C.EXPERIMENT_SUCCEEDED)
        return c is not None and c.status == C.CONDITION_TRUE and c.reason == reason

    @staticmethod
    def has_running_trials(e):
        return bool(e.status and e.status.trials_running)

    @staticmethod
    def mark_created(e, reason, msg): set_condition(e, C.EXPERIMENT_CREATED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_running(e, reason, msg): set_condition(e, C.EXPERIMENT_RUNNING, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_restarting(e, reason, msg):
        remove_condition(e, C.EXPERIMENT_SUCCEEDED)
        remove_condition(e, C.EXPERIMENT_FAILED)
        set_condition(e, C.EXPERIMENT_RESTARTING, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_succeeded(e, reason, msg):
        _flip_running(e, C.EXPERIMENT_RUNNING)
        set_condition(e, C.EXPERIMENT_SUCCEEDED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_failed(e, reason, msg):
        _flip_running(e, C.EXPERIMENT_RUNNING)
        set_condition(e, C.EXPERIMENT_FAILED, C.CONDITION_TRUE, reason, msg)


# ---------------------------------------------------------------- Trial ------------------
class TrialConditions:
    @staticmethod
    def is_created(t): return has_condition(t, C.TRIAL_CREATED)

    @staticmethod
    def is_running(t): return has_condition(t, C.TRIAL_RUNNING)

    @staticmethod
    def is_succeeded(t): return has_condition(t, C.TRIAL_SUCCEEDED)

    @staticmethod
    def is_failed(t): return has_condition(t, C.TRIAL_FAILED)

    @staticmethod
    def is_killed(t): return has_condition(t, C.TRIAL_KILLED)

    @staticmethod
    def is_metrics_unavailable(t): return has_condition(t, C.TRIAL_METRICS_UNAVAILABLE)

    @staticmethod
    def is_early_stopped(t): return has_condition(t, C.TRIAL_EARLY_STOPPED)

    @staticmethod
    def is_completed(t):
        return any(has_condition(t, c) for c in (C.TRIAL_SUCCEEDED, C.TRIAL_FAILED, C.TRIAL_KILLED,
                                                   C.TRIAL_EARLY_STOPPED, C.TRIAL_METRICS_UNAVAILABLE))

    @staticmethod
    def is_observation_available(t) -> bool:
        if t.spec is None or t.spec.objective is None:
            return False
        name = t.spec.objective.objective_metric_name
        obs = t.status.observation if t.status else None
        if obs is not None and obs.metrics:
            for m in obs.metrics:
                if m.name == name and m.latest != C.UNAVAILABLE_METRIC_VALUE:
                    return True
        return False

    @staticmethod
    def mark_created(t, reason, msg): set_condition(t, C.TRIAL_CREATED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_running(t, reason, msg): set_condition(t, C.TRIAL_RUNNING, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_succeeded(t, status, reason, msg):
        _flip_running(t, C.TRIAL_RUNNING)
        set_condition(t, C.TRIAL_SUCCEEDED, status, reason, msg)

    @staticmethod
    def mark_failed(t, reason, msg):
        _flip_running(t, C.TRIAL_RUNNING)
        set_condition(t, C.TRIAL_FAILED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_killed(t, reason, msg):
        _flip_running(t, C.TRIAL_RUNNING)
        set_condition(t, C.TRIAL_KILLED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_metrics_unavailable(t, reason, msg):
        _flip_running(t, C.TRIAL_RUNNING)
        set_condition(t, C.TRIAL_METRICS_UNAVAILABLE, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_early_stopped(t, reason, msg):
        # medianstop/service.py:184-238 appends an EarlyStopped condition (status True)
        _flip_running(t, C.TRIAL_RUNNING)
        set_condition(t, C.TRIAL_EARLY_STOPPED, C.CONDITION_TRUE, reason, msg)


# ---------------------------------------------------------------- Suggestion -------------
class SuggestionConditions:
    @staticmethod
    def is_created(s): return has_condition(s, C.SUGGESTION_CREATED)

    @staticmethod
    def is_running(s): return has_condition(s, C.SUGGESTION_RUNNING)

    @staticmethod
    def is_succeeded(s): return has_condition(s, C.SUGGESTION_SUCCEEDED)

    @staticmethod
    def is_failed(s): return has_condition(s, C.SUGGESTION_FAILED)

    @staticmethod
    def is_deployment_ready(s): return has_condition(s, C.SUGGESTION_DEPLOYMENT_READY)

    @staticmethod
    def is_completed(s): return has_condition(s, C.SUGGESTION_SUCCEEDED) or has_condition(s, C.SUGGESTION_FAILED)

    @staticmethod
    def mark_created(s, reason, msg): set_condition(s, C.SUGGESTION_CREATED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_deployment_ready(s, status, reason, msg):
        set_condition(s, C.SUGGESTION_DEPLOYMENT_READY, status, reason, msg)

    @staticmethod
    def mark_running(s, status, reason, msg): set_condition(s, C.SUGGESTION_RUNNING, status, reason, msg)

    @staticmethod
    def mark_succeeded(s, reason, msg):
        _flip_running(s, C.SUGGESTION_RUNNING)
        set_condition(s, C.SUGGESTION_SUCCEEDED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def mark_failed(s, reason, msg):
        _flip_running(s, C.SUGGESTION_RUNNING)
        set_condition(s, C.SUGGESTION_FAILED, C.CONDITION_TRUE, reason, msg)

    @staticmethod
    def is_restarting(s) -> bool:
        # suggestions/v1beta1/util.go:88-95
        c = get_condition(s, C.SUGGESTION_RUNNING)
        return c is not None and c.status == C.CONDITION_FALSE and c.reason == C.SUGGESTION_RESTARTING_REASON
