"""Adapter between the manager's v1beta1 objects and the native status engine
(``csrc/native/status_engine.cpp``): the reconcile decisions of the reference's Go
controller - trial bucketing and optimal-trial selection (status_util.go:57-183),
the experiment completion check (status_util.go:187-235), parallel admission and
suggestion demand (experiment_controller.go:274-330, 445-493) and the restart rule
(experiment_controller.go:187-212), plus the trial state machine - what a finished process
means for its trial and the resulting condition change (trial_controller_util.go:42-122) -
run in C++; this module only flattens the objects into plain tuples and maps the results back.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from .. import native
from ..api import constants as C

_COND_BITS = {
    C.TRIAL_CREATED: 1 << 0,
    C.TRIAL_RUNNING: 1 << 1,
    C.TRIAL_SUCCEEDED: 1 << 2,
    C.TRIAL_KILLED: 1 << 3,
    C.TRIAL_FAILED: 1 << 4,
    C.TRIAL_METRICS_UNAVAILABLE: 1 << 5,
    C.TRIAL_EARLY_STOPPED: 1 << 6,
}
_STRATEGY = {C.STRATEGY_MIN: 1, C.STRATEGY_MAX: 2, C.STRATEGY_LATEST: 3}
_OBJECTIVE = {C.OBJECTIVE_MINIMIZE: 1, C.OBJECTIVE_MAXIMIZE: 2}
_RESUME = {C.RESUME_NEVER: 0, C.RESUME_LONG_RUNNING: 1, C.RESUME_FROM_VOLUME: 2}

# bucket order of the native TrialBucket enum
BUCKETS = ("killed", "failed", "succeeded", "early", "running", "mu", "pending")
OUTCOMES = ("running", "goal", "max_failed", "max_trials", "suggestion_end")
RESTART = ("none", "restart", "keep_going")
EXIT = ("succeeded", "deadline_exceeded", "killed", "retry", "failed")
TRANSITIONS = ("none", "mark_failed", "mark_succeeded", "complete_observed", "mark_metrics_unavailable",
               "complete_early_stopped")


def _s(v) -> str:
    return "" if v is None else str(v)


def condition_mask(trial) -> int:
    st = trial.status
    mask = 0
    if st is not None and st.conditions:
        for c in st.conditions:
            if c.status == C.CONDITION_TRUE:
                mask |= _COND_BITS.get(c.type, 0)
    return mask


def trial_facts(trial) -> Tuple[str, int, bool, str, str, str, int]:
    """(name, condition mask, has objective metric, min, max, latest, strategy)."""
    obj = trial.spec.objective if trial.spec is not None else None
    name = obj.objective_metric_name if obj is not None else None
    strategy = 0
    for s in (obj.metric_strategies or []) if obj is not None else []:
        if s.name == name:
            strategy = _STRATEGY.get(s.value, 0)
            break
    obs = trial.status.observation if trial.status else None
    if obs is not None:
        for m in obs.metrics or []:
            if m.name == name:
                return (trial.metadata.name, condition_mask(trial), True, _s(m.min), _s(m.max), _s(m.latest),
                        strategy)
    return (trial.metadata.name, condition_mask(trial), False, "", "", "", strategy)


def objective_value(trial) -> str:
    _, _, has, mn, mx, latest, strategy = trial_facts(trial)
    return native.load().objective_value(has, mn, mx, latest, strategy)


def summarize(trials: Sequence, objective_type: Optional[str], goal: Optional[float]):
    """-> ({bucket: [trial indices]}, best index or -1, goal_reached)."""
    buckets, best, goal_reached = native.load().summarize_trials(
        [trial_facts(t) for t in trials], _OBJECTIVE.get(objective_type, 0),
        None if goal is None else float(goal))
    return dict(zip(BUCKETS, buckets)), best, goal_reached


def counts(st) -> Tuple[int, int, int, int, int, int, int]:
    return (st.trials_pending or 0, st.trials_running or 0, st.trials_succeeded or 0, st.trials_failed or 0,
            st.trials_killed or 0, st.trials_early_stopped or 0, st.trial_metrics_unavailable or 0)


def decide_condition(st, goal_reached: bool, suggestion_done: bool, max_failed: Optional[int],
                     max_trials: Optional[int]) -> str:
    return OUTCOMES[native.load().decide_condition(counts(st), goal_reached, suggestion_done, max_failed, max_trials)]


def plan_admission(st, parallel: int, max_trials: Optional[int], n_trials: int,
                   early_stopped_without_observation: int) -> Tuple[int, int, int]:
    """-> (delete_count, add_count, suggestion requests)."""
    return tuple(native.load().plan_admission(counts(st), parallel, max_trials, n_trials,
                                              early_stopped_without_observation))


def plan_restart(succeeded_by_max_trials: bool, resume_policy: Optional[str], max_trials: Optional[int],
                 trials: int, has_running_trials: bool) -> str:
    return RESTART[native.load().plan_restart(succeeded_by_max_trials, _RESUME.get(resume_policy, 0), max_trials,
                                              trials, has_running_trials)]


def classify_exit(early_stopped: bool, exit_code: int, warm_worker: bool, run_early_stopped: bool,
                  deadline_exceeded: bool, trial_killed: bool, attempt: int, backoff_limit: int) -> str:
    """What a finished primary process means for its trial (local Job controller + backoffLimit)."""
    return EXIT[native.load().classify_exit(early_stopped, exit_code, warm_worker, run_early_stopped,
                                            deadline_exceeded, trial_killed, attempt, backoff_limit)]


def trial_transition(job_condition: str, trial, observation_available: bool) -> str:
    """UpdateTrialStatusCondition's decision for a job in ``job_condition`` (Running/Succeeded/Failed)."""
    job = {"Succeeded": 1, "Failed": 2}.get(job_condition, 0)
    return TRANSITIONS[native.load().trial_transition(job, condition_mask(trial), observation_available)]


def bucket_names(trials: Sequence, buckets) -> dict:
    return {k: [trials[i].metadata.name for i in idx] for k, idx in buckets.items()}


__all__: List[str] = ["summarize", "decide_condition", "plan_admission", "plan_restart", "objective_value",
                      "trial_facts", "condition_mask", "classify_exit", "trial_transition", "BUCKETS", "OUTCOMES"]
