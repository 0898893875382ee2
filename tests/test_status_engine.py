"""Native experiment status engine (csrc/native/status_engine.cpp): table-driven cases for
the reconcile decisions of the reference's Go controller - updateTrialsSummary /
getObjectiveMetricValue / UpdateExperimentStatusCondition (experiment/util/status_util.go:57-235),
ReconcileTrials + suggestion demand (experiment_controller.go:274-330, 445-493) and the restart
branch (experiment_controller.go:187-212)."""

import pytest

from katib_amd import native
from katib_amd.api import constants as C
from katib_amd.api.models import (V1beta1Metric, V1beta1MetricStrategy, V1beta1ObjectiveSpec, V1beta1Observation,
                                  V1beta1Trial, V1beta1TrialCondition, V1beta1TrialSpec, V1beta1TrialStatus,
                                  V1ObjectMeta)
from katib_amd.controller import status_engine as SE

N = native.load()
CREATED, RUNNING, SUCCEEDED, KILLED, FAILED, MU, ES = (1 << i for i in range(7))
MIN, MAX, LATEST = 1, 2, 3
UNAV = C.UNAVAILABLE_METRIC_VALUE


def row(name, conds, value=None, strategy=MIN):
    if value is None:
        return (name, conds, False, "", "", "", strategy)
    mn, mx, latest = value if isinstance(value, tuple) else (value, value, value)
    return (name, conds, True, mn, mx, latest, strategy)


@pytest.mark.parametrize("mask,bucket", [
    (0, 6), (CREATED, 6), (CREATED | RUNNING, 4), (CREATED | SUCCEEDED, 2), (CREATED | FAILED, 1),
    (CREATED | KILLED, 0), (CREATED | MU, 5), (CREATED | ES, 3),
    # precedence of the if/else chain: Killed > Failed > Succeeded > EarlyStopped > Running > MetricsUnavailable
    (KILLED | FAILED | SUCCEEDED, 0), (FAILED | SUCCEEDED, 1), (SUCCEEDED | ES | RUNNING, 2), (ES | RUNNING, 3),
    (RUNNING | MU, 4),
])
def test_bucket_precedence(mask, bucket):
    buckets, _, _ = N.summarize_trials([row("t", mask)], 1, None)
    assert [len(b) for b in buckets] == [1 if i == bucket else 0 for i in range(7)]


@pytest.mark.parametrize("has,mn,mx,latest,strategy,want", [
    (False, "", "", "", MIN, UNAV),
    (True, "0.1", "0.9", "0.5", MIN, "0.1"),
    (True, "0.1", "0.9", "0.5", MAX, "0.9"),
    (True, "0.1", "0.9", "0.5", LATEST, "0.5"),
    (True, UNAV, UNAV, "abc", MIN, "abc"),  # min unavailable -> latest
    (True, UNAV, UNAV, "abc", MAX, "abc"),
    (True, "0.1", "0.9", "0.5", 0, UNAV),  # no strategy for the objective metric
])
def test_objective_value(has, mn, mx, latest, strategy, want):
    assert N.objective_value(has, mn, mx, latest, strategy) == want


def test_best_trial_and_goal_minimize():
    rows = [row("a", CREATED | SUCCEEDED, "0.5"), row("b", CREATED | SUCCEEDED, "0.2"),
            row("c", CREATED | RUNNING, "0.3"), row("d", CREATED)]
    _, best, goal = N.summarize_trials(rows, 1, 0.25)
    assert best == 1 and goal
    _, best, goal = N.summarize_trials(rows, 1, 0.1)
    assert best == 1 and not goal
    _, best, goal = N.summarize_trials(rows, 1, None)
    assert best == 1 and not goal


def test_best_trial_and_goal_maximize():
    rows = [row("a", SUCCEEDED, "0.5", MAX), row("b", SUCCEEDED, "0.9", MAX), row("c", SUCCEEDED, "0.7", MAX)]
    _, best, goal = N.summarize_trials(rows, 2, 0.9)
    assert best == 1 and goal
    _, best, goal = N.summarize_trials(rows, 2, 0.95)
    assert best == 1 and not goal


def test_goal_is_checked_against_best_so_far():
    # the goal test runs after each numeric trial against the running best (status_util.go:114-126)
    rows = [row("a", SUCCEEDED, "0.05"), row("b", SUCCEEDED, "0.9")]
    _, best, goal = N.summarize_trials(rows, 1, 0.1)
    assert best == 0 and goal


def test_non_numeric_metric_makes_latest_best():
    rows = [row("a", SUCCEEDED, "0.1"), row("b", SUCCEEDED, "good"), row("c", SUCCEEDED, "0.3")]
    _, best, _ = N.summarize_trials(rows, 1, None)
    # "b" becomes best, then "c" is compared against the numeric best 0.1 and loses
    assert best == 1
    # a non-numeric metric set best first: numeric trials are compared against the
    # zero-initialised bestTrialValue, exactly as status_util.go:99-110 does
    rows = [row("a", SUCCEEDED, "x"), row("b", SUCCEEDED, "0.4")]
    _, best, _ = N.summarize_trials(rows, 1, None)
    assert best == 0  # minimize: 0.4 < 0 is false, "a" stays best
    _, best, goal = N.summarize_trials(rows, 2, 0.3)
    assert best == 1 and goal  # maximize: 0.4 > 0, and the goal is checked on that value
    rows = [row("a", SUCCEEDED, "x"), row("b", SUCCEEDED, "-0.4")]
    _, best, _ = N.summarize_trials(rows, 1, None)
    assert best == 1


def test_unavailable_metrics_are_skipped():
    rows = [row("a", MU), row("b", SUCCEEDED, (UNAV, UNAV, UNAV))]
    _, best, goal = N.summarize_trials(rows, 1, 0.0)
    assert best == -1 and not goal


def counts(pending=0, running=0, succeeded=0, failed=0, killed=0, es=0, mu=0):
    return (pending, running, succeeded, failed, killed, es, mu)


@pytest.mark.parametrize("c,goal,sug_done,max_failed,max_trials,want", [
    (counts(running=2), True, False, None, None, 1),
    (counts(failed=1, mu=1), False, False, 2, 10, 2),  # failed + metricsUnavailable >= maxFailed
    (counts(failed=0), False, False, 0, 10, 0),  # failed must be non-zero
    (counts(succeeded=3, mu=1), False, False, None, 4, 3),  # MU counts as completed here
    (counts(succeeded=2, es=1, killed=1), False, False, None, 4, 3),
    (counts(succeeded=2), False, True, None, 4, 4),  # suggestion end with nothing active
    (counts(succeeded=2, pending=1), False, True, None, 4, 0),
    (counts(succeeded=1), False, False, None, None, 0),
    (counts(succeeded=3, failed=3), True, True, 1, 1, 1),  # goal wins over everything
    (counts(failed=3), False, True, 3, 3, 2),  # maxFailed before maxTrials
])
def test_decide_condition(c, goal, sug_done, max_failed, max_trials, want):
    assert N.decide_condition(c, goal, sug_done, max_failed, max_trials) == want


@pytest.mark.parametrize("c,parallel,max_trials,n,es_no_obs,want", [
    (counts(running=3), 3, 10, 3, 0, (0, 0, 0)),
    (counts(running=5), 3, 10, 5, 0, (2, 0, 0)),  # lowered parallelTrialCount deletes the newest
    (counts(), 3, 10, 0, 0, (0, 3, 3)),
    (counts(running=1, succeeded=8), 3, 10, 9, 0, (0, 1, 10)),  # min(max - completed, parallel) - active
    (counts(running=1, succeeded=8, mu=1), 3, 10, 10, 0, (0, 1, 11)),  # MU is not completed here
    (counts(succeeded=2, es=2), 3, None, 4, 1, (0, 3, 6)),  # early-stopped without observation re-requested
    (counts(succeeded=10), 3, 10, 10, 0, (0, 0, 0)),
])
def test_plan_admission(c, parallel, max_trials, n, es_no_obs, want):
    assert N.plan_admission(c, parallel, max_trials, n, es_no_obs) == want


@pytest.mark.parametrize("by_max,policy,max_trials,trials,running,want", [
    (True, 1, 12, 10, False, 1),  # LongRunning, budget raised
    (True, 2, 12, 10, False, 1),  # FromVolume
    (True, 0, 12, 10, False, 0),  # Never is not restartable
    (True, 1, 10, 10, True, 2),  # budget not raised, trials still running
    (False, 1, 12, 10, False, 0),  # succeeded by goal
    (True, 1, None, 4, False, 1),
    (True, 1, None, 0, False, 0),
])
def test_plan_restart(by_max, policy, max_trials, trials, running, want):
    assert N.plan_restart(by_max, policy, max_trials, trials, running) == want


def _trial(name, conds, value=None, strategy=C.STRATEGY_MIN):
    st = V1beta1TrialStatus(conditions=[V1beta1TrialCondition(type=t, status=s) for t, s in conds])
    if value is not None:
        st.observation = V1beta1Observation(metrics=[V1beta1Metric(name="loss", min=value, max=value, latest=value)])
    spec = V1beta1TrialSpec(objective=V1beta1ObjectiveSpec(
        type="minimize", objective_metric_name="loss",
        metric_strategies=[V1beta1MetricStrategy(name="loss", value=strategy)]))
    return V1beta1Trial(metadata=V1ObjectMeta(name=name), spec=spec, status=st)


def test_adapter_flattens_objects():
    ts = [_trial("a", [(C.TRIAL_CREATED, "True"), (C.TRIAL_SUCCEEDED, "True")], "0.4"),
          _trial("b", [(C.TRIAL_CREATED, "True"), (C.TRIAL_RUNNING, "False"), (C.TRIAL_SUCCEEDED, "True")], "0.2"),
          _trial("c", [(C.TRIAL_CREATED, "True"), (C.TRIAL_RUNNING, "True")]),
          _trial("d", [(C.TRIAL_CREATED, "True"), (C.TRIAL_FAILED, "False")])]
    buckets, best, goal = SE.summarize(ts, "minimize", 0.3)
    names = SE.bucket_names(ts, buckets)
    assert names["succeeded"] == ["a", "b"] and names["running"] == ["c"] and names["pending"] == ["d"]
    assert best == 1 and goal
    assert SE.objective_value(ts[0]) == "0.4" and SE.objective_value(ts[2]) == UNAV


@pytest.mark.parametrize("facts,want", [
    # (early_stopped, exit_code, warm_worker, run_early_stopped, deadline, killed, attempt, backoff)
    ((False, 0, False, False, False, False, 1, 0), 0),
    ((True, 143, False, True, False, False, 1, 0), 0),  # collector stop rules fired
    ((False, 3, True, True, False, False, 1, 0), 0),  # warm worker stopped by the early-stop signal
    ((False, 3, False, True, False, False, 1, 0), 4),  # exit code 3 only counts inside warm workers
    ((False, 1, False, False, True, False, 1, 0), 1),  # activeDeadlineSeconds
    ((False, 137, False, False, False, True, 1, 0), 2),  # killed trial keeps its Killed condition
    ((False, 1, False, False, False, False, 1, 2), 3),  # attempt <= backoffLimit: retry
    ((False, 1, False, False, False, False, 3, 2), 4),
])
def test_classify_exit(facts, want):
    assert N.classify_exit(*facts) == want


@pytest.mark.parametrize("job,mask,obs,want", [
    (0, CREATED | RUNNING, False, 0),
    (2, CREATED | RUNNING, False, 1),
    (2, CREATED | FAILED, False, 0),  # already failed
    (2, CREATED | ES, False, 0),  # early-stopped trials never fail
    (1, CREATED | RUNNING, True, 2),
    (1, CREATED | ES, True, 3),  # early-stopped with an observation: completion only
    (1, CREATED | RUNNING, False, 4),  # no objective metric
    (1, CREATED | MU, False, 0),
    (1, CREATED | ES, False, 5),
    (1, CREATED | SUCCEEDED, True, 4),  # the reference's else-if on an already-succeeded trial
])
def test_trial_transition(job, mask, obs, want):
    assert N.trial_transition(job, mask, obs) == want
