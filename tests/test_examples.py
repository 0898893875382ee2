"""Every CPU example under examples/ that mirrors a reference example
(reference examples/v1beta1/{hp-tuning,early-stopping,metrics-collector,resume-experiment,
trial-template}/*.yaml) loads, validates, and runs to a Succeeded experiment through the
in-process scheduler (reference e2e: test/e2e/v1beta1/scripts/gh-actions/run-e2e-experiment.py)."""
import glob
import os
import sys

import pytest

from katib_amd.api.conditions import ExperimentConditions as EC
from katib_amd.api.yaml_io import load_experiment

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CATALOGUE = sorted(p for d in ("hp-tuning", "early-stopping", "metrics-collector", "resume-experiment",
                               "trial-template")
                   for p in glob.glob(os.path.join(ROOT, "examples", d, "*.yaml"))
                   if "mnist" not in p and "resnet" not in p)


def _load(path):
    e = load_experiment(path)
    c = e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]
    if c["command"][0] == "python3":
        c["command"][0] = sys.executable
    return e


def test_catalogue_covers_reference_examples():
    names = {os.path.relpath(p, os.path.join(ROOT, "examples")) for p in CATALOGUE}
    for ref in ("hp-tuning/random.yaml", "hp-tuning/tpe.yaml", "hp-tuning/grid.yaml", "hp-tuning/cma-es.yaml",
                "hp-tuning/sobol.yaml", "hp-tuning/bayesian-optimization.yaml", "hp-tuning/multivariate-tpe.yaml",
                "hp-tuning/hyperband.yaml", "early-stopping/median-stop.yaml",
                "early-stopping/median-stop-with-json-format.yaml", "metrics-collector/file-metrics-collector.yaml",
                "metrics-collector/file-metrics-collector-with-json-format.yaml",
                "metrics-collector/custom-metrics-collector.yaml", "metrics-collector/metrics-collection-strategy.yaml",
                "resume-experiment/long-running-resume.yaml", "resume-experiment/from-volume-resume.yaml",
                "trial-template/trial-metadata-substitution.yaml"):
        assert ref in names


@pytest.mark.parametrize("path", CATALOGUE, ids=lambda p: os.path.relpath(p, os.path.join(ROOT, "examples")))
def test_example_runs(manager, path):
    e = _load(path)
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, namespace=e.metadata.namespace, timeout=240)
    assert EC.is_succeeded(done), done.status.conditions
    assert done.status.trials_succeeded >= 1
    best = done.status.current_optimal_trial
    assert best.best_trial_name and best.observation.metrics
    names = {m.name for m in best.observation.metrics}
    assert e.spec.objective.objective_metric_name in names
    for extra in e.spec.objective.additional_metric_names or []:
        assert extra in names


def _metric(trial, name):
    return next(m for m in trial.status.observation.metrics if m.name == name)


def _run(manager, rel):
    e = _load(os.path.join(ROOT, "examples", rel))
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, namespace=e.metadata.namespace, timeout=240)
    assert EC.is_succeeded(done), done.status.conditions
    return e, done


def _assignments(trial):
    return {a.name: float(a.value) for a in trial.spec.parameter_assignments}


def test_metrics_collection_strategy_applies_min_and_max(manager):
    """metricStrategies: the objective `loss` keeps its minimum over the 4 steps and `accuracy`
    its maximum; the optimal trial is the one with the smallest min(loss)."""
    e, done = _run(manager, "metrics-collector/metrics-collection-strategy.yaml")
    trials = [t for t in manager.list_trials(e.metadata.name, e.metadata.namespace) if t.status.observation]
    assert trials
    for t in trials:
        p = _assignments(t)
        loss, acc = _metric(t, "loss"), _metric(t, "accuracy")
        base = (p["a"] - 1.5) ** 2 + p["b"] ** 2
        assert float(loss.min) == pytest.approx(base + 0.25, rel=1e-5, abs=1e-6)   # last step
        assert float(loss.max) == pytest.approx(base + 1.0, rel=1e-5, abs=1e-6)    # first step
        assert float(acc.max) == pytest.approx(p["a"] / 2, rel=1e-5, abs=1e-6)     # first step
        assert float(acc.latest) == pytest.approx(p["a"] / 2 - 0.3, rel=1e-5, abs=1e-6)
    best = min(trials, key=lambda t: float(_metric(t, "loss").min))
    assert done.status.current_optimal_trial.best_trial_name == best.metadata.name
    obj = next(m for m in done.status.current_optimal_trial.observation.metrics if m.name == "loss")
    assert float(obj.min) == pytest.approx(float(_metric(best, "loss").min))


@pytest.mark.parametrize("rel", ["early-stopping/median-stop.yaml", "early-stopping/median-stop-with-json-format.yaml"])
def test_median_stop_examples_attach_rules(manager, rel):
    """Median stop: once min_trials_required=2 trials succeeded, later trials carry the rule
    {result, value = mean of the first start_step=2 values, comparison less (maximize),
    startStep 2}. Rule *enforcement* (a trial stopped mid-run, EarlyStopped condition, fewer
    observations) is pinned deterministically in tests/test_controller.py::test_medianstop*."""
    e, done = _run(manager, rel)
    trials = sorted(manager.list_trials(e.metadata.name, e.metadata.namespace),
                    key=lambda t: t.metadata.creation_timestamp)
    ruled = [t for t in trials if t.spec.early_stopping_rules]
    assert ruled, "no trial received a median-stop rule"
    assert len(ruled) < len(trials)  # the first min_trials_required trials ran without one
    for t in ruled:
        r = t.spec.early_stopping_rules[0]
        assert r.name == "result" and r.comparison == "less" and r.start_step == 2
    assert (done.status.trials_succeeded or 0) + (done.status.trials_early_stopped or 0) == len(trials)


@pytest.mark.parametrize("rel", ["resume-experiment/long-running-resume.yaml",
                                 "resume-experiment/from-volume-resume.yaml"])
def test_resume_examples_restart_after_budget_raise(manager, rel):
    """Resume policies: a LongRunning / FromVolume experiment that reached maxTrialCount
    restarts when the budget is raised and runs the extra trials."""
    e, done = _run(manager, rel)
    n0 = done.status.trials_succeeded
    assert n0 == e.spec.max_trial_count
    done.spec.max_trial_count = n0 + 2
    manager.update_experiment(done)
    again = manager.run_until_complete(e.metadata.name, namespace=e.metadata.namespace, timeout=240)
    assert EC.is_succeeded(again)
    assert again.status.trials_succeeded == n0 + 2
