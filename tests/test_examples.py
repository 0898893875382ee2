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
