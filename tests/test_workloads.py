"""Built-in trial workloads run through the scheduler on CPU (tiny sizes); the same
experiments run one trial per MI355X with ``gpus: 1``."""
import os

import pytest

from katib_amd.api.conditions import ExperimentConditions as EC
from katib_amd.api.yaml_io import load_experiment

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")


def _shrink(e, extra_args, max_trials=4, parallel=2):
    spec = e.spec.trial_template.trial_spec["spec"]
    spec["gpus"] = 0
    spec["args"] = list(spec.get("args", [])) + extra_args
    e.spec.max_trial_count = max_trials
    e.spec.parallel_trial_count = parallel
    e.spec.max_failed_trial_count = min(e.spec.max_failed_trial_count or 0, max_trials)
    return e


def test_mnist_mlp_workload_direct():
    from katib_amd.workloads import mnist_mlp

    acc = mnist_mlp.main(["--epochs", "2", "--num-train", "4000", "--num-valid", "1000", "--lr", "0.1",
                          "--hidden", "128"])
    assert 0.2 < acc <= 1.0


def test_tpe_mnist_mlp_example(manager):
    e = _shrink(load_experiment(os.path.join(EX, "hp-tuning", "tpe-mnist-mlp.yaml")),
                ["--epochs=1", "--num-train=3000", "--num-valid=500"])
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=300)
    assert EC.is_succeeded(done), done.status.conditions
    names = {m.name for m in done.status.current_optimal_trial.observation.metrics}
    assert names == {"Validation-accuracy", "loss"}


def test_resnet_hyperband_medianstop_example(manager):
    e = _shrink(load_experiment(os.path.join(EX, "early-stopping", "hyperband-medianstop-resnet18.yaml")),
                ["--num-train=256", "--num-valid=128", "--width=4", "--batch-size=64", "--capture=0"],
                max_trials=8, parallel=8)
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=600)
    assert EC.is_succeeded(done), done.status.conditions
    assert done.status.trials_succeeded + (done.status.trials_early_stopped or 0) == 8


def test_gpt2_pbt_example(manager):
    e = _shrink(load_experiment(os.path.join(EX, "pbt", "pbt-gpt2-small.yaml")),
                ["--model=tiny", "--steps=5", "--num-tokens=20000", "--batch-size=4", "--capture=0"],
                max_trials=12, parallel=5)
    for s in e.spec.algorithm.algorithm_settings:
        if s.name == "n_population":
            s.value = "5"
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=600)
    trials = manager.list_trials(e.metadata.name)
    failed = [t.status.conditions[-1].message for t in trials if t.status.conditions[-1].type == "Failed"]
    assert not failed, failed
    assert EC.is_succeeded(done), done.status.conditions
    parents = [t.metadata.labels.get("pbt.suggestion.katib.kubeflow.org/parent") for t in trials]
    assert any(parents)  # later generations continue from a parent checkpoint
