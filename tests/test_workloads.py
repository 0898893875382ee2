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
    """Two HyperBand rounds: the second round's trials carry the median-stop rule computed
    from the first round's trials (at these CPU sizes accuracies sit near chance, so whether
    the rule fires is noise; tests/test_gpu_workloads.py runs the example at full size on an
    MI355X and asserts early stops)."""
    e = _shrink(load_experiment(os.path.join(EX, "early-stopping", "hyperband-medianstop-resnet18.yaml")),
                ["--num-train=256", "--num-valid=128", "--width=4", "--batch-size=64", "--capture=0"],
                max_trials=16, parallel=8)
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=900)
    assert EC.is_succeeded(done), done.status.conditions
    es = done.status.trials_early_stopped or 0
    assert done.status.trials_succeeded + es == 16
    ruled = [t for t in manager.list_trials(e.metadata.name) if t.spec.early_stopping_rules]
    assert ruled and all(r.name == "Validation-accuracy" and r.comparison == "less"
                         for t in ruled for r in t.spec.early_stopping_rules)


def test_synthetic_tasks_discriminate_hyperparameters():
    """The synthetic teachers do not saturate: across the TPE example's lr range the MLP's
    validation accuracy spreads by >= 0.1 (workloads/common.py teachers)."""
    from katib_amd.workloads import mnist_mlp

    accs = [mnist_mlp.main(["--epochs", "1", "--num-train", "8000", "--num-valid", "2000", "--lr", str(lr),
                            "--hidden", "128"]) for lr in (0.005, 0.05, 0.3)]
    assert max(accs) - min(accs) >= 0.1, accs
    assert max(accs) < 0.97, accs  # label noise keeps it off the ceiling


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
    import glob

    # suggestion_trial_dir is remapped to each member's own directory under the state dir
    members = glob.glob(os.path.join(manager.state_dir, "pbt", e.metadata.name, "*", "model.pt"))
    assert len(members) >= 5


def test_enas_child_example(manager):
    e = load_experiment(os.path.join(EX, "nas", "enas-cifar10.yaml"))
    e.spec.nas_config.graph_config.num_layers = 3
    e = _shrink(e, ["--num-train=256", "--num-valid=128", "--batch-size=64", "--capture=0", "--num_epochs=1"],
                max_trials=4, parallel=2)
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=600)
    assert EC.is_succeeded(done), done.status.conditions
    m = {x.name: x for x in done.status.current_optimal_trial.observation.metrics}
    assert 0.0 <= float(m["Validation-Accuracy"].latest) <= 1.0
    assert len(manager.list_trials(e.metadata.name)) == 4


def test_enas_child_ops_shapes():
    from katib_amd.workloads.enas_child import ChildNet
    import torch

    emb = {"0": {"opt_type": "convolution", "opt_id": 0, "filter_size": "3", "num_filter": "8", "stride": "2"},
           "1": {"opt_type": "separable_convolution", "opt_id": 1, "filter_size": "5", "num_filter": "8",
                 "stride": "1", "depth_multiplier": "2"},
           "2": {"opt_type": "depthwise_convolution", "opt_id": 2, "filter_size": "3", "stride": "1",
                 "depth_multiplier": "1"},
           "3": {"opt_type": "reduction", "opt_id": 3, "reduction_type": "avg_pooling", "pool_size": 2}}
    cfg = {"num_layers": 4, "input_sizes": [32, 32, 3], "output_sizes": [10], "embedding": emb}
    arch = [[0], [1, 1], [2, 0, 1], [3, 1, 0, 1]]
    net = ChildNet(arch, cfg)
    out = net(torch.randn(2, 3, 32, 32))
    assert out.shape == (2, 10)
    # layer 2 concatenates layer 1 (8ch, 16x16) with the zero-padded 32x32 input (3ch)
    assert net.ops[1].cout == 8 and net.ops[1].hw == 32


def test_pytorchjob_two_ranks_example(manager):
    """Master + Worker replicas -> a 2-rank gloo job on CPU (RCCL on GPUs)."""
    e = load_experiment(os.path.join(EX, "distributed", "pytorchjob-mnist.yaml"))
    for role in ("Master", "Worker"):
        c = e.spec.trial_template.trial_spec["spec"]["pytorchReplicaSpecs"][role]["template"]["spec"]["containers"][0]
        c["resources"] = {}
        c["command"] += ["--num-train=512", "--num-test=256", "--backend=gloo"]
    e.spec.max_trial_count, e.spec.parallel_trial_count, e.spec.max_failed_trial_count = 2, 1, 1
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=600)
    assert EC.is_succeeded(done), done.status.conditions
    m = {x.name: x for x in done.status.current_optimal_trial.observation.metrics}
    assert float(m["loss"].latest) > 0


def test_simple_pbt_example(manager):
    e = load_experiment(os.path.join(EX, "pbt", "simple-pbt.yaml"))
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=300)
    assert EC.is_succeeded(done), done.status.conditions
    best = float(done.status.current_optimal_trial.observation.metrics[0].max)
    assert best > 0.3  # members keep training from their parents' checkpoints


def test_darts_example_cpu(manager):
    e = load_experiment(os.path.join(EX, "nas", "darts-cifar10.yaml"))
    c = e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]
    c["resources"] = {}
    c["command"] += ["--num-train=64", "--max-steps=1", "--capture=0", "--ops=torch"]
    for s in e.spec.algorithm.algorithm_settings:
        if s.name == "num_epochs":
            s.value = "1"
    e.spec.algorithm.algorithm_settings.append(type(e.spec.algorithm.algorithm_settings[0])(name="batch_size",
                                                                                            value="8"))
    e.spec.max_trial_count, e.spec.parallel_trial_count, e.spec.max_failed_trial_count = 1, 1, 1
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=600)
    assert EC.is_succeeded(done), [t.status.conditions[-1].message for t in manager.list_trials(e.metadata.name)]
    t = manager.get_trial(done.status.current_optimal_trial.best_trial_name)
    geno = [m for m in t.status.observation.metrics if m.name == "Best-Genotype"]
    assert geno and geno[0].latest.startswith("Genotype(normal=")
