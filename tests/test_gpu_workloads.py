"""BASELINE workloads through the scheduler on one MI355X (warm per-GPU workers)."""
import glob
import os

import pytest

from katib_amd.api.conditions import ExperimentConditions as EC
from katib_amd.api.yaml_io import load_experiment

pytestmark = pytest.mark.gpu
EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")


def _mgr(tmp_path, slots):
    from katib_amd.controller.manager import Manager

    m = Manager(state_dir=str(tmp_path / "state"), num_devices=1, journal=False)
    m.config.amd.slots_per_device = slots
    m.slots = m.N.SlotPool(1, slots)
    return m


def test_pbt_gpt2_p2p_handoff(tmp_path):
    m = _mgr(tmp_path, 5)
    try:
        e = load_experiment(os.path.join(EX, "pbt", "pbt-gpt2-small.yaml"))
        spec = e.spec.trial_template.trial_spec["spec"]
        spec["args"] = [a for a in spec["args"] if not a.startswith("--steps") and not a.startswith("--batch")] + [
            "--model=mini", "--steps=10", "--num-tokens=50000", "--batch-size=4"]
        for s in e.spec.algorithm.algorithm_settings:
            if s.name == "n_population":
                s.value = "5"
        e.spec.max_trial_count, e.spec.parallel_trial_count, e.spec.max_failed_trial_count = 12, 5, 2
        m.create_experiment(e)
        done = m.run_until_complete(e.metadata.name, timeout=900)
        msgs = [t.status.conditions[-1].message[-1500:] for t in m.list_trials(e.metadata.name)
                if t.status.conditions[-1].type == "Failed"]
        assert EC.is_succeeded(done), msgs
        logs = "".join(open(p).read() for p in glob.glob(str(tmp_path / "state" / "trials" / "*" / "*" / "metrics.log")))
        assert "checkpoint_source=p2p" in logs  # children loaded their parent's weights GPU-to-GPU
    finally:
        m.shutdown()


def test_tpe_mnist_mlp_on_gpu(tmp_path):
    m = _mgr(tmp_path, 4)
    try:
        e = load_experiment(os.path.join(EX, "hp-tuning", "tpe-mnist-mlp.yaml"))
        e.spec.max_trial_count, e.spec.parallel_trial_count, e.spec.max_failed_trial_count = 8, 4, 1
        e.spec.objective.goal = None
        m.create_experiment(e)
        done = m.run_until_complete(e.metadata.name, timeout=600)
        assert EC.is_succeeded(done), done.status.conditions
        best = {x.name: x for x in done.status.current_optimal_trial.observation.metrics}
        assert float(best["Validation-accuracy"].max) > 0.5
    finally:
        m.shutdown()
