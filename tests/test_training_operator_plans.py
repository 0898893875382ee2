"""Launch plans of the Kubeflow training-operator trial kinds: the
reference's TFJob, MXJob, MPIJob and XGBoostJob examples
(``examples/v1beta1/kubeflow-training-operator/*.yaml``) become local replica processes with
the env each framework's launcher expects - ``TF_CONFIG`` cluster + task (TFJob), ``DMLC_*``
(MXJob), torchrun-style ranks (XGBoostJob / PyTorchJob), the launcher only (MPIJob: mpirun spawns
the workers) - with every rendezvous port taken from free_port's ledger and re-drawn per launch
attempt. A TFJob-shaped experiment runs end to end on the CPU with a stand-in program."""
import json
import os
import sys

import pytest

from katib_amd.api.conditions import ExperimentConditions as EC
from katib_amd.api.yaml_io import load_experiment
from katib_amd.controller import jobs
from katib_amd.controller.jobs import assign_ports, make_plan

REF = "/root/reference/examples/v1beta1/kubeflow-training-operator"
need_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference examples not present")


def _plan(name, container):
    e = load_experiment(os.path.join(REF, name))
    return make_plan(e.spec.trial_template.trial_spec, container, e.spec.trial_template.primary_pod_labels)


def _ports(plan):
    out = []
    for r in plan.replicas:
        for k in ("MASTER_PORT", "DMLC_PS_ROOT_PORT"):
            if k in r.env:
                out.append(int(r.env[k]))
        if "TF_CONFIG" in r.env:
            for addrs in json.loads(r.env["TF_CONFIG"])["cluster"].values():
                out += [int(a.rsplit(":", 1)[1]) for a in addrs]
    return out


@need_ref
def test_tfjob_plan_tf_config():
    plan = _plan("tfjob-mnist-with-summaries.yaml", "tensorflow")
    assert plan.kind == "TFJob" and plan.ports_managed and len(plan.replicas) == 2
    cfgs = [json.loads(r.env["TF_CONFIG"]) for r in plan.replicas]
    assert all(c["cluster"] == cfgs[0]["cluster"] for c in cfgs)
    workers = cfgs[0]["cluster"]["worker"]
    assert len(workers) == 2 and len(set(workers)) == 2 and all(w.startswith("127.0.0.1:") for w in workers)
    assert [c["task"] for c in cfgs] == [{"type": "worker", "index": 0}, {"type": "worker", "index": 1}]
    assert plan.replicas[0].primary and not plan.replicas[1].primary  # no Chief: worker 0 reports
    for p in _ports(plan):  # every task address came from the ledger (no port + 1 + 64 k arithmetic)
        assert p in jobs._RECENT_PORTS


@need_ref
def test_mxjob_plan_dmlc_env():
    plan = _plan("mxjob-byteps.yaml", "mxnet")
    roles = [(r.role, r.env["DMLC_ROLE"]) for r in plan.replicas]
    assert {x for _, x in roles} >= {"scheduler", "server", "worker"}
    assert all(r.env["DMLC_PS_ROOT_URI"] == "127.0.0.1" for r in plan.replicas)
    assert len({r.env["DMLC_PS_ROOT_PORT"] for r in plan.replicas}) == 1
    assert plan.primary.role == "scheduler"


@need_ref
def test_mpijob_plan_launcher_only():
    plan = _plan("mpijob-horovod.yaml", "training-container")
    assert [r.role for r in plan.replicas] == ["launcher"] and plan.replicas[0].primary
    assert "mpirun" in " ".join(plan.replicas[0].argv)


@need_ref
def test_xgboostjob_plan_ranks():
    plan = _plan("xgboostjob-lightgbm.yaml", "xgboost")
    ranks = [r.env["RANK"] for r in plan.replicas]
    assert ranks == [str(i) for i in range(len(plan.replicas))] and len(plan.replicas) == 3
    assert len({r.env["MASTER_PORT"] for r in plan.replicas}) == 1 and plan.replicas[0].role == "master"


@need_ref
@pytest.mark.parametrize("name,container", [("tfjob-mnist-with-summaries.yaml", "tensorflow"),
                                            ("mxjob-byteps.yaml", "mxnet"),
                                            ("xgboostjob-lightgbm.yaml", "xgboost"),
                                            ("pytorchjob-mnist.yaml", "pytorch")])
def test_assign_ports_redraws_every_rendezvous_port(name, container):
    """a retry (or a launch after waiting for slots) gets fresh ports, consistently
    rewritten in every replica."""
    plan = _plan(name, container)
    before = _ports(plan)
    assign_ports(plan)
    after = _ports(plan)
    assert len(after) == len(before) and not set(after) & set(before)
    if "TF_CONFIG" in plan.replicas[0].env:
        cl = [json.loads(r.env["TF_CONFIG"])["cluster"] for r in plan.replicas]
        assert all(c == cl[0] for c in cl)
    for k in ("MASTER_PORT", "DMLC_PS_ROOT_PORT"):
        vals = {r.env[k] for r in plan.replicas if k in r.env}
        assert len(vals) <= 1


STAND_IN = r'''
import json, os, socket, sys, time
cfg = json.loads(os.environ["TF_CONFIG"])
me = cfg["cluster"][cfg["task"]["type"]][cfg["task"]["index"]]
s = socket.socket(); s.bind(("127.0.0.1", int(me.rsplit(":", 1)[1])))  # my task address is free and mine
assert len(cfg["cluster"]["worker"]) == 2
time.sleep(0.5)
print("accuracy=%.3f" % (0.5 + float(sys.argv[1])))
'''


def test_tfjob_trial_runs_end_to_end_cpu(tmp_path):
    from katib_amd.controller.manager import Manager

    exp = {
        "apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
        "metadata": {"name": "tfjob-standin", "namespace": "default"},
        "spec": {
            "objective": {"type": "maximize", "objectiveMetricName": "accuracy"},
            "algorithm": {"algorithmName": "random"},
            "parallelTrialCount": 2, "maxTrialCount": 2, "maxFailedTrialCount": 0,
            "parameters": [{"name": "x", "parameterType": "double", "feasibleSpace": {"min": "0.1", "max": "0.4"}}],
            "trialTemplate": {
                "primaryContainerName": "tensorflow",
                "trialParameters": [{"name": "x", "reference": "x"}],
                "trialSpec": {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "spec": {"tfReplicaSpecs": {
                    "Worker": {"replicas": 2, "restartPolicy": "OnFailure", "template": {"spec": {"containers": [{
                        "name": "tensorflow", "image": "n/a",
                        "command": [sys.executable, "-c", STAND_IN, "${trialParameters.x}"]}]}}}}}}}}}
    from katib_amd.api.models import V1beta1Experiment

    m = Manager(state_dir=str(tmp_path / "state"), num_devices=0, journal=False)
    try:
        e = V1beta1Experiment.from_k8s(exp)
        m.create_experiment(e)
        done = m.run_until_complete("tfjob-standin", timeout=120)
        trials = m.list_trials("tfjob-standin")
        assert EC.is_succeeded(done), [t.status.conditions[-1].message for t in trials]
        assert done.status.trials_succeeded == 2
        best = done.status.current_optimal_trial
        acc = [float(x.max) for x in best.observation.metrics if x.name == "accuracy"][0]
        assert 0.6 <= acc <= 0.9
    finally:
        m.shutdown()
