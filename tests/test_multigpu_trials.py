"""Multi-GPU trials through the scheduler (VERDICT r2 'Next round' item 1).

A ``batch/v1 Job`` / ``LocalProcess`` trial asking for ``amd.com/gpu: N`` runs as N rank
processes with the torchrun env; rank 0 is the metrics primary; every rank sees the trial's
whole device list and picks ``LOCAL_RANK % device_count`` (``parallel/comm.py``). On CPU
the ranks fall back to gloo, so the same plans run end to end here."""
import os

import pytest

from katib_amd.api.conditions import ExperimentConditions as EC
from katib_amd.api.yaml_io import load_experiment
from katib_amd.controller.jobs import JobSpecError, make_plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def _job(gpus, env=None):
    c = {"name": "training-container", "command": ["python3", "-m", "x"], "resources": {"limits": {"amd.com/gpu": gpus}}}
    if env:
        c["env"] = [{"name": k, "value": v} for k, v in env.items()]
    return {"apiVersion": "batch/v1", "kind": "Job", "spec": {"template": {"spec": {"containers": [c]}}}}


def test_job_two_gpus_is_two_ranks():
    plan = make_plan(_job(2), "training-container")
    assert plan.share_devices and plan.total_gpus == 2 and len(plan.replicas) == 2
    r0, r1 = plan.replicas
    assert r0.primary and not r1.primary and r0.gpus == r1.gpus == 1
    for i, r in enumerate(plan.replicas):
        e = r.env
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(i), str(i), "2", "2")
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == r0.env["MASTER_PORT"]
        assert r.argv == ["python3", "-m", "x"]


def test_single_launch_opt_out_and_one_gpu():
    plan = make_plan(_job(4, {"KATIB_AMD_LAUNCH": "single"}), "training-container")
    assert len(plan.replicas) == 1 and plan.replicas[0].gpus == 4 and not plan.share_devices
    assert len(make_plan(_job(4), "training-container", multi_gpu_launch="single").replicas) == 1
    plan = make_plan(_job(1), "training-container")
    assert len(plan.replicas) == 1 and "RANK" not in plan.replicas[0].env
    with pytest.raises(JobSpecError):
        make_plan(_job(2, {"KATIB_AMD_LAUNCH": "bogus"}), "training-container")


def test_local_process_entrypoint_ranks():
    spec = {"apiVersion": "katib-amd.io/v1", "kind": "LocalProcess",
            "spec": {"entrypoint": "katib_amd.workloads.mnist_mlp:main", "gpus": 3, "args": ["--epochs=1"]}}
    plan = make_plan(spec, "")
    assert len(plan.replicas) == 3 and all(r.entrypoint for r in plan.replicas)
    assert [r.env["RANK"] for r in plan.replicas] == ["0", "1", "2"]


def test_pytorchjob_replicas_share_devices():
    e = load_experiment(os.path.join(EX, "distributed", "pytorchjob-mnist.yaml"))
    plan = make_plan(e.spec.trial_template.trial_spec, "pytorch")
    assert plan.share_devices
    ranks = [(r.env["RANK"], r.env["LOCAL_RANK"], r.env["LOCAL_WORLD_SIZE"]) for r in plan.replicas]
    assert ranks == [(str(i), str(i), str(len(plan.replicas))) for i in range(len(plan.replicas))]


def test_slot_pool_stacks_slots_on_one_device():
    from katib_amd import native

    N = native.load()
    p = N.SlotPool(1, 2)
    assert p.acquire(2) == [0, 0] and p.acquire(1) == []
    q = N.SlotPool(4, 2)
    a = q.acquire(4)
    assert sorted(a) == [0, 1, 2, 3]


def _darts_2gpu():
    e = load_experiment(os.path.join(EX, "nas", "darts-cifar10.yaml"))
    c = e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]
    c["resources"] = {"limits": {"amd.com/gpu": 2}}
    return e, c


def test_darts_job_two_gpus_runs_two_ranks_cpu(tmp_path):
    """examples/nas/darts-cifar10.yaml with amd.com/gpu: 2 on a node with 1 (fake) GPU and two
    slots per GPU: two rank processes (gloo on CPU), one Best-Genotype from rank 0."""
    from katib_amd.controller.manager import Manager

    m = Manager(state_dir=str(tmp_path / "state"), num_devices=1, journal=False)
    m.config.amd.slots_per_device = 2
    m.slots = m.N.SlotPool(1, 2)
    try:
        e, c = _darts_2gpu()
        c["command"] += ["--num-train=64", "--max-steps=1", "--capture=0", "--ops=torch"]
        for s in e.spec.algorithm.algorithm_settings:
            if s.name == "num_epochs":
                s.value = "1"
        e.spec.algorithm.algorithm_settings.append(
            type(e.spec.algorithm.algorithm_settings[0])(name="batch_size", value="8"))
        m.create_experiment(e)
        done = m.run_until_complete(e.metadata.name, timeout=600)
        trials = m.list_trials(e.metadata.name)
        assert EC.is_succeeded(done), [t.status.conditions[-1].message for t in trials]
        t = m.get_trial(done.status.current_optimal_trial.best_trial_name)
        geno = [x for x in t.status.observation.metrics if x.name == "Best-Genotype"]
        assert geno and geno[0].latest.startswith("Genotype(normal=")
        tdir = os.path.join(m.state_dir, "trials", "default", t.metadata.name)
        assert os.path.exists(os.path.join(tdir, "rank-1.log"))  # the second rank ran, logged apart
        log0 = open(os.path.join(tdir, "metrics.log")).read()
        assert log0.count("Best-Genotype=") == 1
    finally:
        m.shutdown()


RANK_CRASH = r'''
import os, sys, time
rank = int(os.environ["RANK"])
open(os.path.join(sys.argv[1], "rank%d.pid" % rank), "w").write(str(os.getpid()))
if rank == 1:
    time.sleep(1.0)
    os.kill(os.getpid(), 9)  # a rank dies mid-run (OOM kill, segfault, ...)
for i in range(600):  # rank 0 would keep "training" for a minute
    print("loss=%f" % (1.0 / (i + 1)), flush=True)
    time.sleep(0.1)
'''


def test_crashed_rank_fails_trial_and_stops_rank0(tmp_path):
    """when a non-primary rank of a 2-rank trial dies, the trial is Failed and
    rank 0 is stopped within seconds (it would otherwise run on - or hang in its next collective)."""
    import signal
    import sys
    import time

    from katib_amd.api.models import V1beta1Experiment
    from katib_amd.controller.manager import Manager

    piddir = tmp_path / "pids"
    piddir.mkdir()
    c = {"name": "training-container", "command": [sys.executable, "-c", RANK_CRASH, str(piddir), "${trialParameters.x}"],
         "resources": {"limits": {"amd.com/gpu": 2}}}
    exp = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
           "metadata": {"name": "rank-crash", "namespace": "default"},
           "spec": {"objective": {"type": "minimize", "objectiveMetricName": "loss"},
                    "algorithm": {"algorithmName": "random"}, "parallelTrialCount": 1, "maxTrialCount": 1,
                    "maxFailedTrialCount": 1,
                    "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                    "trialTemplate": {"primaryContainerName": "training-container",
                                      "trialParameters": [{"name": "x", "reference": "x"}],
                                      "trialSpec": {"apiVersion": "batch/v1", "kind": "Job", "spec": {"template": {
                                          "spec": {"containers": [c], "restartPolicy": "Never"}}}}}}}
    m = Manager(state_dir=str(tmp_path / "state"), num_devices=1, journal=False)
    m.config.amd.slots_per_device = 2
    m.slots = m.N.SlotPool(1, 2)
    m.config.amd.warm_workers = False
    try:
        m.create_experiment(V1beta1Experiment.from_k8s(exp))
        t0 = time.time()
        done = m.run_until_complete("rank-crash", timeout=60)
        wall = time.time() - t0
        trials = m.list_trials("rank-crash")
        assert len(trials) == 1
        conds = [c.type for c in trials[0].status.conditions]
        assert "Failed" in conds, conds
        assert EC.is_failed(done) or EC.is_succeeded(done)
        assert wall < 20, wall
        pid0 = int((piddir / "rank0.pid").read_text())
        deadline = time.time() + 10
        alive = True
        while time.time() < deadline and alive:
            try:
                os.kill(pid0, 0)
                with open("/proc/%d/stat" % pid0) as f:
                    alive = f.read().split()[2] != "Z"
            except (OSError, ProcessLookupError):
                alive = False
            time.sleep(0.1)
        if alive:
            os.kill(pid0, signal.SIGKILL)
        assert not alive, "rank 0 kept running after rank 1 died"
    finally:
        m.shutdown()


def test_single_process_multi_gpu_needs_distinct_devices(tmp_path):
    """slots stack on one device only for rank plans (one process per slot). A single
    process asking for 2 GPUs on a 1-GPU node with 2 slots per device is Unschedulable instead of
    silently getting devices [0, 0]."""
    from katib_amd import native
    from katib_amd.api.models import V1beta1Experiment
    from katib_amd.controller.manager import Manager

    N = native.load()
    p = N.SlotPool(1, 2)
    assert p.acquire(2, True) == [] and p.acquire(2) == [0, 0]
    q = N.SlotPool(3, 2)
    assert sorted(q.acquire(3, True)) == [0, 1, 2] and sorted(q.acquire(3, True)) == [0, 1, 2]
    assert q.acquire(1, True) == []

    c = {"name": "c", "command": ["python3", "-c", "print('loss=1')"], "resources": {"limits": {"amd.com/gpu": 2}},
         "env": [{"name": "KATIB_AMD_LAUNCH", "value": "single"}]}
    exp = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
           "metadata": {"name": "single-2gpu", "namespace": "default"},
           "spec": {"objective": {"type": "minimize", "objectiveMetricName": "loss"},
                    "algorithm": {"algorithmName": "random"}, "parallelTrialCount": 1, "maxTrialCount": 1,
                    "maxFailedTrialCount": 1,
                    "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                    "trialTemplate": {"primaryContainerName": "c", "trialParameters": [{"name": "x", "reference": "x"}],
                                      "trialSpec": {"apiVersion": "batch/v1", "kind": "Job", "spec": {"template": {
                                          "spec": {"containers": [dict(c, args=["${trialParameters.x}"])]}}}}}}}
    m = Manager(state_dir=str(tmp_path / "state"), num_devices=1, journal=False)
    m.config.amd.slots_per_device = 2
    m.slots = m.N.SlotPool(1, 2)
    try:
        m.create_experiment(V1beta1Experiment.from_k8s(exp))
        m.run_until_complete("single-2gpu", timeout=30)
        t = m.list_trials("single-2gpu")[0]
        assert t.status.conditions[-1].reason.endswith("Unschedulable"), t.status.conditions[-1]
    finally:
        m.shutdown()


def test_multi_replica_multi_gpu_job_is_scheduled(tmp_path):
    """a PyTorchJob with Master (2 GPUs) + Worker (2 GPUs) on a 2-device node with two
    slots per device fits (4 slots) and its replicas share the trial's devices, so it must launch
    instead of pending forever on an all-distinct request for 4 devices."""
    import sys

    from katib_amd.api.models import V1beta1Experiment
    from katib_amd.controller.manager import Manager

    def rep(name):
        return {"replicas": 1, "template": {"spec": {"containers": [
            {"name": "pytorch", "command": [sys.executable, "-c", "print('loss=0.5')", "${trialParameters.x}"],
             "resources": {"limits": {"amd.com/gpu": 2}}}]}}}

    spec = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "spec": {"pytorchReplicaSpecs": {"Master": rep("m"), "Worker": rep("w")}}}
    plan = make_plan(spec, "pytorch")
    assert plan.share_devices and plan.total_gpus == 4
    exp = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
           "metadata": {"name": "ptj-4gpu", "namespace": "default"},
           "spec": {"objective": {"type": "minimize", "objectiveMetricName": "loss"},
                    "algorithm": {"algorithmName": "random"}, "parallelTrialCount": 1, "maxTrialCount": 1,
                    "maxFailedTrialCount": 1,
                    "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                    "trialTemplate": {"primaryContainerName": "pytorch",
                                      "trialParameters": [{"name": "x", "reference": "x"}],
                                      "trialSpec": spec}}}
    m = Manager(state_dir=str(tmp_path / "state"), num_devices=2, journal=False)
    m.config.amd.slots_per_device = 2
    m.slots = m.N.SlotPool(2, 2)
    m.config.amd.warm_workers = False
    try:
        m.create_experiment(V1beta1Experiment.from_k8s(exp))
        done = m.run_until_complete("ptj-4gpu", timeout=60)
        t = m.list_trials("ptj-4gpu")[0]
        assert EC.is_succeeded(done), t.status.conditions[-1]
        assert t.status.conditions[-1].type == "Succeeded", t.status.conditions[-1]
    finally:
        m.shutdown()


def test_distinct_request_beyond_healthy_devices_is_unschedulable(tmp_path):
    """A single process asking for more distinct GPUs than the node has healthy (quarantined
    devices excluded) fails Unschedulable instead of pending forever."""
    import sys

    from katib_amd.api.models import V1beta1Experiment
    from katib_amd.controller.manager import Manager

    c = {"name": "c", "command": [sys.executable, "-c", "print('loss=1')", "${trialParameters.x}"],
         "resources": {"limits": {"amd.com/gpu": 2}}, "env": [{"name": "KATIB_AMD_LAUNCH", "value": "single"}]}
    exp = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
           "metadata": {"name": "single-2gpu-q", "namespace": "default"},
           "spec": {"objective": {"type": "minimize", "objectiveMetricName": "loss"},
                    "algorithm": {"algorithmName": "random"}, "parallelTrialCount": 1, "maxTrialCount": 1,
                    "maxFailedTrialCount": 1,
                    "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                    "trialTemplate": {"primaryContainerName": "c", "trialParameters": [{"name": "x", "reference": "x"}],
                                      "trialSpec": {"apiVersion": "batch/v1", "kind": "Job", "spec": {"template": {
                                          "spec": {"containers": [c]}}}}}}}
    m = Manager(state_dir=str(tmp_path / "state"), num_devices=2, journal=False)
    m.config.amd.slots_per_device = 2
    m.slots = m.N.SlotPool(2, 2)
    m.slots.quarantine(1)
    try:
        m.create_experiment(V1beta1Experiment.from_k8s(exp))
        m.run_until_complete("single-2gpu-q", timeout=30)
        t = m.list_trials("single-2gpu-q")[0]
        assert t.status.conditions[-1].reason.endswith("Unschedulable"), t.status.conditions[-1]
    finally:
        m.shutdown()
