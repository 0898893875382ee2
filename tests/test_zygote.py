"""Fork server for cold Python trials: a zygote that has
imported torch (never the GPU) forks one fresh process per trial; the trial is re-parented to the
scheduler (child subreaper) and supervised by the native runtime exactly like an exec'd one."""
import os
import sys
import time

import pytest

from katib_amd.controller.zygote import Zygote


def test_eligible_commands():
    py = sys.executable
    assert Zygote.eligible([py, "-m", "katib_amd.workloads.mnist_mlp", "--epochs=1"])
    assert Zygote.eligible([py, "-c", "print(1)"])
    assert Zygote.eligible([py, "train.py", "--lr=0.1"])
    assert not Zygote.eligible([py, "-u", "-m", "x"])  # interpreter flags: exec
    assert not Zygote.eligible(["/bin/sh", "-c", "echo hi"])
    assert not Zygote.eligible([py])


def _read_all(fd):
    out = b""
    while True:
        b = os.read(fd, 65536)
        if not b:
            return out.decode()
        out += b


def test_zygote_child_env_cwd_exit_code(tmp_path):
    z = Zygote(str(tmp_path), preload="")
    try:
        r, w = os.pipe()
        code = "import os, sys; print('V=%s' % os.environ['KATIB_T'], os.getcwd(), sys.argv[1:]); sys.exit(3)"
        env = dict(os.environ, KATIB_T="42")
        pid = z.spawn([sys.executable, "-c", code, "a", "b"], env, str(tmp_path), w)
        os.close(w)
        out = _read_all(r)
        os.close(r)
        _, st = os.waitpid(pid, 0)  # re-parented to this process (subreaper)
        assert os.WIFEXITED(st) and os.WEXITSTATUS(st) == 3
        assert "V=42" in out and str(tmp_path) in out and "['a', 'b']" in out, out
        # a module run as __main__ with its own process group; uncaught exception -> exit 1 + traceback
        r, w = os.pipe()
        pid = z.spawn([sys.executable, "-c", "import os; print(os.getpgid(0) == os.getpid()); raise ValueError('boom')"],
                      dict(os.environ), str(tmp_path), w)
        os.close(w)
        out = _read_all(r)
        os.close(r)
        _, st = os.waitpid(pid, 0)
        assert os.WEXITSTATUS(st) == 1 and "True" in out and "ValueError: boom" in out, out
    finally:
        z.close()


def test_manager_runs_job_trials_through_zygote(tmp_path):
    """examples/hp-tuning/random-quadratic.yaml (python3 -c trials) end to end: every trial is
    forked by the fork server, metrics are collected, the experiment succeeds; a trial killed by
    the scheduler (deadline) dies with its process group."""
    from katib_amd.api.conditions import ExperimentConditions as EC
    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.controller.manager import Manager

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = load_experiment(os.path.join(root, "examples", "hp-tuning", "random-quadratic.yaml"))
    e.spec.max_trial_count, e.spec.parallel_trial_count = 4, 2
    m = Manager(state_dir=str(tmp_path / "s"), num_devices=0, journal=False)
    assert m.start_zygote(wait=True)
    try:
        m.create_experiment(e)
        done = m.run_until_complete(e.metadata.name, timeout=120)
        assert EC.is_succeeded(done), done.status.conditions
        launchers = {r.launcher for r in m.runs.values()}
        assert launchers == {"zygote"}, launchers
        assert done.status.trials_succeeded == 4
    finally:
        m.shutdown()


def test_zygote_trial_deadline_kill(tmp_path):
    from katib_amd.api.models import V1beta1Experiment
    from katib_amd.controller.manager import Manager

    c = {"name": "c", "command": [sys.executable, "-c",
                                   "import time\nprint('loss=1.0', flush=True)\ntime.sleep(60)", "${trialParameters.x}"]}
    exp = {"apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
           "metadata": {"name": "zy-deadline", "namespace": "default"},
           "spec": {"objective": {"type": "minimize", "objectiveMetricName": "loss"},
                    "algorithm": {"algorithmName": "random"}, "parallelTrialCount": 1, "maxTrialCount": 1,
                    "maxFailedTrialCount": 1,
                    "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                    "trialTemplate": {"primaryContainerName": "c", "trialParameters": [{"name": "x", "reference": "x"}],
                                      "trialSpec": {"apiVersion": "batch/v1", "kind": "Job", "spec": {
                                          "activeDeadlineSeconds": 2,
                                          "template": {"spec": {"containers": [c]}}}}}}}
    m = Manager(state_dir=str(tmp_path / "s"), num_devices=0, journal=False)
    assert m.start_zygote(wait=True)
    try:
        t0 = time.time()
        m.create_experiment(V1beta1Experiment.from_k8s(exp))
        m.run_until_complete("zy-deadline", timeout=60)
        assert time.time() - t0 < 30
        t = m.list_trials("zy-deadline")[0]
        assert t.status.conditions[-1].type == "Failed", t.status.conditions[-1]
        assert {r.launcher for r in m.runs.values()} == {"zygote"}
    finally:
        m.shutdown()


def test_trials_before_the_server_is_up_are_execd(tmp_path):
    """The fork server starts with the first eligible trial; trials launched while it imports torch
    are fork+exec'd instead of waiting for it, later ones are forked from it."""
    from katib_amd.api.conditions import ExperimentConditions as EC
    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.controller.manager import Manager

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = load_experiment(os.path.join(root, "examples", "hp-tuning", "random-quadratic.yaml"))
    e.spec.max_trial_count, e.spec.parallel_trial_count, e.spec.max_failed_trial_count = 2, 1, 1
    m = Manager(state_dir=str(tmp_path / "s"), num_devices=0, journal=False)
    try:
        m.create_experiment(e)
        done = m.run_until_complete(e.metadata.name, timeout=120)
        assert EC.is_succeeded(done)
        first = min(m.runs.values(), key=lambda r: r.started)
        assert first.launcher == "exec"
    finally:
        m.shutdown()
