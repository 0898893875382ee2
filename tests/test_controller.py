"""End-to-end control plane: experiments run through the in-process scheduler with real
trial subprocesses (reference e2e strategy: test/e2e/v1beta1/scripts/gh-actions/run-e2e-experiment.py
asserts the experiment reaches Succeeded with the expected trial counts and an optimal trial)."""
import json
import os
import sys
import textwrap

import pytest
import yaml

from katib_amd.api import constants as C
from katib_amd.api.conditions import ExperimentConditions as EC
from katib_amd.api.yaml_io import load_experiment

PY = sys.executable
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def quadratic_yaml(name="q", algorithm="random", settings=None, parallel=2, max_trials=6, max_failed=3, goal=None,
                   params=None, command=None, extra_spec=""):
    settings = settings or []
    max_failed = min(max_failed, max_trials)
    params = params or [
        {"name": "a", "parameterType": "double", "feasibleSpace": {"min": "0", "max": "2"}},
        {"name": "b", "parameterType": "double", "feasibleSpace": {"min": "-1", "max": "1"}},
    ]
    names = [p["name"] for p in params]
    if command is None:
        assigns = "; ".join("%s=${trialParameters.%s}" % (n, n) for n in names)
        command = [PY, "-c", "%s; print('result=%%s' %% (4*float(a) - float(b)**2))" % assigns]
    spec = {
        "apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment", "metadata": {"name": name},
        "spec": {
            "objective": {"type": "maximize", "objectiveMetricName": "result"},
            "algorithm": {"algorithmName": algorithm, "algorithmSettings": settings},
            "parallelTrialCount": parallel, "maxTrialCount": max_trials, "maxFailedTrialCount": max_failed,
            "parameters": params,
            "trialTemplate": {
                "primaryContainerName": "training-container",
                "trialParameters": [{"name": n, "reference": n} for n in names],
                "trialSpec": {"apiVersion": "batch/v1", "kind": "Job", "spec": {"template": {"spec": {
                    "containers": [{"name": "training-container", "image": "python", "command": command,
                                    "env": [{"name": "TRIAL_PARAMS", "value": " ".join(
                                        "%s=${trialParameters.%s}" % (n, n) for n in names)}]}],
                    "restartPolicy": "Never"}}}},
            },
        },
    }
    if goal is not None:
        spec["spec"]["objective"]["goal"] = goal
    text = yaml.safe_dump(spec)
    if extra_spec:
        d = yaml.safe_load(text)
        d["spec"].update(yaml.safe_load(extra_spec))
        text = yaml.safe_dump(d)
    return load_experiment(text)


def _reason(e):
    return [c.reason for c in e.status.conditions if c.status == "True"][-1]


def test_random_quadratic_example_completes(manager):
    import os

    e = load_experiment(os.path.join(os.path.dirname(__file__), "..", "examples", "hp-tuning",
                                     "random-quadratic.yaml"))
    e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]["command"][0] = PY
    manager.create_experiment(e)
    done = manager.run_until_complete("random-quadratic", timeout=120)
    assert EC.is_succeeded(done)
    assert _reason(done) in (C.EXPERIMENT_MAX_TRIALS_REACHED_REASON, C.EXPERIMENT_GOAL_REACHED_REASON)
    assert done.status.trials_succeeded >= 1
    best = done.status.current_optimal_trial
    assert best.best_trial_name
    vals = {m.name: float(m.latest) for m in best.observation.metrics}
    a = float([p.value for p in best.parameter_assignments if p.name == "a"][0])
    b = float([p.value for p in best.parameter_assignments if p.name == "b"][0])
    assert abs(vals["result"] - (4 * a - b * b)) < 1e-6
    # every other succeeded trial is no better than the optimum
    for t in manager.list_trials("random-quadratic"):
        if t.status.observation and t.status.observation.metrics:
            assert float(t.status.observation.metrics[0].max) <= vals["result"] + 1e-9
    logs = manager.get_observation_log(best.best_trial_name, "result")
    assert len(logs) == 1 and logs[0][1] == "result"


@pytest.mark.parametrize("algorithm,settings,params", [
    ("random", [{"name": "random_state", "value": "3"}], None),
    ("tpe", [{"name": "random_state", "value": "3"}, {"name": "gamma", "value": "0.3"}], None),
    ("multivariate-tpe", [{"name": "n_startup_trials", "value": "2"}], None),
    ("cmaes", [{"name": "random_state", "value": "3"}], None),
    ("sobol", [], None),
    ("bayesianoptimization", [{"name": "random_state", "value": "3"}, {"name": "n_initial_points", "value": "2"}],
     None),
    ("grid", [], [{"name": "a", "parameterType": "double", "feasibleSpace": {"min": "0", "max": "2", "step": "1"}},
                  {"name": "b", "parameterType": "int", "feasibleSpace": {"min": "-1", "max": "1"}}]),
])
def test_algorithms_end_to_end(manager, algorithm, settings, params):
    e = quadratic_yaml(name="alg-" + algorithm, algorithm=algorithm, settings=settings, params=params,
                       parallel=2, max_trials=6)
    manager.create_experiment(e)
    done = manager.run_until_complete(e.metadata.name, timeout=180)
    assert EC.is_succeeded(done), done.status.conditions
    assert done.status.trials_succeeded == 6
    trials = manager.list_trials(e.metadata.name)
    assert len(trials) == 6
    seen = set()
    for t in trials:
        pa = tuple((p.name, p.value) for p in t.spec.parameter_assignments)
        seen.add(pa)
        for p in t.spec.parameter_assignments:
            v = float(p.value)
            if p.name == "a":
                assert 0 <= v <= 2
            else:
                assert -1 <= v <= 1
    if algorithm == "grid":
        assert len(seen) == 6  # 3 x 3 grid, no repeats


def test_goal_reached(manager):
    e = quadratic_yaml(name="goal", goal=-100.0, parallel=1, max_trials=10)
    manager.create_experiment(e)
    done = manager.run_until_complete("goal", timeout=60)
    assert _reason(done) == C.EXPERIMENT_GOAL_REACHED_REASON
    assert done.status.trials_succeeded == 1


def test_max_failed_trials(manager):
    e = quadratic_yaml(name="failing", command=[PY, "-c", "import sys; sys.exit(3)"], parallel=2, max_trials=6,
                       max_failed=2)
    manager.create_experiment(e)
    done = manager.run_until_complete("failing", timeout=60)
    assert EC.is_failed(done)
    assert _reason(done) == C.EXPERIMENT_FAILED_REASON
    assert done.status.trials_failed >= 2


def test_metrics_unavailable(manager):
    e = quadratic_yaml(name="nometrics", command=[PY, "-c", "print('nothing here')"], parallel=1, max_trials=2,
                       max_failed=2)
    manager.create_experiment(e)
    done = manager.run_until_complete("nometrics", timeout=60)
    trials = manager.list_trials("nometrics")
    assert all(any(c.type == "MetricsUnavailable" and c.status == "True" for c in t.status.conditions)
               for t in trials)
    assert EC.is_failed(done)


def test_file_collector_json_format(manager, tmp_path):
    path = str(tmp_path / "metrics.json")
    code = textwrap.dedent("""
        import json, sys
        a = float(sys.argv[1]); b = float(sys.argv[2])
        with open(%r, "a") as f:
            for step in range(3):
                f.write(json.dumps({"result": str(4*a - b*b - (2 - step)), "step": str(step)}) + "\\n")
    """ % path)
    e = quadratic_yaml(name="filejson", command=[PY, "-c", code, "${trialParameters.a}", "${trialParameters.b}"],
                       parallel=1, max_trials=2,
                       extra_spec=yaml.safe_dump({"metricsCollectorSpec": {
                           "collector": {"kind": "File"},
                           "source": {"fileSystemPath": {"path": path, "kind": "File", "format": "JSON"}}}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("filejson", timeout=60)
    assert EC.is_succeeded(done)
    t = manager.get_trial(done.status.current_optimal_trial.best_trial_name)
    m = t.status.observation.metrics[0]
    assert float(m.max) - float(m.min) == pytest.approx(2.0)


def test_stdout_custom_filter(manager):
    code = "print('epoch 1 acc: 0.5'); print('epoch 2 acc: 0.75')"
    e = quadratic_yaml(name="filter", command=[PY, "-c", code], parallel=1, max_trials=1,
                       params=[{"name": "a", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                       extra_spec=yaml.safe_dump({
                           "objective": {"type": "maximize", "objectiveMetricName": "acc"},
                           "metricsCollectorSpec": {"collector": {"kind": "StdOut"},
                                                    "source": {"filter": {"metricsFormat": [r"(\w+):\s*([\d.]+)"]}}}}))
    e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]["command"].append(
        "${trialParameters.a}")
    manager.create_experiment(e)
    done = manager.run_until_complete("filter", timeout=60)
    m = done.status.current_optimal_trial.observation.metrics[0]
    assert (m.name, m.min, m.max, m.latest) == ("acc", "0.5", "0.75", "0.75")


def test_tfevent_collector(manager, tmp_path):
    logdir = str(tmp_path / "tb")
    code = textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        from katib_amd.metricscollector.tfevent import EventWriter
        w = EventWriter(%r + "/test")
        for s in range(3):
            w.add_scalar("accuracy", 0.5 + 0.1 * s, s)
        w.close()
    """ % (ROOT, logdir))
    e = quadratic_yaml(name="tfevent", command=[PY, "-c", code, "${trialParameters.a}"], parallel=1, max_trials=1,
                       params=[{"name": "a", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                       extra_spec=yaml.safe_dump({
                           "objective": {"type": "maximize", "objectiveMetricName": "test/accuracy"},
                           "metricsCollectorSpec": {"collector": {"kind": "TensorFlowEvent"},
                                                    "source": {"fileSystemPath": {"path": logdir,
                                                                                  "kind": "Directory"}}}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("tfevent", timeout=60)
    assert EC.is_succeeded(done), done.status.conditions
    m = done.status.current_optimal_trial.observation.metrics[0]
    assert m.name == "test/accuracy" and float(m.max) == pytest.approx(0.7) and float(m.min) == pytest.approx(0.5)


def test_medianstop_early_stopping(manager, tmp_path):
    # the k-th trial to start reports loss k + 0.01*step: once two trials have succeeded the
    # median-stop rule (loss > mean of their first start_step values) stops every later one
    counter = str(tmp_path / "counter")
    code = textwrap.dedent("""
        import fcntl, os, sys, time
        with open(%r, "a+") as f:
            fcntl.flock(f, fcntl.LOCK_EX)
            f.seek(0)
            k = len(f.read())
            f.write("x")
        for s in range(12):
            print("loss=%%f" %% (k + 0.01 * s), flush=True)
            time.sleep(0.05)
    """ % counter)
    e = quadratic_yaml(name="medianstop", command=[PY, "-u", "-c", code, "${trialParameters.a}"], parallel=1,
                       max_trials=6,
                       params=[{"name": "a", "parameterType": "double", "feasibleSpace": {"min": "0", "max": "10"}}],
                       extra_spec=yaml.safe_dump({
                           "objective": {"type": "minimize", "objectiveMetricName": "loss"},
                           "earlyStopping": {"algorithmName": "medianstop", "algorithmSettings": [
                               {"name": "min_trials_required", "value": "2"}, {"name": "start_step", "value": "2"}]}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("medianstop", timeout=120)
    trials = sorted(manager.list_trials("medianstop"), key=lambda t: t.metadata.creation_timestamp)
    stopped = [t for t in trials if any(c.type == "EarlyStopped" and c.status == "True" for c in t.status.conditions)]
    assert stopped, [t.status.conditions for t in trials]
    assert all(t.spec.early_stopping_rules for t in stopped)
    rule = stopped[0].spec.early_stopping_rules[0]
    assert rule.name == "loss" and rule.comparison == "greater" and rule.start_step == 2
    assert float(rule.value) == pytest.approx(0.505)  # mean of (0.005, 1.005)
    assert EC.is_succeeded(done)
    assert done.status.trials_early_stopped == len(stopped)
    for t in stopped:  # stopped after start_step reports, long before the 12 steps end
        assert len(manager.get_observation_log(t.metadata.name, "loss")) < 12


def test_resume_long_running(manager):
    e = quadratic_yaml(name="resume", parallel=1, max_trials=2,
                       extra_spec=yaml.safe_dump({"resumePolicy": "LongRunning"}))
    manager.create_experiment(e)
    done = manager.run_until_complete("resume", timeout=60)
    assert _reason(done) == C.EXPERIMENT_MAX_TRIALS_REACHED_REASON
    done.spec.max_trial_count = 4
    manager.update_experiment(done)
    done = manager.run_until_complete("resume", timeout=60)
    assert done.status.trials_succeeded == 4 and EC.is_succeeded(done)


def test_resume_never_is_not_restartable(manager):
    e = quadratic_yaml(name="never", parallel=1, max_trials=1)
    manager.create_experiment(e)
    done = manager.run_until_complete("never", timeout=60)
    done.spec.max_trial_count = 3
    from katib_amd.api.validation import ValidationError

    with pytest.raises(ValidationError):
        manager.update_experiment(done)


def test_delete_experiment_cleans_up(manager):
    e = quadratic_yaml(name="del", parallel=1, max_trials=1)
    manager.create_experiment(e)
    done = manager.run_until_complete("del", timeout=60)
    tname = done.status.current_optimal_trial.best_trial_name
    assert manager.get_observation_log(tname)
    manager.delete_experiment("del")
    assert not manager.list_trials("del")
    assert manager.get_observation_log(tname) == []


def test_hyperband_end_to_end(manager):
    code = "import sys; r=int(sys.argv[2]); print('acc=%f' % (float(sys.argv[1]) * r / 9.0))"
    params = [{"name": "lr", "parameterType": "double", "feasibleSpace": {"min": "0.1", "max": "1.0"}},
              {"name": "epochs", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "9"}}]
    e = quadratic_yaml(name="hb", algorithm="hyperband",
                       settings=[{"name": "resource_name", "value": "epochs"}, {"name": "eta", "value": "3"},
                                 {"name": "r_l", "value": "9"}],
                       params=params, parallel=9, max_trials=20,
                       command=[PY, "-c", code, "${trialParameters.lr}", "${trialParameters.epochs}"],
                       extra_spec=yaml.safe_dump({"objective": {"type": "maximize", "objectiveMetricName": "acc"}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("hb", timeout=180)
    assert EC.is_succeeded(done), done.status.conditions
    epochs = sorted({int(p.value) for t in manager.list_trials("hb") for p in t.spec.parameter_assignments
                     if p.name == "epochs"})
    assert epochs[0] == 1 and 9 in epochs  # first bracket r=1 rung, promoted trials at r_l
    sugg = manager.get_suggestion("hb")
    names = {s.name for s in sugg.status.algorithm_settings}
    assert {"eta", "s_max", "r_l", "current_s", "current_i", "evaluating_trials"} <= names


def test_pbt_end_to_end(manager, tmp_path):
    code = textwrap.dedent("""
        import os, sys, json
        lr = float(sys.argv[1]); d = sys.argv[2]  # suggestion_trial_dir, mapped to the member's dir
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, "ckpt.json")
        st = json.load(open(p)) if os.path.exists(p) else {"step": 0, "acc": 0.0}
        for _ in range(3):
            st["step"] += 1
            st["acc"] += lr * (1.0 - st["acc"])
            print("Validation-accuracy=%f" % st["acc"])
        json.dump(st, open(p, "w"))
    """)
    params = [{"name": "lr", "parameterType": "double", "feasibleSpace": {"min": "0.01", "max": "0.5",
                                                                          "step": "0.01"}}]
    e = quadratic_yaml(name="pbt", algorithm="pbt",
                       settings=[{"name": "suggestion_trial_dir", "value": str(tmp_path / "pbt")},
                                 {"name": "n_population", "value": "5"},
                                 {"name": "truncation_threshold", "value": "0.4"}],
                       params=params, parallel=5, max_trials=15, max_failed=3,
                       command=[PY, "-c", code, "${trialParameters.lr}", str(tmp_path / "pbt")],
                       extra_spec=yaml.safe_dump({"objective": {"type": "maximize",
                                                                "objectiveMetricName": "Validation-accuracy"}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("pbt", timeout=240)
    assert EC.is_succeeded(done), done.status.conditions
    trials = manager.list_trials("pbt")
    gens = {t.metadata.labels.get("pbt.suggestion.katib.kubeflow.org/generation") for t in trials}
    assert len(gens) >= 2
    # children resumed from a parent checkpoint keep improving
    assert float(done.status.current_optimal_trial.observation.metrics[0].max) > 0.5


def test_prometheus_counters(manager):
    e = quadratic_yaml(name="prom", parallel=2, max_trials=3)
    manager.create_experiment(e)
    manager.run_until_complete("prom", timeout=60)
    text = manager.metrics.expose()
    assert 'katib_trial_created_total{namespace="default"} 3' in text
    assert 'katib_experiment_succeeded_total{namespace="default"} 1' in text


def test_function_kind_via_sdk_tune(manager):
    from katib_amd.sdk import KatibClient, search

    def objective(parameters):
        x = float(parameters["x"])
        print("score=%f" % (-(x - 1.0) ** 2))

    client = KatibClient(manager=manager)
    client.tune(name="tune", objective=objective, parameters={"x": search.double(min=-2, max=3)},
                objective_metric_name="score", max_trial_count=4, parallel_trial_count=2,
                algorithm_name="random")
    done = manager.run_until_complete("tune", timeout=120)
    assert EC.is_succeeded(done), done.status.conditions
    assert client.get_optimal_hyperparameters("tune").best_trial_name
    assert done.status.trials_succeeded == 4


def test_trial_timeline_trace(manager, tmp_path):
    """utils/tracing: every trial leaves created -> launched -> first metric -> done, every
    GetSuggestions call a span; the Chrome trace export is valid JSON with those events."""
    import json
    import os

    e = load_experiment(os.path.join(os.path.dirname(__file__), "..", "examples", "hp-tuning",
                                     "random-quadratic.yaml"))
    e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]["command"][0] = PY
    e.spec.max_trial_count = 3
    manager.create_experiment(e)
    done = manager.run_until_complete("random-quadratic", timeout=120)
    assert EC.is_succeeded(done)
    tr = manager.tracer
    names = [t.metadata.name for t in manager.list_trials("random-quadratic")]
    for n in names:
        kinds = [(ev["name"], ev["ph"]) for ev in tr.trial_timeline(n)]
        assert ("trial.created", "i") in kinds and ("trial", "B") in kinds and ("trial", "E") in kinds
        assert ("trial.first_metric", "i") in kinds
    assert any(ev["name"] == "suggestion.GetSuggestions" for ev in tr.events)
    lat = tr.phase_latencies()
    assert lat["run_s"] > 0 and lat["queue_s"] >= 0
    path = tmp_path / "trace.json"
    tr.export(str(path))
    doc = json.loads(path.read_text())
    assert any(ev.get("name") == "trial" and ev.get("ph") == "b" for ev in doc["traceEvents"])


def _cond(t, typ):
    return any(c.type == typ and c.status == "True" for c in t.status.conditions)


def test_fault_injection_paths(manager):
    """controller/faults.FaultPlan drives each failure path deterministically: a launch
    failure, a crash on exit, dropped metrics; the rest of the trials succeed."""
    from katib_amd.controller.faults import FaultPlan

    plan = FaultPlan().add("launch", "fail", index=0).add("exit", "crash", index=1).add("exit", "drop_metrics", index=2)
    manager.fault_injector = plan
    e = quadratic_yaml(name="faults", parallel=1, max_trials=5, max_failed=4)
    manager.create_experiment(e)
    done = manager.run_until_complete("faults", timeout=120)
    trials = sorted(manager.list_trials("faults"), key=lambda t: plan._order.get(t.metadata.name, 99))
    assert [a for _, _, a in plan.log] == ["fail", "crash", "drop_metrics"]
    assert _cond(trials[0], "Failed") and "LaunchError" in trials[0].status.conditions[-1].reason
    assert _cond(trials[1], "Failed")  # crash, backoffLimit 0
    assert _cond(trials[2], "MetricsUnavailable")
    assert all(_cond(t, "Succeeded") for t in trials[3:])
    assert done.status.trials_succeeded == 2


def test_gpu_fault_quarantines_device(tmp_path):
    """A trial dying on SIGSEGV on a GPU records a device fault; the device is quarantined at
    the configured threshold and later trials are placed on the remaining devices."""
    from katib_amd.controller.faults import FaultPlan
    from katib_amd.controller.manager import Manager

    m = Manager(state_dir=str(tmp_path / "state"), num_devices=2, journal=False)
    try:
        m.config.amd.fault_quarantine_threshold = 2
        m.fault_injector = FaultPlan().add("exit", "gpu_fault", index=None, times=2)
        e = quadratic_yaml(name="gfault", parallel=1, max_trials=4, max_failed=4, extra_spec="""
trialTemplate:
  primaryContainerName: training-container
  trialParameters: [{name: a, reference: a}, {name: b, reference: b}]
  trialSpec:
    apiVersion: batch/v1
    kind: Job
    spec:
      template:
        spec:
          containers:
          - name: training-container
            image: python
            command: ["%s", "-c", "print('result=${trialParameters.a}${trialParameters.b}'[:8])"]
            resources: {limits: {amd.com/gpu: 1}}
          restartPolicy: Never
""" % PY)
        m.create_experiment(e)
        done = m.run_until_complete("gfault", timeout=120)
        assert done.status.trials_failed == 2 and done.status.trials_succeeded == 2
        assert len(m.slots.quarantined()) >= 1
    finally:
        m.shutdown()


def test_prometheus_collector(manager):
    """PrometheusMetric: the scheduler scrapes the trial's /metrics endpoint (port from
    KATIB_PROMETHEUS_PORT) and records every changed sample of the experiment's metrics."""
    code = textwrap.dedent("""
        import os, threading, time
        from http.server import BaseHTTPRequestHandler, HTTPServer
        state = {"acc": 0.25, "loss": 2.0}
        class H(BaseHTTPRequestHandler):
            def log_message(self, *a): pass
            def do_GET(self):
                if self.path != os.environ["KATIB_PROMETHEUS_PATH"]:
                    self.send_response(404); self.end_headers(); return
                body = ("# HELP acc accuracy\\n# TYPE acc gauge\\nacc %s\\nloss{split=\\"train\\"} %s\\n"
                        "other_metric 7\\n" % (state["acc"], state["loss"])).encode()
                self.send_response(200); self.send_header("Content-Length", str(len(body))); self.end_headers()
                self.wfile.write(body)
        srv = HTTPServer(("127.0.0.1", int(os.environ["KATIB_PROMETHEUS_PORT"])), H)
        threading.Thread(target=srv.serve_forever, daemon=True).start()
        for acc, loss in ((0.5, 1.0), (0.75, 0.5)):
            time.sleep(0.8)
            state["acc"], state["loss"] = acc, loss
        time.sleep(0.8)  # keep the endpoint up for a last scrape
    """)
    e = quadratic_yaml(name="prom", command=[PY, "-c", code, "${trialParameters.a}"], parallel=1, max_trials=1,
                       params=[{"name": "a", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                       extra_spec=yaml.safe_dump({
                           "objective": {"type": "maximize", "objectiveMetricName": "acc",
                                         "additionalMetricNames": ["loss"]},
                           "metricsCollectorSpec": {"collector": {"kind": "PrometheusMetric"}}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("prom", timeout=60)
    assert EC.is_succeeded(done), done.status.conditions
    ms = {m.name: m for m in done.status.current_optimal_trial.observation.metrics}
    assert (ms["acc"].min, ms["acc"].max, ms["acc"].latest) == ("0.25", "0.75", "0.75")
    assert ms["loss"].latest == "0.5"
    trial = done.status.current_optimal_trial.best_trial_name
    values = [v for _, n, v in manager.get_observation_log(trial) if n == "acc"]
    assert values == ["0.25", "0.5", "0.75"]  # one entry per change, not per scrape


def test_prometheus_final_value_published_right_before_exit(manager):
    """A trial that publishes its objective and exits at once: the value between the last
    scrape and the exit reaches the observation log through KATIB_PROMETHEUS_FINAL."""
    code = textwrap.dedent("""
        import sys
        sys.path.insert(0, %r)
        from katib_amd.metricscollector.prometheus import TrialExporter
        ex = TrialExporter()
        ex.set("acc", 0.125)
        ex.set("acc", 0.875)
        ex.close()
    """ % ROOT)
    e = quadratic_yaml(name="promfinal", command=[PY, "-c", code, "${trialParameters.a}"], parallel=1, max_trials=1,
                       params=[{"name": "a", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "2"}}],
                       extra_spec=yaml.safe_dump({
                           "objective": {"type": "maximize", "objectiveMetricName": "acc"},
                           "metricsCollectorSpec": {"collector": {"kind": "PrometheusMetric"}}}))
    manager.create_experiment(e)
    done = manager.run_until_complete("promfinal", timeout=60)
    assert EC.is_succeeded(done), done.status.conditions
    ms = {m.name: m for m in done.status.current_optimal_trial.observation.metrics}
    assert ms["acc"].latest == "0.875"


def test_prometheus_label_sets_do_not_interleave():
    from katib_amd.metricscollector.prometheus import Scraper

    sc = Scraper(1, "/metrics", ["loss"])
    assert [v for _, _, v in sc.observe('loss{split="train"} 1\nloss{split="val"} 2\n', 0.0)] == ["1"]
    assert sc.observe('loss{split="train"} 1\nloss{split="val"} 3\n', 1.0) == []  # val is ignored
    assert [v for _, _, v in sc.observe('loss 5\nloss{split="train"} 1\n', 2.0)] == ["5"]  # unlabelled wins


def test_prometheus_exposition_parser():
    from katib_amd.metricscollector.prometheus import Scraper, parse_exposition

    text = ("# HELP acc x\n# TYPE acc gauge\nacc 0.5\nacc{split=\"val\"} 0.25 1700000000000\n"
            "accuracy 9\nloss NaN\nbad line here\nloss +Inf\n")
    assert parse_exposition(text, ["acc", "loss"]) == [
        ("acc", "0.5", None), ("acc", "0.25", 1700000000000), ("loss", "NaN", None), ("loss", "+Inf", None)]
    sc = Scraper(1, "/metrics", ["acc"])
    first = sc.observe("acc 1\n", 0.0)
    assert first == [("1970-01-01T00:00:00Z", "acc", "1")]
    assert sc.observe("acc 1\n", 1.0) == [] and sc.observe("acc 2\n", 1.5)[0][2] == "2"
    assert sc.observe("acc 2 1700000000250\n", 2.0) == [("2023-11-14T22:13:20.25Z", "acc", "2")]


def test_free_port_never_repeats_recent_ports():
    """Concurrent trial launches get distinct rendezvous / Prometheus ports (the
    port is probed before the trial binds it, so two launches must not be handed the same one)."""
    import threading

    from katib_amd.controller.jobs import free_port

    got = []
    lock = threading.Lock()

    def take():
        for _ in range(25):
            p = free_port()
            with lock:
                got.append(p)

    ts = [threading.Thread(target=take) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(got) == 200 and len(set(got)) == 200
