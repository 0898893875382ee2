"""CLI, HTTP API daemon, remote SDK client, standalone gRPC servers and the standalone
file metrics collector (reference binaries: katib-controller, db-manager, suggestion
and early-stopping services, file-metricscollector)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(ROOT, "examples", "hp-tuning", "random-quadratic.yaml")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    return dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))


def _start(args, ready):
    p = subprocess.Popen([sys.executable, "-m", "katib_amd"] + args, stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True, env=_env(), cwd=ROOT)
    t0 = time.time()
    lines = []
    while time.time() - t0 < 60:
        ln = p.stdout.readline()
        if not ln:
            break
        lines.append(ln)
        if ready in ln:
            return p, ln
    p.kill()
    raise RuntimeError("server did not start: %s" % "".join(lines))


def _stop(p):
    p.terminate()
    try:
        p.wait(timeout=20)
    except subprocess.TimeoutExpired:
        p.kill()


def test_cli_run_example(tmp_path):
    out = subprocess.run([sys.executable, "-m", "katib_amd", "run", EXAMPLE, "--gpus", "0", "--json",
                          "--state-dir", str(tmp_path)], capture_output=True, text=True, env=_env(), cwd=ROOT,
                         timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["condition"] == "Succeeded" and res["optimal_trial"]["metrics"]["result"]


def test_serve_remote_client_and_ui_endpoints(tmp_path):
    port = _port()
    p, _ = _start(["serve", "--port", str(port), "--state-dir", str(tmp_path), "--gpus", "0"], '"api"')
    try:
        from katib_amd.api.yaml_io import load_experiment
        from katib_amd.sdk import KatibClient

        client = KatibClient(host="http://127.0.0.1:%d" % port)
        e = load_experiment(EXAMPLE)
        e.spec.max_trial_count = 3
        e.spec.max_failed_trial_count = 1
        client.create_experiment(e)
        with pytest.raises(RuntimeError):
            client.create_experiment(e)  # already exists
        client.wait_for_experiment_condition("random-quadratic", timeout=120, polling_interval=0.5)
        best = client.get_optimal_hyperparameters("random-quadratic")
        assert best.best_trial_name
        assert client.get_trial_metrics(best.best_trial_name)
        assert len(client.list_trials("random-quadratic")) == 3
        import urllib.request

        base = "http://127.0.0.1:%d" % port
        csv = json.loads(urllib.request.urlopen(
            base + "/katib/fetch_hp_job_info/?experimentName=random-quadratic&namespace=default").read())
        head, *rows = csv.splitlines()
        assert head == "Status,trialName,result,a,b" and len(rows) == 3
        info = json.loads(urllib.request.urlopen(
            base + "/katib/fetch_hp_job_trial_info/?trialName=%s&namespace=default" % best.best_trial_name).read())
        assert info.startswith("metricName,time,value\nresult,")
        assert "katib_trial_created_total" in urllib.request.urlopen(base + "/metrics").read().decode()
        client.delete_experiment("random-quadratic")
        assert client.list_experiments() == []
    finally:
        _stop(p)


def test_daemon_cli_apply_get(tmp_path):
    port = _port()
    p, _ = _start(["serve", "--port", str(port), "--state-dir", str(tmp_path), "--gpus", "0"], '"api"')
    try:
        host = ["--host", "http://127.0.0.1:%d" % port]
        out = subprocess.run([sys.executable, "-m", "katib_amd", "apply", "-f", EXAMPLE] + host, capture_output=True,
                             text=True, env=_env(), cwd=ROOT, timeout=60)
        assert "created" in out.stdout, out.stderr
        for _ in range(240):
            out = subprocess.run([sys.executable, "-m", "katib_amd", "get", "experiments"] + host,
                                 capture_output=True, text=True, env=_env(), cwd=ROOT, timeout=60)
            if "Succeeded" in out.stdout:
                break
            time.sleep(0.5)
        assert "Succeeded" in out.stdout
        out = subprocess.run([sys.executable, "-m", "katib_amd", "get", "trials", "-e", "random-quadratic"] + host,
                             capture_output=True, text=True, env=_env(), cwd=ROOT, timeout=60)
        assert "result=" in out.stdout
    finally:
        _stop(p)


def test_db_manager_and_file_metrics_collector(tmp_path):
    import grpc

    from katib_amd.rpc import api_pb2 as api
    from katib_amd.rpc.client import DBManagerStub

    port = _port()
    p, _ = _start(["db-manager", "--address", "127.0.0.1:%d" % port, "--journal", str(tmp_path / "obs.jsonl")],
                  "listening")
    try:
        log = str(tmp_path / "metrics.log")
        code = "import time\nfor i in range(50):\n    print('loss=%f' % (1.0 - 0.001 * i), flush=True)\n" \
               "    time.sleep(0.02)\n"
        out = subprocess.run([sys.executable, "-m", "katib_amd", "metrics-collector", "-t", "trial-x", "-m",
                              "loss", "-o-type", "minimize", "-s-db", "127.0.0.1:%d" % port, "-path", log,
                              "-stop-rule", "loss;0.99;greater;3", "--", sys.executable, "-c", code],
                             capture_output=True, text=True, env=_env(), cwd=ROOT, timeout=120)
        assert out.returncode == 0, out.stdout + out.stderr
        with grpc.insecure_channel("127.0.0.1:%d" % port) as ch:
            rep = DBManagerStub(ch).GetObservationLog(api.GetObservationLogRequest(trial_name="trial-x"))
        vals = [float(m.metric.value) for m in rep.observation_log.metric_logs]
        # stopped early: best loss still > 0.99 after the 3rd report, long before the 50 steps finish
        assert 3 <= len(vals) < 50 and vals[0] == 1.0
    finally:
        _stop(p)


def test_suggestion_server_grpc():
    import grpc

    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.api.defaults import set_default
    from katib_amd.controller.converters import convert_experiment
    from katib_amd.rpc import api_pb2 as api
    from katib_amd.rpc.client import HealthStub, SuggestionStub

    port = _port()
    p, _ = _start(["suggestion-server", "--algorithm", "random", "--address", "127.0.0.1:%d" % port], "listening")
    try:
        e = set_default(load_experiment(EXAMPLE))
        with grpc.insecure_channel("127.0.0.1:%d" % port) as ch:
            req = api.GetSuggestionsRequest(experiment=convert_experiment(e, None), trials=[],
                                            current_request_number=3, total_request_number=3)
            rep = SuggestionStub(ch).GetSuggestions(req, timeout=30)
            assert len(rep.parameter_assignments) == 3
            SuggestionStub(ch).ValidateAlgorithmSettings(
                api.ValidateAlgorithmSettingsRequest(experiment=convert_experiment(e, None)), timeout=30)
            assert HealthStub(ch).Check(api.HealthCheckRequest(service="")).status == 1
    finally:
        _stop(p)


def test_ui_backend_routes(manager):
    """UI backend routes of cmd/ui/v1beta1/main.go:48-70 on the in-process server: index,
    experiments CRUD, trial/suggestion fetch, trial logs, namespaces, template CRUD."""
    import urllib.error
    import urllib.request

    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.controller.apiserver import ApiServer

    srv = ApiServer(manager, port=0).start()
    base = "http://127.0.0.1:%d" % srv.port

    def call(path, body=None):
        req = urllib.request.Request(base + path, data=None if body is None else json.dumps(body).encode(),
                                     method="GET" if body is None else "POST")
        try:
            return urllib.request.urlopen(req).read()
        except urllib.error.HTTPError as ex:
            raise AssertionError("%s: %s" % (path, ex.read().decode()))

    try:
        page = call("/katib/")
        for el in (b'id="exps"', b'id="v-create"', b"formExperiment", b"parallel(", b"genotypeSvg"):
            assert el in page  # list, creation wizard, trials charts, NAS architecture view
        algos = json.loads(call("/katib/fetch_algorithms"))
        assert "random" in algos["algorithms"] and "medianstop" in algos["earlyStopping"]
        e = load_experiment(EXAMPLE)
        e.spec.max_trial_count, e.spec.parallel_trial_count, e.spec.max_failed_trial_count = 2, 1, 1
        import yaml as _yaml

        call("/katib/create_experiment/", {"postData": _yaml.safe_dump(e.to_k8s())})  # the editor sends YAML text
        manager.run_until_complete("random-quadratic", timeout=120)
        try:  # a finished experiment with resumePolicy Never cannot be restarted (validator.go:98-124)
            call("/katib/edit_experiment_budget", {"experimentName": "random-quadratic", "namespace": "default",
                                                   "maxTrialCount": 4})
            raise RuntimeError("budget edit of a finished Never-policy experiment was accepted")
        except AssertionError as ex:
            assert "can be restarted" in str(ex)
        exps = json.loads(call("/katib/fetch_experiments/?namespace=default"))
        assert [(x["name"], x["type"], x["status"]) for x in exps] == [("random-quadratic", "hp", "Succeeded")]
        assert exps[0]["trialsSucceeded"] == 2
        got = json.loads(call("/katib/fetch_experiment/?experimentName=random-quadratic&namespace=default"))
        assert got["spec"]["maxTrialCount"] == 2
        sug = json.loads(call("/katib/fetch_suggestion/?suggestionName=random-quadratic&namespace=default"))
        assert sug["kind"] == "Suggestion"
        trial = manager.list_trials("random-quadratic")[0].metadata.name
        tj = json.loads(call("/katib/fetch_trial/?trialName=%s&namespace=default" % trial))
        assert tj["metadata"]["name"] == trial
        logs = json.loads(call("/katib/fetch_trial_logs/?trialName=%s&namespace=default" % trial))
        assert "result=" in logs
        assert "default" in json.loads(call("/katib/fetch_namespaces"))
        # template add / edit / delete (util.go:180-240)
        tpl = {"updatedConfigMapNamespace": "default", "updatedConfigMapName": "my-templates",
               "updatedConfigMapPath": "a.yaml", "updatedTemplateYaml": "kind: Job\n"}
        view = json.loads(call("/katib/add_template/", tpl))["Data"]
        names = {(d["ConfigMapNamespace"], c["ConfigMapName"]) for d in view for c in d["ConfigMaps"]}
        assert ("default", "my-templates") in names
        view = json.loads(call("/katib/edit_template/", dict(tpl, configMapPath="a.yaml", updatedConfigMapPath="b.yaml",
                                                               updatedTemplateYaml="kind: Job # v2\n")))["Data"]
        cm = [c for d in view for c in d["ConfigMaps"] if c["ConfigMapName"] == "my-templates"][0]
        assert cm["Templates"] == [{"Path": "b.yaml", "Yaml": "kind: Job # v2\n"}]
        view = json.loads(call("/katib/delete_template/", dict(tpl, updatedConfigMapPath="b.yaml")))["Data"]
        assert not [c for d in view for c in d["ConfigMaps"] if c["ConfigMapName"] == "my-templates"]
        assert json.loads(call("/katib/delete_experiment/?experimentName=random-quadratic&namespace=default")) == []
    finally:
        srv.stop()


def test_ui_frontend_endpoints_exist(manager):
    """Contract between the single-page UI and its backend: every ``/katib/...`` path the page
    calls is routed by the API server (a request may fail on its arguments or a missing resource,
    but never with the unrouted-path answer)."""
    import re
    import urllib.error
    import urllib.request

    from katib_amd.controller.apiserver import ApiServer

    page = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "katib_amd", "controller",
                             "ui", "index.html")).read()
    paths = sorted(set(re.findall(r"""["'`](/katib/[a-z_]+)""", page)))
    assert len(paths) >= 10, paths
    srv = ApiServer(manager, port=0).start()
    base = "http://127.0.0.1:%d" % srv.port
    post_only = ("create_experiment", "edit_experiment_budget", "add_template", "edit_template", "delete_template")
    try:
        for p in paths:
            post = any(p.endswith(x) for x in post_only)
            req = urllib.request.Request(base + p + ("" if post else "?namespace=default"),
                                         data=b"{}" if post else None, method="POST" if post else "GET")
            try:
                code, body = urllib.request.urlopen(req).status, b""
            except urllib.error.HTTPError as ex:
                code, body = ex.code, ex.read()
            assert b"could not find the requested resource" not in body, (p, code, body[:200])
    finally:
        srv.stop()
