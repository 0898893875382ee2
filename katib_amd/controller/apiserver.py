"""HTTP JSON API over a :class:`~katib_amd.controller.manager.Manager` - the node's
replacement for the Kubernetes API server (CRUD on Experiments/Trials/Suggestions)
plus the Katib UI backend endpoints (reference ``pkg/ui/v1beta1/backend.go:49-772``,
``hp.go:38-320``, ``nas.go:30-109``) and the Prometheus ``/metrics`` endpoint
(reference ``cmd/katib-controller`` metricsAddr ``:8080``).

Routes (``{ns}`` = namespace):

* ``GET/POST /apis/kubeflow.org/v1beta1/namespaces/{ns}/experiments`` (POST body YAML or JSON)
* ``GET/PUT/DELETE /apis/kubeflow.org/v1beta1/namespaces/{ns}/experiments/{name}``
* ``GET /apis/kubeflow.org/v1beta1/namespaces/{ns}/trials[?labelSelector=katib.kubeflow.org/experiment=X]``
* ``GET /apis/kubeflow.org/v1beta1/namespaces/{ns}/trials/{name}``, ``.../suggestions[/{name}]``
* ``POST /api/v1/namespaces/{ns}/configmaps`` (trial templates), ``GET`` to list
* ``GET /katib/observation_logs?trialName=&metricName=&startTime=&endTime=``
* ``GET /katib/fetch_hp_job_info/?experimentName=&namespace=`` - JSON-encoded CSV
  ``Status,trialName,<objective>,<additional...>,<params...>`` with the best value per
  metric, as the reference UI backend returns it
* ``GET /katib/fetch_hp_job_trial_info/?trialName=&namespace=`` - JSON-encoded CSV
  ``metricName,time,value``
* ``GET /katib/fetch_nas_job_info/?experimentName=&namespace=`` - per-trial architecture
* ``GET /metrics``, ``/healthz``, ``/readyz``

Errors come back as ``{"kind": "Status", "code": c, "reason": r, "message": m}``
(400 invalid, 404 not found, 409 already exists) so the remote client can raise the
same exceptions as the in-process one.
"""

from __future__ import annotations

import json
import os
import re
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Optional
from urllib.parse import parse_qs, urlparse

import yaml

from ..api import constants as C
from ..api.models import V1beta1Experiment
from ..api.validation import ValidationError

_API = re.compile(r"^/apis/kubeflow\.org/v1beta1/namespaces/([^/]+)/(experiments|trials|suggestions)(?:/([^/]+))?/?$")
_CM = re.compile(r"^/api/v1/namespaces/([^/]+)/configmaps/?$")


class _Err(Exception):
    def __init__(self, code, reason, message):
        super().__init__(message)
        self.code, self.reason, self.message = code, reason, message


def _best_values(trial, logs):
    """Best value per metric by objective direction (hp.go:140-166)."""
    best = {}
    minimize = trial.spec.objective.type == "minimize"
    for _, name, value in logs:
        if name not in best:
            best[name] = value
            continue
        try:
            cur, prev = float(value), float(best[name])
        except ValueError:
            continue
        if (minimize and cur < prev) or (not minimize and cur > prev):
            best[name] = value
    return best


COOKIE = "katib_amd_token"  # UI session cookie name (see Handler._authorized)


def is_loopback(address: str) -> bool:
    """True for addresses only this host can reach (127.0.0.0/8, ::1, localhost, unix sockets).
    An empty host, ``0.0.0.0`` and ``::`` bind every interface: exposed."""
    host = address.rsplit(":", 1)[0] if address.count(":") == 1 else address
    host = host.strip("[]")
    if address.startswith("unix:") or host in ("localhost", "::1"):
        return True
    return host.startswith("127.")


class ApiServer:
    """HTTP API + UI. ``token``: when set, every request except the health probes must carry
    ``Authorization: Bearer <token>`` (the reference sits behind cluster auth / ingress; a node
    daemon that accepts trial commands must not be open to the network)."""

    def __init__(self, manager, address: str = "127.0.0.1", port: int = 8080, token: Optional[str] = None):
        self.m = manager
        self.token = token or None
        handler = self._make_handler()
        self.httpd = ThreadingHTTPServer((address, port), handler)
        self.port = self.httpd.server_address[1]
        self._thread: Optional[threading.Thread] = None

    def start(self):
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="katib-amd-api", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    # ------------------------------------------------------------------ dispatch
    def handle(self, method: str, path: str, query: dict, body: bytes):
        m = self.m
        if path in ("/healthz", "/readyz"):
            return 200, "text/plain", b"ok"
        if path == "/metrics":
            return 200, "text/plain; version=0.0.4", m.metrics.expose().encode()
        if path in ("/openapi/v2", "/swagger.json"):  # generated from the model table (api/openapi.py)
            from ..api import openapi

            return 200, "application/json", openapi.dumps(include_k8s=True).encode()
        if path == "/katib/trace":  # Chrome/Perfetto timeline of trials and suggestion calls
            return _json(m.tracer.chrome_trace())
        if path == "/katib/trace/latencies":
            return _json(m.tracer.phase_latencies())
        if path == "/katib/observation_logs":
            logs = m.get_observation_log(_q(query, "trialName"), _q(query, "metricName", ""),
                                         _q(query, "startTime", ""), _q(query, "endTime", ""))
            return _json({"metricLogs": [{"timeStamp": t, "metric": {"name": n, "value": v}} for t, n, v in logs]})
        ui = self._ui(method, path.rstrip("/"), query, body)
        if ui is not None:
            return ui
        if path.rstrip("/") == "/katib/fetch_hp_job_info":
            return _json(self._hp_job_info(_q(query, "experimentName"), _q(query, "namespace")))
        if path.rstrip("/") == "/katib/fetch_hp_job_trial_info":
            return _json(self._hp_trial_info(_q(query, "trialName"), _q(query, "namespace")))
        if path.rstrip("/") == "/katib/fetch_nas_job_info":
            return _json(self._nas_job_info(_q(query, "experimentName"), _q(query, "namespace")))
        mm = _CM.match(path)
        if mm:
            ns = mm.group(1)
            if method == "POST":
                cm = _load_body(body)
                md = cm.get("metadata") or {}
                m.add_configmap(md.get("namespace") or ns, md["name"], cm.get("data") or {}, md.get("labels"))
                return _json(cm, 201)
            return _json({"items": [{"metadata": {"namespace": n_, "name": name_}, "data": data}
                                    for n_, name_, data in m.configmaps.list() if n_ == ns]})
        mm = _API.match(path)
        if not mm:
            raise _Err(404, "NotFound", "the server could not find the requested resource")
        ns, kind, name = mm.groups()
        if kind == "experiments":
            if method == "GET" and name:
                return _json(self._get(m.get_experiment, name, ns, "experiments").to_k8s())
            if method == "GET":
                return _json({"items": [e.to_k8s() for e in m.list_experiments(ns)]})
            if method == "POST":
                exp = V1beta1Experiment.from_k8s(_load_body(body))
                try:
                    out = m.create_experiment(exp, ns)
                except ValidationError as e:
                    raise _Err(400, "Invalid", str(e))
                except ValueError as e:
                    if "already exists" in str(e):
                        raise _Err(409, "AlreadyExists", str(e))
                    raise _Err(400, "BadRequest", str(e))
                return _json(out.to_k8s(), 201)
            if method == "PUT" and name:
                exp = V1beta1Experiment.from_k8s(_load_body(body))
                exp.metadata.namespace = exp.metadata.namespace or ns
                try:
                    return _json(m.update_experiment(exp).to_k8s())
                except ValidationError as e:
                    raise _Err(400, "Invalid", str(e))
                except KeyError:
                    raise _Err(404, "NotFound", 'experiments.kubeflow.org "%s" not found' % name)
            if method == "DELETE" and name:
                self._get(m.get_experiment, name, ns, "experiments")
                m.delete_experiment(name, ns)
                return _json({"kind": "Status", "status": "Success"})
        if kind == "trials":
            if name:
                return _json(self._get(m.get_trial, name, ns, "trials").to_k8s())
            exp = None
            sel = _q(query, "labelSelector", "")
            if sel.startswith(C.LABEL_EXPERIMENT_NAME + "="):
                exp = sel.split("=", 1)[1]
            return _json({"items": [t.to_k8s() for t in m.list_trials(exp, ns)]})
        if kind == "suggestions":
            if name:
                return _json(self._get(m.get_suggestion, name, ns, "suggestions").to_k8s())
            return _json({"items": [s.to_k8s() for s in m.list_suggestions(ns)]})
        raise _Err(405, "MethodNotAllowed", "%s not allowed on %s" % (method, path))

    # ------------------------------------------------------------------ UI backend
    def _ui(self, method, path, query, body):
        """The UI backend routes of ``cmd/ui/v1beta1/main.go:48-70`` (handlers in
        ``pkg/ui/v1beta1/backend.go``) on the in-process store, plus the single-page UI
        (``ui/index.html``) at ``/`` and ``/katib/``. Returns None for other paths."""
        m = self.m
        if path in ("", "/katib") and method == "GET":
            with open(os.path.join(os.path.dirname(__file__), "ui", "index.html"), "rb") as f:
                return 200, "text/html; charset=utf-8", f.read()
        if path == "/katib/fetch_experiments":  # backend.go:138-179, util.go:36-66 (ExperimentView)
            ns = query.get("namespace") or [None]
            out = []
            for n in ns:
                for e in m.list_experiments(n):
                    conds = (e.status.conditions if e.status else None) or []
                    view = {"name": e.metadata.name, "namespace": e.metadata.namespace,
                            "type": "nas" if e.spec.nas_config is not None else "hp",
                            "status": conds[-1].type if conds else ""}
                    view.update(e.to_k8s().get("status") or {})
                    out.append(view)
            return _json(out)
        if path == "/katib/fetch_algorithms":  # the UI's algorithm / early-stopping pickers
            return _json({"algorithms": sorted(m.config.suggestions), "earlyStopping": sorted(m.config.early_stoppings)})
        if path == "/katib/edit_experiment_budget" and method == "POST":  # SDK edit_experiment_budget
            data = _load_body(body) or {}
            exp = self._get(m.get_experiment, data.get("experimentName"), data.get("namespace"), "experiments")
            for key, attr in (("maxTrialCount", "max_trial_count"), ("parallelTrialCount", "parallel_trial_count"),
                              ("maxFailedTrialCount", "max_failed_trial_count")):
                if data.get(key) is not None:
                    setattr(exp.spec, attr, int(data[key]))
            try:
                return _json(m.update_experiment(exp).to_k8s())
            except ValidationError as e:
                raise _Err(400, "Invalid", str(e))
        if path == "/katib/create_experiment" and method == "POST":  # backend.go:86-136
            data = _load_body(body)
            doc = data.get("postData") if isinstance(data, dict) and "postData" in data else None
            if isinstance(doc, str):  # the UI's editor sends YAML (or JSON) text
                try:
                    doc = yaml.safe_load(doc)
                except yaml.YAMLError as e:
                    raise _Err(400, "BadRequest", "postData is not valid YAML/JSON: %s" % e)
            if doc is None:
                raise _Err(500, "InternalError", "Couldn't load the 'postData' field of the request's data")
            try:
                out = m.create_experiment(V1beta1Experiment.from_k8s(doc))
            except (ValidationError, ValueError) as e:
                raise _Err(500, "InternalError", str(e))
            return _json(out.to_k8s())
        if path == "/katib/delete_experiment":  # backend.go:181-263
            name, ns = _q(query, "experimentName"), _q(query, "namespace")
            self._get(m.get_experiment, name, ns, "experiments")
            m.delete_experiment(name, ns)
            return self._ui(method, "/katib/fetch_experiments", {"namespace": [ns]}, b"")
        if path == "/katib/fetch_experiment":  # backend.go:463-512
            return _json(self._get(m.get_experiment, _q(query, "experimentName"), _q(query, "namespace"),
                                   "experiments").to_k8s())
        if path == "/katib/fetch_suggestion":  # backend.go:514-564
            return _json(self._get(m.get_suggestion, _q(query, "suggestionName"), _q(query, "namespace"),
                                   "suggestions").to_k8s())
        if path == "/katib/fetch_trial":  # backend.go:566-615
            return _json(self._get(m.get_trial, _q(query, "trialName"), _q(query, "namespace"),
                                   "trials").to_k8s())
        if path == "/katib/fetch_trial_logs":  # backend.go:617-700: the primary container's log
            name, ns = _q(query, "trialName"), _q(query, "namespace")
            self._get(m.get_trial, name, ns, "trials")
            log = os.path.join(m.state_dir, "trials", ns, name, "metrics.log")
            text = ""
            if os.path.exists(log):
                with open(log, errors="replace") as f:
                    text = f.read()
            return _json(text)
        if path == "/katib/fetch_namespaces":  # backend.go:439-461
            nss = {e.metadata.namespace for e in m.list_experiments(None)} | {n for n, _, _ in m.configmaps.list()}
            return _json(sorted(nss | {"default"}))
        if path == "/katib/fetch_trial_templates":  # backend.go:265-289, util.go:80-130
            return _json({"Data": self._templates_view()})
        if path in ("/katib/add_template", "/katib/edit_template", "/katib/delete_template") and method == "POST":
            return _json({"Data": self._update_template(path.rsplit("/", 1)[1].split("_")[0], _load_body(body))})
        return None

    def _templates_view(self):
        by_ns = {}
        for ns, name, data in self.m.configmaps.trial_templates():
            by_ns.setdefault(ns, []).append({"ConfigMapName": name, "Templates": [
                {"Path": k, "Yaml": v} for k, v in sorted(data.items())]})
        return [{"ConfigMapNamespace": ns, "ConfigMaps": cms} for ns, cms in sorted(by_ns.items())]

    def _update_template(self, action, data):
        """``updateTrialTemplates`` (util.go:180-240): add / edit (rename path) / delete one
        template entry; a ConfigMap left empty is deleted."""
        ns, name = data["updatedConfigMapNamespace"], data["updatedConfigMapName"]
        path = data["updatedConfigMapPath"]
        store = self.m.configmaps
        try:
            templates = dict(store.get(ns, name))
        except KeyError:
            if action != "add":
                raise _Err(500, "InternalError", 'configmaps "%s" not found' % name)
            templates = {}
        if action == "add":
            templates[path] = data["updatedTemplateYaml"]
        elif action == "edit":
            templates.pop(data["configMapPath"], None)
            templates[path] = data["updatedTemplateYaml"]
        else:
            templates.pop(path, None)
        if templates:
            self.m.add_configmap(ns, name, templates, {C.LABEL_TRIAL_TEMPLATE_CONFIGMAP_NAME:
                                                       C.LABEL_TRIAL_TEMPLATE_CONFIGMAP_VALUE})
        else:
            store.delete(ns, name)
        return self._templates_view()

    @staticmethod
    def _get(fn, name, ns, plural):
        try:
            return fn(name, ns)
        except KeyError:
            raise _Err(404, "NotFound", '%s.kubeflow.org "%s" not found' % (plural, name))

    def _hp_job_info(self, name, ns):
        e = self._get(self.m.get_experiment, name, ns, "experiments")
        metrics = [e.spec.objective.objective_metric_name] + list(e.spec.objective.additional_metric_names or [])
        params = [p.name for p in e.spec.parameters or []]
        lines = [",".join(["Status", "trialName"] + metrics + params)]
        for t in self.m.list_trials(name, ns):
            last = t.status.conditions[-1].type if t.status and t.status.conditions else ""
            row = {}
            if any(c.type in ("Succeeded", "EarlyStopped") and c.status == "True" for c in t.status.conditions or []):
                row = _best_values(t, self.m.get_observation_log(t.metadata.name))
            for pa in t.spec.parameter_assignments or []:
                row.setdefault(pa.name, pa.value)
            lines.append(",".join([last, t.metadata.name] + [row.get(k, "") for k in metrics + params]))
        return "\n".join(lines)

    def _hp_trial_info(self, name, ns):
        self._get(self.m.get_trial, name, ns, "trials")
        lines = ["metricName,time,value"]
        for ts, n, v in self.m.get_observation_log(name):
            lines.append("%s,%s,%s" % (n, ts[:19], v))
        return "\n".join(lines)

    def _nas_job_info(self, name, ns):
        self._get(self.m.get_experiment, name, ns, "experiments")
        out = []
        for t in self.m.list_trials(name, ns):
            arch = {pa.name: pa.value for pa in t.spec.parameter_assignments or []}
            metrics = {}
            if t.status.observation is not None:
                metrics = {mt.name: mt.latest for mt in t.status.observation.metrics or []}
            out.append({"trialName": t.metadata.name, "assignments": arch, "metrics": metrics,
                        "status": t.status.conditions[-1].type if t.status.conditions else ""})
        return out

    def _make_handler(self):
        server = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, fmt, *args):  # quiet
                pass

            def _authorized(self, path, query) -> bool:
                """Bearer header (SDK / CLI), or the UI's session cookie. A browser cannot send
                the header, so opening ``/?token=<token>`` once sets an HttpOnly SameSite=Strict
                cookie holding it (``self._set_cookie``) and later UI requests carry that."""
                self._set_cookie = None
                if server.token is None or path in ("/healthz", "/readyz"):
                    return True
                import hmac

                want = server.token.encode()
                got = self.headers.get("Authorization") or ""
                if hmac.compare_digest(got.encode(), b"Bearer " + want):
                    return True
                for part in (self.headers.get("Cookie") or "").split(";"):
                    k, _, v = part.strip().partition("=")
                    if k == COOKIE and hmac.compare_digest(v.encode(), want):
                        return True
                # ?token= only on the UI entry path, answered with a redirect that sets the cookie and
                # strips the query (_do): the token never sits in a page URL the UI then works under
                q = (query.get("token") or [""])[0]
                if q and path == "/" and hmac.compare_digest(q.encode(), want):
                    self._set_cookie = "%s=%s; HttpOnly; SameSite=Strict; Path=/" % (COOKIE, server.token)
                    return True
                return False

            def _do(self, method):
                u = urlparse(self.path)
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n) if n else b""
                query = parse_qs(u.query)
                try:
                    if not self._authorized(u.path, query):
                        raise _Err(401, "Unauthorized", "missing or wrong bearer token")
                    if "token" in query:
                        if self._set_cookie is None:
                            raise _Err(400, "BadRequest", "the token query parameter is only accepted on /")
                        self.send_response(303)
                        self.send_header("Location", "/")
                        self.send_header("Set-Cookie", self._set_cookie)
                        self.send_header("Referrer-Policy", "no-referrer")
                        self.send_header("Content-Length", "0")
                        self.end_headers()
                        return
                    code, ctype, data = server.handle(method, u.path, query, body)
                except _Err as e:
                    code, ctype = e.code, "application/json"
                    data = json.dumps({"kind": "Status", "code": e.code, "reason": e.reason,
                                       "message": e.message}).encode()
                except Exception as e:  # noqa: BLE001 - reported to the client
                    code, ctype = 500, "application/json"
                    data = json.dumps({"kind": "Status", "code": 500, "reason": "InternalError",
                                       "message": str(e)}).encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.send_header("Referrer-Policy", "no-referrer")
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                self._do("GET")

            def do_POST(self):
                self._do("POST")

            def do_PUT(self):
                self._do("PUT")

            def do_DELETE(self):
                self._do("DELETE")

        return Handler


def _q(query, key, default=None):
    v = query.get(key)
    if not v:
        if default is None:
            raise _Err(400, "BadRequest", "no '%s' provided" % key)
        return default
    return v[0]


def _json(obj, code=200):
    return code, "application/json", json.dumps(obj).encode()


def _load_body(body: bytes):
    text = body.decode()
    try:
        return json.loads(text)
    except json.JSONDecodeError:
        return yaml.safe_load(text)
