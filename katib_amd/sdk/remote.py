"""HTTP client with the :class:`~katib_amd.controller.manager.Manager` method surface,
talking to a scheduler daemon's :mod:`~katib_amd.controller.apiserver` (``katib-amd
serve``). ``KatibClient(host="http://127.0.0.1:8080")`` uses it, so the SDK works the
same against an in-process scheduler and a long-running node daemon (the reference
SDK talks to the Kubernetes API server the same way)."""

from __future__ import annotations

import json
import os
import urllib.error
import urllib.parse
import urllib.request
from typing import List, Optional

from ..api.models import V1beta1Experiment, V1beta1Suggestion, V1beta1Trial
from ..api.validation import ValidationError

_BASE = "/apis/kubeflow.org/v1beta1/namespaces/%s/%s"


class RemoteManager:
    def __init__(self, host: str, namespace: str = "default", timeout: float = 60.0, token: Optional[str] = None):
        self.host = host.rstrip("/")
        if "://" not in self.host:
            self.host = "http://" + self.host
        self.namespace = namespace
        self.timeout = timeout
        # bearer token of a daemon listening off loopback (katib-amd serve --token-file)
        self.token = token or os.environ.get("KATIB_AMD_API_TOKEN") or None

    def _headers(self, data) -> dict:
        h = {"Content-Type": "application/json"} if data else {}
        if self.token:
            h["Authorization"] = "Bearer " + self.token
        return h

    def _req(self, method: str, path: str, body=None, query=None):
        url = self.host + path
        if query:
            url += "?" + urllib.parse.urlencode(query)
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(url, data=data, method=method, headers=self._headers(data))
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return json.loads(r.read().decode() or "null")
        except urllib.error.HTTPError as e:
            try:
                st = json.loads(e.read().decode())
                msg = st.get("message", str(e))
            except Exception:
                msg = str(e)
            if e.code == 404:
                raise KeyError(msg)
            if e.code == 400 and st.get("reason") == "Invalid":
                raise ValidationError(msg)
            if e.code in (400, 409):
                raise ValueError(msg)
            raise RuntimeError(msg)

    def _ns(self, ns):
        return ns or self.namespace

    # experiments
    def create_experiment(self, exp: V1beta1Experiment, namespace: Optional[str] = None) -> V1beta1Experiment:
        ns = self._ns(namespace or (exp.metadata.namespace if exp.metadata else None))
        return V1beta1Experiment.from_k8s(self._req("POST", _BASE % (ns, "experiments"), exp.to_k8s()))

    def update_experiment(self, exp: V1beta1Experiment) -> V1beta1Experiment:
        ns = self._ns(exp.metadata.namespace)
        return V1beta1Experiment.from_k8s(
            self._req("PUT", _BASE % (ns, "experiments") + "/" + exp.metadata.name, exp.to_k8s()))

    def get_experiment(self, name: str, namespace: Optional[str] = None) -> V1beta1Experiment:
        return V1beta1Experiment.from_k8s(self._req("GET", _BASE % (self._ns(namespace), "experiments") + "/" + name))

    def list_experiments(self, namespace: Optional[str] = None) -> List[V1beta1Experiment]:
        out = self._req("GET", _BASE % (self._ns(namespace), "experiments"))
        return [V1beta1Experiment.from_k8s(i) for i in out["items"]]

    def delete_experiment(self, name: str, namespace: Optional[str] = None):
        self._req("DELETE", _BASE % (self._ns(namespace), "experiments") + "/" + name)

    # trials / suggestions
    def get_trial(self, name: str, namespace: Optional[str] = None) -> V1beta1Trial:
        return V1beta1Trial.from_k8s(self._req("GET", _BASE % (self._ns(namespace), "trials") + "/" + name))

    def list_trials(self, experiment_name: Optional[str] = None, namespace: Optional[str] = None):
        q = {"labelSelector": "katib.kubeflow.org/experiment=%s" % experiment_name} if experiment_name else None
        out = self._req("GET", _BASE % (self._ns(namespace), "trials"), query=q)
        return [V1beta1Trial.from_k8s(i) for i in out["items"]]

    def get_suggestion(self, name: str, namespace: Optional[str] = None) -> V1beta1Suggestion:
        return V1beta1Suggestion.from_k8s(self._req("GET", _BASE % (self._ns(namespace), "suggestions") + "/" + name))

    def list_suggestions(self, namespace: Optional[str] = None):
        out = self._req("GET", _BASE % (self._ns(namespace), "suggestions"))
        return [V1beta1Suggestion.from_k8s(i) for i in out["items"]]

    # observations / templates
    def get_observation_log(self, trial_name: str, metric_name: str = "", start_time: str = "", end_time: str = ""):
        out = self._req("GET", "/katib/observation_logs", query={
            "trialName": trial_name, "metricName": metric_name, "startTime": start_time, "endTime": end_time})
        return [(m["timeStamp"], m["metric"]["name"], m["metric"]["value"]) for m in out["metricLogs"]]

    def add_configmap(self, namespace: str, name: str, data, labels=None):
        self._req("POST", "/api/v1/namespaces/%s/configmaps" % namespace,
                  {"metadata": {"name": name, "namespace": namespace, "labels": labels or {}}, "data": data})

    def metrics_text(self) -> str:
        req = urllib.request.Request(self.host + "/metrics", headers=self._headers(None))
        with urllib.request.urlopen(req, timeout=self.timeout) as r:
            return r.read().decode()
