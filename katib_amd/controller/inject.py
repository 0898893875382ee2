"""Metrics-collector injection for trials that run as Kubernetes pods
(reference ``pkg/webhook/v1beta1/pod/inject_webhook.go:123-331`` and ``utils.go:38-290``).

The node-local scheduler never needs this: its supervisor redirects the trial's
output and runs the native collector itself. When trials are instead submitted to a
cluster (a Job rendered by :class:`~katib_amd.controller.manifest.Generator`), this
module rewrites the pod the way the reference's ``/mutate-pod`` webhook does, with
``katib_amd.metricscollector.file_collector`` (same flags) as the sidecar:

* the primary container's command is wrapped in ``sh -c "<cmd> 1>file 2>&1 && echo
  completed > $$$$.pid"`` (plus the early-stopped branch when the trial has rules);
* a shared ``metrics-volume`` emptyDir is mounted on the primary and sidecar
  containers at the metrics directory;
* the sidecar gets ``-t -m -o-type -s-db -path -f -format -w -stop-rule -s-earlystop``.

Pods and trials are handled in manifest (dict) form. A container without an explicit
``command`` is rejected: resolving the image entrypoint needs a registry, which this
framework never contacts.
"""

from __future__ import annotations

import copy
import os
from typing import Dict, List, Optional, Tuple

from ..api import constants as C

METRICS_VOLUME = "metrics-volume"
METRIC_LOGGER_COLLECTOR_CONTAINER_NAME = "metrics-logger-and-collector"
METRIC_COLLECTOR_CONTAINER_NAME = "metrics-collector"
NEED_WRAP_WORKER_COLLECTORS = (C.COLLECTOR_STDOUT, C.COLLECTOR_FILE)
FILE_KIND, DIRECTORY_KIND, INVALID_KIND = C.FS_KIND_FILE, C.FS_KIND_DIRECTORY, "Invalid"


class InjectError(ValueError):
    pass


def db_manager_addr() -> str:
    """GetDBManagerAddr (pkg/apis/manager/v1beta1/util.go)."""
    ns = os.environ.get("KATIB_DB_MANAGER_SERVICE_NAMESPACE", "kubeflow")
    ip = os.environ.get("KATIB_DB_MANAGER_SERVICE_IP", "katib-db-manager")
    port = os.environ.get("KATIB_DB_MANAGER_SERVICE_PORT", str(C.DEFAULT_DB_MANAGER_PORT))
    return "%s.%s:%s" % (ip, ns, port) if ns else "%s:%s" % (ip, port)


def early_stopping_endpoint(suggestion_name: str, algorithm: str, namespace: str) -> str:
    return "%s-%s.%s:%d" % (suggestion_name, algorithm, namespace, C.DEFAULT_EARLY_STOPPING_PORT)


def is_primary_pod(pod_labels: Optional[Dict[str, str]], primary_labels: Dict[str, str]) -> bool:
    pod_labels = pod_labels or {}
    return all(k in pod_labels and pod_labels[k] == v for k, v in primary_labels.items())


def primary_container_index(containers: List[Dict], name: str) -> int:
    for i, c in enumerate(containers or []):
        if c.get("name") == name:
            return i
    return -1


def container_command(container: Dict) -> List[str]:
    args = list(container.get("command") or [])
    if not args:
        raise InjectError("container %s has no command; the image entrypoint cannot be resolved without a "
                          "registry, set spec.containers[].command" % container.get("name"))
    return args + list(container.get("args") or [])


def mount_path(mc: Dict) -> Tuple[str, str]:
    """getMountPath (utils.go:125-140)."""
    kind = ((mc or {}).get("collector") or {}).get("kind")
    fsp = (((mc or {}).get("source") or {}).get("fileSystemPath")) or {}
    if kind == C.COLLECTOR_STDOUT:
        return C.DEFAULT_FILE_PATH, FILE_KIND
    if kind == C.COLLECTOR_FILE:
        return fsp.get("path", ""), FILE_KIND
    if kind == C.COLLECTOR_TFEVENT:
        return fsp.get("path", ""), DIRECTORY_KIND
    if kind == C.COLLECTOR_CUSTOM and fsp:
        return fsp.get("path", ""), fsp.get("kind", "")
    return "", INVALID_KIND


def need_wrap_worker_container(mc: Dict) -> bool:
    return ((mc or {}).get("collector") or {}).get("kind") in NEED_WRAP_WORKER_COLLECTORS


def early_stopping_command(metrics_dir: str) -> str:
    # $$$$ becomes the shell's pid after Kubernetes' $$ -> $ expansion; inside $( ) one $$ is enough
    pid_file = os.path.join(metrics_dir, "$$$$.pid")
    pid_cond = os.path.join(metrics_dir, "$$.pid")
    return ("if test -f %s && [ $(head -n 1 %s) = %s ]; then echo Training Container was Early Stopped; "
            "else echo Training Container was Failed; exit 1; fi" % (pid_file, pid_cond, C.TRAINING_EARLY_STOPPED))


def mark_completed_command(metrics_dir: str) -> str:
    return "echo %s > %s" % (C.TRAINING_COMPLETED, os.path.join(metrics_dir, "$$$$.pid"))


def wrap_worker_container(trial: Dict, pod: Dict, metrics_file: str, path_kind: str) -> None:
    """wrapWorkerContainer (utils.go:152-197); mutates ``pod`` in place."""
    spec = trial.get("spec") or {}
    containers = (pod.get("spec") or {}).get("containers") or []
    idx = primary_container_index(containers, spec.get("primaryContainerName"))
    if idx < 0:
        raise InjectError("Unable to find primary container %s in mutated pod containers %s"
                          % (spec.get("primaryContainerName"), [c.get("name") for c in containers]))
    command = ["sh", "-c"]
    args = container_command(containers[idx])
    if args[0] in ("sh", "bash") and len(args) > 1 and args[1] == "-c":
        command, args = args[:2], args[2:]
    mc = spec.get("metricsCollector") or {}
    if (mc.get("collector") or {}).get("kind") == C.COLLECTOR_STDOUT:
        args.append("1>%s 2>&1" % metrics_file)
    metrics_dir = os.path.dirname(metrics_file) if path_kind == FILE_KIND else metrics_file
    if spec.get("earlyStoppingRules"):
        args += ["||", early_stopping_command(metrics_dir)]
    args += ["&&", mark_completed_command(metrics_dir)]
    c = containers[idx]
    c["command"] = command
    c["args"] = [" ".join(args)]


def mutate_metrics_collector_volume(pod: Dict, path: str, sidecar: str, primary: str, path_kind: str) -> None:
    vol = {"name": METRICS_VOLUME, "emptyDir": {}}
    d = os.path.dirname(path) if path_kind == FILE_KIND else path
    for c in pod["spec"]["containers"]:
        if c.get("name") in (sidecar, primary):
            c.setdefault("volumeMounts", []).append({"name": METRICS_VOLUME, "mountPath": d})
    pod["spec"].setdefault("volumes", []).append(vol)


def mutate_pod_metadata(pod: Dict, trial: Dict) -> None:
    md = pod.setdefault("metadata", {})
    labels = dict(md.get("labels") or {})
    labels.update((trial.get("metadata") or {}).get("labels") or {})
    labels[C.LABEL_TRIAL_NAME] = (trial.get("metadata") or {}).get("name")
    md["labels"] = labels


def sidecar_container_name(kind: str) -> str:
    if kind in (C.COLLECTOR_STDOUT, C.COLLECTOR_FILE):
        return METRIC_LOGGER_COLLECTOR_CONTAINER_NAME
    return METRIC_COLLECTOR_CONTAINER_NAME


def metrics_collector_args(trial: Dict, metric_names: str, mc: Dict, collector_config: Dict,
                           es_rules: List[str], suggestions: Optional[Dict[Tuple[str, str], str]] = None,
                           db_addr: Optional[str] = None) -> List[str]:
    """getMetricsCollectorArgs (inject_webhook.go:294-331). ``suggestions`` maps
    (namespace, suggestion name) -> algorithm name (the early-stopping endpoint's
    service name); a missing entry is an error, as a missing Suggestion is there."""
    md = trial.get("metadata") or {}
    spec = trial.get("spec") or {}
    args = ["-t", md.get("name"), "-m", metric_names, "-o-type", (spec.get("objective") or {}).get("type"),
            "-s-db", db_addr or db_manager_addr()]
    path, _ = mount_path(mc)
    if path:
        args += ["-path", path]
    src = mc.get("source") or {}
    fmts = (src.get("filter") or {}).get("metricsFormat") or []
    if fmts:
        args += ["-f", ";".join(fmts)]
    kind = (mc.get("collector") or {}).get("kind")
    if kind == C.COLLECTOR_FILE and src.get("fileSystemPath") is not None:
        args += ["-format", src["fileSystemPath"].get("format", "")]
    if kind == C.COLLECTOR_STDOUT:
        args += ["-format", C.FORMAT_TEXT]
    if collector_config.get("waitAllProcesses") is not None:
        args += ["-w", "true" if collector_config["waitAllProcesses"] else "false"]
    if es_rules:
        for r in es_rules:
            args += ["-stop-rule", r]
        name = (md.get("labels") or {}).get(C.LABEL_EXPERIMENT_NAME)
        ns = md.get("namespace")
        algo = (suggestions or {}).get((ns, name))
        if algo is None:
            raise InjectError('suggestions.kubeflow.org "%s" not found' % name)
        args += ["-s-earlystop", early_stopping_endpoint(name, algo, ns)]
    return args


def early_stopping_rule_flags(trial: Dict) -> List[str]:
    """Rules as ``name;value;comparison;startStep`` (inject_webhook.go:202-208)."""
    return ["%s;%s;%s;%d" % (r.get("name"), r.get("value"), r.get("comparison"), int(r.get("startStep") or 0))
            for r in (trial.get("spec") or {}).get("earlyStoppingRules") or []]


def mutate_pod(pod: Dict, trial: Dict, collector_config: Dict, collector_image: str = "",
               suggestions: Optional[Dict[Tuple[str, str], str]] = None, db_addr: Optional[str] = None) -> Dict:
    """Mutate (inject_webhook.go:123-189) for a pod owned by ``trial``; returns a new pod."""
    out = copy.deepcopy(pod)
    mutate_pod_metadata(out, trial)
    spec = trial.get("spec") or {}
    primary_labels = spec.get("primaryPodLabels")
    if primary_labels and not is_primary_pod((pod.get("metadata") or {}).get("labels"), primary_labels):
        return out
    mc = spec.get("metricsCollector") or {}
    kind = (mc.get("collector") or {}).get("kind")
    if kind == C.COLLECTOR_NONE:
        return out
    if kind == C.COLLECTOR_CUSTOM:
        sidecar = copy.deepcopy(mc["collector"]["customCollector"])
    else:
        obj = spec.get("objective") or {}
        names = ";".join([obj.get("objectiveMetricName", "")] + list(obj.get("additionalMetricNames") or []))
        args = metrics_collector_args(trial, names, mc, collector_config, early_stopping_rule_flags(trial),
                                      suggestions, db_addr)
        sidecar = {"name": sidecar_container_name(kind),
                   "image": collector_image or collector_config.get("image", ""), "args": args}
        if collector_config.get("imagePullPolicy"):
            sidecar["imagePullPolicy"] = collector_config["imagePullPolicy"]
        if collector_config.get("resources"):
            sidecar["resources"] = copy.deepcopy(collector_config["resources"])
    out.setdefault("spec", {}).setdefault("containers", []).append(sidecar)
    out["spec"]["shareProcessNamespace"] = True
    path, path_kind = mount_path(mc)
    if path:
        mutate_metrics_collector_volume(out, path, sidecar.get("name"), spec.get("primaryContainerName"), path_kind)
    if need_wrap_worker_container(mc):
        wrap_worker_container(trial, out, path, path_kind)
    return out
