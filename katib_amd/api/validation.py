"""Experiment validation: the ``/validate-experiment`` webhook
(reference ``pkg/webhook/v1beta1/experiment/validator/validator.go:67-524``).

Error strings are the reference's so existing tooling that matches on them keeps
working. Kubernetes-only checks (namespace injection label, leftover PV of a
FromVolume experiment) do not apply to a node-local scheduler and are skipped.
"""

from __future__ import annotations

import json
import os
import re
from typing import Optional

from . import constants as C
from .conditions import ExperimentConditions as EC
from .models import V1beta1Experiment

_NAME_RE = re.compile(r"^[a-z]([-a-z0-9]*[a-z0-9])?")
_META_RE = re.compile(C.TRIAL_TEMPLATE_META_REPLACE_REGEX)
_META_PARSE_RE = re.compile(C.TRIAL_TEMPLATE_META_PARSE_REGEX)
_PARAM_RE = re.compile(C.TRIAL_TEMPLATE_PARAM_REPLACE_REGEX)
_TWO_GROUPS = re.compile(r".*\(.*\).*\(.*\).*")


class ValidationError(ValueError):
    pass


def is_meta_key(ref: str) -> bool:
    m = _META_RE.search(ref)
    if not m:
        return False
    key = m.group(1)
    if key in C.TRIAL_TEMPLATE_META_KEYS:
        return True
    sub = _META_PARSE_RE.search(key)
    return bool(sub) and sub.group(1) in C.TRIAL_TEMPLATE_META_KEYS


def _spec_equal(a, b) -> bool:
    return a.to_k8s() == b.to_k8s()


def is_restartable(e) -> bool:
    """IsCompletedExperimentRestartable (status_util.go:240-246)."""
    return (EC.is_succeeded(e) and EC.is_completed_reason(e, C.EXPERIMENT_MAX_TRIALS_REACHED_REASON)
            and e.spec.resume_policy in (C.RESUME_LONG_RUNNING, C.RESUME_FROM_VOLUME))


def validate_experiment(inst: V1beta1Experiment, old: Optional[V1beta1Experiment] = None, *,
                        suggestion_algorithms=None, early_stopping_algorithms=None, template_getter=None,
                        metrics_collectors=None):
    name = inst.metadata.name if inst.metadata else ""
    if not name or not _NAME_RE.match(name):
        raise ValidationError(
            "name must consist of lower case alphanumeric characters or '-', start with an alphabetic character, "
            "and end with an alphanumeric character (e.g. 'my-name', or 'abc-123', regex used for validation is "
            "'^[a-z]([-a-z0-9]*[a-z0-9])?)'")
    s = inst.spec
    if s.max_failed_trial_count is not None and s.max_failed_trial_count < 0:
        raise ValidationError("spec.maxFailedTrialCount should not be less than 0")
    if s.max_trial_count is not None and s.max_trial_count <= 0:
        raise ValidationError("spec.maxTrialCount must be greater than 0")
    if s.parallel_trial_count is not None and s.parallel_trial_count <= 0:
        raise ValidationError("spec.parallelTrialCount must be greater than 0")
    if s.max_failed_trial_count is not None and s.max_trial_count is not None:
        if s.max_failed_trial_count > s.max_trial_count:
            raise ValidationError("spec.maxFailedTrialCount should be less than or equal to spec.maxTrialCount")
    if s.parallel_trial_count is not None and s.max_trial_count is not None:
        if s.parallel_trial_count > s.max_trial_count:
            raise ValidationError("spec.paralelTrialCount should be less than or equal to spec.maxTrialCount")

    if old is not None:
        restarting = not _spec_equal(inst.spec, old.spec)
        if restarting and EC.is_completed(old) and not is_restartable(old):
            raise ValidationError(
                "Experiment can be restarted if it is in succeeded state by reaching max trials and "
                "spec.resumePolicy = LongRunning or spec.resumePolicy = FromVolume, when experiment is completed")
        trials = old.status.trials if old.status and old.status.trials else 0
        if restarting and s.max_trial_count is not None and s.max_trial_count <= trials:
            raise ValidationError("spec.maxTrialCount: %d must be greater than status.trials count: %d"
                                  % (s.max_trial_count, trials))
        cmp_old = old.spec.deepcopy()
        cmp_old.max_failed_trial_count = s.max_failed_trial_count
        cmp_old.max_trial_count = s.max_trial_count
        cmp_old.parallel_trial_count = s.parallel_trial_count
        if not _spec_equal(inst.spec, cmp_old):
            raise ValidationError(
                "only spec.parallelTrialCount, spec.maxTrialCount and spec.maxFailedTrialCount are editable")

    _validate_objective(s.objective)
    _validate_algorithm(s.algorithm, suggestion_algorithms)
    _validate_early_stopping(s.early_stopping, early_stopping_algorithms)
    if s.resume_policy not in ("", None) + C.RESUME_POLICIES:
        raise ValidationError("invalid ResumePolicyType %s" % s.resume_policy)
    _validate_trial_template(inst, template_getter)
    if not s.parameters and s.nas_config is None:
        raise ValidationError("spec.parameters or spec.nasConfig must be specified")
    if s.parameters and s.nas_config is not None:
        raise ValidationError("only one of spec.parameters and spec.nasConfig can be specified")
    if s.parameters:
        _validate_parameters(s.parameters)
    _validate_metrics_collector(inst, metrics_collectors)


def _validate_objective(obj):
    if obj is None:
        raise ValidationError("no spec.objective specified")
    if obj.type not in (C.OBJECTIVE_MINIMIZE, C.OBJECTIVE_MAXIMIZE):
        raise ValidationError("spec.objective.type must be %s or %s" % (C.OBJECTIVE_MINIMIZE, C.OBJECTIVE_MAXIMIZE))
    if not obj.objective_metric_name:
        raise ValidationError("no spec.objective.objectiveMetricName specified")
    if obj.objective_metric_name in (obj.additional_metric_names or []):
        raise ValidationError("spec.objective.additionalMetricNames should not contain "
                              "spec.objective.objectiveMetricName")


def _validate_algorithm(ag, known):
    if ag is None:
        raise ValidationError("no spec.algorithm specified")
    if not ag.algorithm_name:
        raise ValidationError("no spec.algorithm.name specified")
    if known is not None and ag.algorithm_name not in known:
        raise ValidationError("unable to get Suggestion config data for algorithm %s: "
                              "failed to find algorithm '%s' config in katib-config" % (ag.algorithm_name,
                                                                                         ag.algorithm_name))


def _validate_early_stopping(es, known):
    if es is None:
        return
    if not es.algorithm_name:
        raise ValidationError("no spec.earlyStopping.algorithmName specified")
    if known is not None and es.algorithm_name not in known:
        raise ValidationError("unable to get EarlyStopping config data for algorithm %s: "
                              "failed to find early stopping algorithm '%s' config in katib-config"
                              % (es.algorithm_name, es.algorithm_name))


def _validate_parameters(params):
    for i, p in enumerate(params):
        pt = p.parameter_type or ""
        if pt not in C.PARAMETER_TYPES + ("unknown", ""):
            raise ValidationError("parameterType: %s is not supported in spec.parameters[%d]: %s" % (pt, i, p.to_k8s()))
        fs = p.feasible_space
        if fs is None or not fs.to_k8s():
            raise ValidationError("feasibleSpace must be specified in spec.parameters[%d]: %s" % (i, p.to_k8s()))
        if pt in (C.PARAMETER_DOUBLE, C.PARAMETER_INT):
            if fs.list:
                raise ValidationError("feasibleSpace.list is not supported for parameterType: %s in "
                                      "spec.parameters[%d]: %s" % (pt, i, p.to_k8s()))
            if not fs.max and not fs.min:
                raise ValidationError("feasibleSpace.max or feasibleSpace.min must be specified for parameterType: "
                                      "%s in spec.parameters[%d]: %s" % (pt, i, p.to_k8s()))
        elif pt in (C.PARAMETER_CATEGORICAL, C.PARAMETER_DISCRETE):
            if fs.max or fs.min or fs.step:
                raise ValidationError("feasibleSpace .max, .min and .step is not supported for parameterType: %s in "
                                      "spec.parameters[%d]: %s" % (pt, i, p.to_k8s()))


def _validate_trial_template(inst, template_getter):
    t = inst.spec.trial_template
    if t is None:
        raise ValidationError("spec.trialTemplate must be specified")
    if not t.primary_container_name:
        raise ValidationError("spec.trialTemplate.primaryContainerName must be specified")
    if not t.success_condition or not t.failure_condition:
        raise ValidationError("spec.trialTemplate.successCondition and spec.trialTemplate.failureCondition must be "
                              "specified")
    if t.trial_parameters is None:
        raise ValidationError("spec.trialTemplate.trialParameters must be specified")
    if t.trial_spec is None and t.config_map is None:
        raise ValidationError("spec.trialTemplate.trialSpec or spec.trialTemplate.configMap must be specified")
    if t.trial_spec is not None and t.config_map is not None:
        raise ValidationError("only one of spec.trialTemplate.trialSpec or spec.trialTemplate.configMap can be "
                              "specified")
    if t.config_map is not None and (not t.config_map.config_map_name or not t.config_map.config_map_namespace
                                     or not t.config_map.template_path):
        raise ValidationError("for spec.trialTemplate.configMap .configMapName and .configMapNamespace and "
                              ".templatePath must be specified")
    try:
        if template_getter is not None:
            tpl = template_getter(inst)
        else:
            tpl = json.dumps(t.trial_spec)
    except Exception as e:
        raise ValidationError("unable to parse spec.trialTemplate: %s" % e)
    exp_params = {p.name for p in (inst.spec.parameters or [])}
    names, refs = set(), set()
    for p in t.trial_parameters:
        if not p.name or not p.reference or "{" in p.name or "}" in p.name:
            raise ValidationError("invalid spec.trialTemplate.trialParameters: %s" % p.to_k8s())
        if p.name in names:
            raise ValidationError("parameter name %s can't be duplicated in spec.trialTemplate.trialParameters" % p.name)
        if p.reference in refs:
            raise ValidationError("parameter reference %s can't be duplicated in spec.trialTemplate.trialParameters"
                                  % p.reference)
        names.add(p.name)
        refs.add(p.reference)
        if exp_params and not is_meta_key(p.reference) and p.reference not in exp_params:
            raise ValidationError("parameter reference %s does not exist in spec.parameters" % p.reference)
        ph = C.TRIAL_TEMPLATE_PARAM_REPLACE_FORMAT % p.name
        if ph not in tpl:
            raise ValidationError("parameter name: %s in spec.trialParameters not found in spec.trialTemplate: %s"
                                  % (p.name, tpl))
        tpl = tpl.replace(ph, "test-value")
    left = _PARAM_RE.findall(tpl)
    if left:
        raise ValidationError("parameters: %s in spec.trialTemplate not found in spec.trialParameters" % left)
    try:
        run_spec = _parse_spec(tpl)
    except Exception:
        raise ValidationError("unable to convert spec.trialTemplate: %s to unstructured" % tpl)
    md = run_spec.get("metadata") or {}
    if md.get("name") or md.get("namespace"):
        raise ValidationError("metadata.name and metadata.namespace in spec.trialTemplate must be omitted")
    if not run_spec.get("apiVersion") or not run_spec.get("kind"):
        raise ValidationError("APIVersion and Kind in spec.trialTemplate must be specified")
    validate_trial_job(run_spec)


# Field sets of the batch/v1 Job object graph down to the containers. A template field
# outside them would be dropped by the typed conversion, which the reference rejects
# (validator.go:376-421: convert to batchv1.Job, diff, only "remove" ops allowed).
# ``None`` marks a subtree that is not checked further.
_CONTAINER = dict.fromkeys((
    "name", "image", "command", "args", "workingDir", "ports", "envFrom", "env", "resources", "resizePolicy",
    "restartPolicy", "volumeMounts", "volumeDevices", "livenessProbe", "readinessProbe", "startupProbe",
    "lifecycle", "terminationMessagePath", "terminationMessagePolicy", "imagePullPolicy", "securityContext",
    "stdin", "stdinOnce", "tty"))
_CONTAINER.update(command=[None], args=[None])
_POD_SPEC = dict.fromkeys((
    "volumes", "ephemeralContainers", "restartPolicy", "terminationGracePeriodSeconds",
    "activeDeadlineSeconds", "dnsPolicy", "nodeSelector", "serviceAccountName", "serviceAccount",
    "automountServiceAccountToken", "nodeName", "hostNetwork", "hostPID", "hostIPC", "shareProcessNamespace",
    "securityContext", "imagePullSecrets", "hostname", "subdomain", "affinity", "schedulerName", "tolerations",
    "hostAliases", "priorityClassName", "priority", "dnsConfig", "readinessGates", "runtimeClassName",
    "enableServiceLinks", "preemptionPolicy", "overhead", "topologySpreadConstraints", "setHostnameAsFQDN", "os",
    "hostUsers", "schedulingGates", "resourceClaims"))
_POD_SPEC.update(containers=[_CONTAINER], initContainers=[_CONTAINER])
_META = dict.fromkeys((
    "name", "generateName", "namespace", "selfLink", "uid", "resourceVersion", "generation", "creationTimestamp",
    "deletionTimestamp", "deletionGracePeriodSeconds", "labels", "annotations", "ownerReferences", "finalizers",
    "managedFields"))
_JOB_SPEC = dict.fromkeys((
    "parallelism", "completions", "activeDeadlineSeconds", "podFailurePolicy", "successPolicy", "backoffLimit",
    "backoffLimitPerIndex", "maxFailedIndexes", "selector", "manualSelector", "ttlSecondsAfterFinished",
    "completionMode", "suspend", "podReplacementPolicy", "managedBy"))
_JOB_SPEC["template"] = {"metadata": _META, "spec": _POD_SPEC}
_JOB = {"apiVersion": None, "kind": None, "metadata": _META, "spec": _JOB_SPEC, "status": None}


def _schema_diff(obj, schema, path):
    if schema is None or obj is None:
        return None
    if isinstance(schema, list):
        if not isinstance(obj, list):
            return "%s: expected a list, got %s" % (path, type(obj).__name__)
        for i, v in enumerate(obj):
            err = _schema_diff(v, schema[0], "%s/%d" % (path, i))
            if err:
                return err
        return None
    if not isinstance(obj, dict):
        return "%s: expected an object, got %s" % (path, type(obj).__name__)
    for k, v in obj.items():
        if k not in schema:
            return "%s/%s - %s" % (path, k, json.dumps(v))
        err = _schema_diff(v, schema[k], "%s/%s" % (path, k))
        if err:
            return err
    return None


def validate_trial_job(run_spec: dict):
    """validateTrialJob (validator.go:376-395): only batch/v1 Jobs are checked."""
    if run_spec.get("kind") != C.JOB_KIND_JOB or run_spec.get("apiVersion") != "batch/v1":
        return
    err = _schema_diff(run_spec, _JOB, "")
    if err:
        raise ValidationError("unable to convert spec.TrialTemplate to %s: %s" % (C.JOB_KIND_JOB, err))
    containers = (((run_spec.get("spec") or {}).get("template") or {}).get("spec") or {}).get("containers")
    if not containers:
        raise ValidationError("invalid spec.trialTemplate: unable to convert spec.TrialTemplate to Job: "
                              "spec.template.spec.containers is required")


def _parse_spec(s: str):
    import yaml

    try:
        return json.loads(s)
    except ValueError:
        return yaml.safe_load(s)


def _validate_metrics_collector(inst, configured):
    mc = inst.spec.metrics_collector_spec
    kind = mc.collector.kind if mc and mc.collector else C.COLLECTOR_STDOUT
    if configured is not None and kind in (C.COLLECTOR_STDOUT, C.COLLECTOR_FILE, C.COLLECTOR_TFEVENT,
                                           C.COLLECTOR_PROMETHEUS) and kind not in configured:
        raise ValidationError("GetMetricsCollectorConfigData failed: failed to find metrics collector '%s' config "
                              "in katib-config" % kind)
    src = mc.source if mc else None
    fsp = src.file_system_path if src else None
    if kind in (C.COLLECTOR_NONE, C.COLLECTOR_STDOUT):
        pass
    elif kind == C.COLLECTOR_FILE:
        if fsp is None or fsp.kind != C.FS_KIND_FILE or not os.path.isabs(fsp.path or ""):
            raise ValidationError("file path where metrics file exists is required by "
                                  ".spec.metricsCollectorSpec.source.fileSystemPath.path")
        if fsp.format not in (C.FORMAT_TEXT, C.FORMAT_JSON):
            raise ValidationError("format of metrics file is required by "
                                  ".spec.metricsCollectorSpec.source.fileSystemPath.format")
        if fsp.format == C.FORMAT_JSON and src.filter is not None:
            raise ValidationError(".spec.metricsCollectorSpec.source.filter must be nil when format of metrics "
                                  "file is JSON")
    elif kind == C.COLLECTOR_TFEVENT:
        if fsp is None or fsp.kind != C.FS_KIND_DIRECTORY or not os.path.isabs(fsp.path or ""):
            raise ValidationError("directory path where tensorflow event files exist is required by "
                                  ".spec.metricsCollectorSpec.source.fileSystemPath.path")
        if fsp.format:
            raise ValidationError(".spec.metricsCollectorSpec.source.fileSystemPath.format must be empty")
    elif kind == C.COLLECTOR_PROMETHEUS:
        port = src.http_get.port if src and src.http_get else None
        try:
            ok = int(port) > 0
        except (TypeError, ValueError):
            ok = False
        if not ok:
            raise ValidationError(".spec.metricsCollectorSpec.source.httpGet.port must be a positive integer value "
                                  "for metrics collector kind: %s" % kind)
        if not (src.http_get.path or "").startswith("/"):
            raise ValidationError(".spec.metricsCollectorSpec.source.httpGet.path is invalid for metrics collector "
                                  "kind: %s" % kind)
    elif kind == C.COLLECTOR_CUSTOM:
        if mc.collector.custom_collector is None:
            raise ValidationError(".spec.metricsCollectorSpec.collector.customCollector is required for metrics "
                                  "collector kind: %s" % kind)
        if fsp is not None and (not os.path.isabs(fsp.path or "")
                                or fsp.kind not in (C.FS_KIND_DIRECTORY, C.FS_KIND_FILE)):
            raise ValidationError(".spec.metricsCollectorSpec.source is invalid")
    else:
        raise ValidationError("invalid metrics collector kind: %s" % kind)
    if src is not None and src.filter is not None and src.filter.metrics_format:
        for f in src.filter.metrics_format:
            try:
                re.compile(f)
            except re.error as e:
                raise ValidationError('invalid "%s" in .spec.metricsCollectorSpec.source.filter: %s' % (f, e))
            if not _TWO_GROUPS.match(f):
                raise ValidationError('invalid "%s" in .spec.metricsCollectorSpec.source.filter: two top '
                                      'subexpressions are required' % f)
