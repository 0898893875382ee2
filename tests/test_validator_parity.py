"""Table-driven port of the experiment webhook's unit tests
(reference ``pkg/webhook/v1beta1/experiment/validator/validator_test.go``) and of
GetDeployedJobStatus's tests (``pkg/controller.v1beta1/trial/util/job_util_test.go``).

Each case keeps the reference's description; the fake experiment, Job and trial
parameters are the ones of validator_test.go:1227-1349, written as manifests.
"""
import copy
import json

import pytest
import yaml

from katib_amd.api import constants as C
from katib_amd.api.models import V1beta1Experiment
from katib_amd.api.validation import (ValidationError, _validate_metrics_collector, _validate_parameters,
                                      _validate_trial_template, validate_experiment, validate_trial_job)
from katib_amd.controller import gjson


def fake_job():
    return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"creationTimestamp": None},
            "spec": {"template": {"metadata": {"creationTimestamp": None}, "spec": {"containers": [{
                "name": "training-container", "image": "docker.io/kubeflowkatib/pytorch-mnist-cpu",
                "command": ["python3", "--epochs=1", "--batch-size=16", "/opt/pytorch-mnist/mnist.py",
                            "--lr=${trialParameters.learningRate}", "--momentum=${trialParameters.momentum}"],
                "resources": {}}]}}},
            "status": {}}


def fake_manifest():
    return {
        "apiVersion": "kubeflow.org/v1beta1", "kind": "Experiment",
        "metadata": {"name": "fake", "namespace": "fakens"},
        "spec": {
            "maxTrialCount": 6,
            "metricsCollectorSpec": {"collector": {"kind": "StdOut"}},
            "objective": {"type": "maximize", "goal": 0.11, "objectiveMetricName": "testme"},
            "algorithm": {"algorithmName": "test", "algorithmSettings": [{"name": "test1", "value": "value1"}]},
            "earlyStopping": {"algorithmName": "test", "algorithmSettings": [{"name": "test1", "value": "value1"}]},
            "parameters": [
                {"name": "lr", "parameterType": "int", "feasibleSpace": {"max": "5", "min": "1"}},
                {"name": "momentum", "parameterType": "categorical",
                 "feasibleSpace": {"list": ["0.95", "0.85", "0.75"]}},
            ],
            "trialTemplate": {
                "primaryContainerName": "training-container",
                "successCondition": C.DEFAULT_JOB_SUCCESS_CONDITION,
                "failureCondition": C.DEFAULT_JOB_FAILURE_CONDITION,
                "trialSpec": fake_job(),
                "trialParameters": [
                    {"name": "learningRate", "description": "Learning rate", "reference": "lr"},
                    {"name": "momentum", "description": "Momentum for the training model", "reference": "momentum"},
                ],
            },
        },
    }


def fake(mut=None):
    m = fake_manifest()
    if mut is not None:
        mut(m)
    return V1beta1Experiment.from_k8s(m)


def _set(path, value):
    def mut(m):
        cur = m
        for k in path[:-1]:
            cur = cur[k]
        if value is _DEL:
            cur.pop(path[-1], None)
        else:
            cur[path[-1]] = copy.deepcopy(value)
    return mut


_DEL = object()
S = ("spec",)


def _status_trials(n, failed):
    def mut(m):
        m["status"] = {"trials": n}
        m["spec"]["maxFailedTrialCount"] = failed
    return mut


def _succeeded_never(m):
    m["spec"]["resumePolicy"] = "Never"
    m["status"] = {"conditions": [{"type": "Succeeded", "status": "True", "reason": C.EXPERIMENT_MAX_TRIALS_REACHED_REASON,
                                   "message": "Experiment is succeeded"}]}


def _both(**kw):
    def mut(m):
        m["spec"].update(kw)
    return mut


# (description, mutation of the new experiment, mutation of the old one or None, expect error)
EXPERIMENT_CASES = [
    ("Name is invalid", _set(("metadata", "name"), "1234-test"), None, True),
    ("Objective is nil", _set(S + ("objective",), _DEL), None, True),
    ("Objective type is unknown", _set(S + ("objective", "type"), ""), None, True),
    ("Objective metric name is empty", _set(S + ("objective", "objectiveMetricName"), ""), None, True),
    ("additionalMetricNames should not contain objective metric name",
     _set(S + ("objective",), {"type": "maximize", "goal": 0.11, "objectiveMetricName": "objective",
                               "additionalMetricNames": ["objective", "objective-1"]}), None, True),
    ("Algorithm is nil", _set(S + ("algorithm",), _DEL), None, True),
    ("Algorithm name is empty", _set(S + ("algorithm", "algorithmName"), ""), None, True),
    ("EarlyStopping is nil", _set(S + ("earlyStopping",), _DEL), None, False),
    ("EarlyStopping AlgorithmName is empty", _set(S + ("earlyStopping", "algorithmName"), ""), None, True),
    ("Run validator for correct experiment", None, None, False),
    ("Max failed trial count is negative", _set(S + ("maxFailedTrialCount",), -1), None, True),
    ("Max trial count is negative", _set(S + ("maxTrialCount",), -1), None, True),
    ("Parallel trial count is negative", _set(S + ("parallelTrialCount",), -1), None, True),
    ("Run validator to correct resume experiment", None, lambda m: None, False),
    ("Resume succeeded experiment with ResumePolicy = NeverResume", None, _succeeded_never, True),
    ("Resume experiment with MaxTrialCount <= Status.Trials", None, _status_trials(6, 2), True),
    ("Change algorithm name when resuming experiment", None, _set(S + ("algorithm", "algorithmName"), "not-test"),
     True),
    ("Invalid resume policy", _set(S + ("resumePolicy",), "invalid-policy"), None, True),
    ("Parameters and NAS config is nil", _set(S + ("parameters",), []), None, True),
    ("Parameters and NAS config is not nil", _set(S + ("nasConfig",), {"operations": [{"operationType": "op1"}]}),
     None, True),
    ("Trial template is nil", _set(S + ("trialTemplate",), _DEL), None, True),
    ("Invalid feasible space in parameters", _set(S + ("parameters", 1, "feasibleSpace", "max"), "5"), None, True),
    ("maxFailedTrialCount greater than maxTrialCount", _both(maxTrialCount=5, maxFailedTrialCount=6), None, True),
    ("maxFailedTrialCount equal to maxTrialCount", _both(maxTrialCount=5, maxFailedTrialCount=5), None, False),
    ("parallelTrialCount greater than maxTrialCount", _both(maxTrialCount=5, parallelTrialCount=6), None, True),
    ("parallelTrialCount equal to maxTrialCount", _both(maxTrialCount=5, parallelTrialCount=5), None, False),
]


@pytest.mark.parametrize("desc,mut,old_mut,err", EXPERIMENT_CASES, ids=[c[0] for c in EXPERIMENT_CASES])
def test_validate_experiment(desc, mut, old_mut, err):
    inst = fake(mut)
    old = fake(old_mut) if old_mut is not None else None
    algos = {"test"}
    if err:
        with pytest.raises(ValidationError):
            validate_experiment(inst, old, suggestion_algorithms=algos, early_stopping_algorithms=algos)
    else:
        validate_experiment(inst, old, suggestion_algorithms=algos, early_stopping_algorithms=algos)


PARAMETER_CASES = [
    ("Invalid parameter type", _set(S + ("parameters", 0, "parameterType"), "invalid-type")),
    ("Feasible space is nil", _set(S + ("parameters", 0, "feasibleSpace"), {})),
    ("Not empty list for int parameter type", _set(S + ("parameters", 0, "feasibleSpace", "list"), ["invalid-list"])),
    ("Empty max and min for int parameter type",
     _set(S + ("parameters", 0, "feasibleSpace"), {"max": "", "min": "", "step": "1"})),
    ("Not empty max for categorical parameter type", _set(S + ("parameters", 1, "feasibleSpace", "max"), "1")),
]


@pytest.mark.parametrize("desc,mut", PARAMETER_CASES, ids=[c[0] for c in PARAMETER_CASES])
def test_validate_parameters(desc, mut):
    with pytest.raises(ValidationError):
        _validate_parameters(fake(mut).spec.parameters)


def _job_str(mut=None):
    j = fake_job()
    if mut is not None:
        mut(j)
    return json.dumps(j)


def _cmd(j):
    return j["spec"]["template"]["spec"]["containers"][0]["command"]


INVALID_PARAMETER_JOB = """apiVersion: batch/v1
kind: Job
spec:
  template:
    spec:
      containers:
        - name: fake-trial
          image: test-image
          command:
            - --invalidParameter={'num_layers': 2, 'input_sizes': [32, 32, 3]}
            - --lr=${trialParameters.learningRate}"
            - --num-layers=${trialParameters.numberLayers}"""


def _getter(text=None, exc=None):
    def get(_inst):
        if exc is not None:
            raise exc
        return text if text is not None else _job_str()
    return get


def _cm(path=None):
    def mut(m):
        t = m["spec"]["trialTemplate"]
        t.pop("trialSpec")
        t["configMap"] = {"configMapName": "config-map-name", "configMapNamespace": "config-map-namespace"}
        if path:
            t["configMap"]["templatePath"] = path
    return mut


def _tp(i, key, value):
    return _set(S + ("trialTemplate", "trialParameters", i, key), value)


def _dup(key):
    def mut(m):
        tp = m["spec"]["trialTemplate"]["trialParameters"]
        tp[1][key] = tp[0][key]
    return mut


def _no_params_wrong_ref(m):
    m["spec"].pop("parameters")
    m["spec"]["trialTemplate"]["trialParameters"][1]["reference"] = "wrong-ref"


def _metadata(m):
    m["spec"]["trialTemplate"]["trialSpec"]["metadata"].update(name="trial-name", namespace="trial-namespace")


# (description, mutation, template getter, expect error)
TRIAL_TEMPLATE_CASES = [
    ("Trial parameters is nil", _set(S + ("trialTemplate", "trialParameters"), _DEL), None, True),
    ("Trial spec nil", _set(S + ("trialTemplate", "trialSpec"), _DEL), None, True),
    ("Trial spec and ConfigMap is not nil",
     _set(S + ("trialTemplate", "configMap"), {"configMapName": "config-map-name"}), None, True),
    ("Missed template path in ConfigMap", _cm(), None, True),
    ("Wrong template path in ConfigMap", _cm("wrong-path"), _getter(exc=KeyError("NotFound")), True),
    ("Empty reference or name in Trial parameters", _tp(0, "reference", ""), None, True),
    ("Wrong name in Trial parameters", _tp(0, "name", "{invalid-name}"), None, True),
    ("Duplicate name in Trial parameters", _dup("name"), None, True),
    ("Duplicate reference in Trial parameters", _dup("reference"), None, True),
    ("Trial template contains Trial parameters which weren't referenced from spec.parameters",
     _tp(1, "reference", "wrong-ref"), None, True),
    ("Trial template contains Trial parameters when spec.parameters is empty", _no_params_wrong_ref, None, False),
    ("Trial template contains Trial metadata reference as parameter", _tp(1, "reference", "${trialSpec.Name}"),
     None, False),
    ("Trial template contains Trial annotation reference as parameter",
     _tp(1, "reference", "${trialSpec.Annotations[test-annotation]}"), None, False),
    ("Trial template contains Trial's label reference as parameter",
     _tp(1, "reference", "${trialSpec.Labels[test-label]}"), None, False),
    ("Trial template doesn't contain parameter from Trial parameters", None,
     _getter(_job_str(lambda j: _cmd(j).__setitem__(2, "--lr=${trialParameters.invalidParameter}"))), True),
    ("Trial template contains extra parameter", None,
     _getter(_job_str(lambda j: _cmd(j).append("--extra-parameter=${trialParameters.extraParameter}"))), True),
    ("Trial template is unable to convert to unstructured after substitution", None, _getter(INVALID_PARAMETER_JOB),
     True),
    ("Trial template contains metadata.name or metadata.namespace", _metadata, None, True),
    ("Trial template doesn't contain APIVersion or Kind", None,
     _getter(_job_str(lambda j: j.__setitem__("apiVersion", ""))), True),
    ("Trial template has custom Kind", None, _getter(_job_str(lambda j: j.__setitem__("kind", "CustomKind"))), False),
    ("Trial template doesn't have PrimaryContainerName", _set(S + ("trialTemplate", "primaryContainerName"), ""),
     None, True),
    ("Trial template doesn't have SuccessCondition", _set(S + ("trialTemplate", "successCondition"), ""), None, True),
]


@pytest.mark.parametrize("desc,mut,getter,err", TRIAL_TEMPLATE_CASES, ids=[c[0] for c in TRIAL_TEMPLATE_CASES])
def test_validate_trial_template(desc, mut, getter, err):
    inst = fake(mut)
    if err:
        with pytest.raises(ValidationError):
            _validate_trial_template(inst, getter)
    else:
        _validate_trial_template(inst, getter)


TRIAL_JOB_CASES = [
    ("Trial template has invalid Batch Job parameter", """apiVersion: batch/v1
kind: Job
spec:
  template:
    spec:
      containers:
        name: container-must-be-list""", True),
    ("Trial template has invalid Batch Job structure", """apiVersion: batch/v1
kind: Job
spec:
  template:
    invalidSpec: not-job-format
    spec:
      containers:
        - name: invalid-list""", True),
    ("Valid case with nvidia.com/gpu resource in Trial template", """apiVersion: batch/v1
kind: Job
spec:
  template:
    spec:
      containers:
        - resources:
            limits:
              nvidia.com/gpu: 1
            requests:
              nvidia.com/gpu: 1""", False),
    ("Only validate Kuernetes Job", """apiVersion: test/v1
kind: Job
spec:
  template:
    spec:
      containers:
      - name: container""", False),
]


@pytest.mark.parametrize("desc,text,err", TRIAL_JOB_CASES, ids=[c[0] for c in TRIAL_JOB_CASES])
def test_validate_trial_job(desc, text, err):
    spec = yaml.safe_load(text)
    if err:
        with pytest.raises(ValidationError):
            validate_trial_job(spec)
    else:
        validate_trial_job(spec)


def _mc(collector, source=None):
    spec = {"collector": collector}
    if source is not None:
        spec["source"] = source
    return _set(S + ("metricsCollectorSpec",), spec)


FILE_TEXT = {"path": "/absolute/path", "kind": "File", "format": "TEXT"}
METRICS_COLLECTOR_CASES = [
    ("Invalid metrics collector Kind", _mc({"kind": "invalid-kind"}), True),
    ("Invalid path for File metrics collector",
     _mc({"kind": "File"}, {"fileSystemPath": {"path": "not/absolute/path", "format": "TEXT"}}), True),
    ("Invalid path for TF event metrics collector",
     _mc({"kind": "TensorFlowEvent"}, {"fileSystemPath": {"path": "not/absolute/path"}}), True),
    ("Invalid file format for TF event metrics collector",
     _mc({"kind": "TensorFlowEvent"},
         {"fileSystemPath": {"path": "/absolute/path", "format": "JSON", "kind": "Directory"}}), True),
    ("Invalid port for Prometheus metrics collector",
     _mc({"kind": "PrometheusMetric"}, {"httpGet": {"port": "Port"}}), True),
    ("Invalid path for Prometheus metrics collector",
     _mc({"kind": "PrometheusMetric"}, {"httpGet": {"port": 8888, "path": "not/valid/path"}}), True),
    ("Empty container for Custom metrics collector", _mc({"kind": "Custom"}), True),
    ("Invalid path for Custom metrics collector",
     _mc({"kind": "Custom", "customCollector": {"name": "my-collector"}},
         {"fileSystemPath": {"path": "not/absolute/path"}}), True),
    ("Invalid metrics format regex for File metrics collector",
     _mc({"kind": "File"}, {"filter": {"metricsFormat": ["["]}, "fileSystemPath": FILE_TEXT}), True),
    ("One subexpression in metrics format",
     _mc({"kind": "File"}, {"filter": {"metricsFormat": [r"{metricName: ([\w|-]+)}"]}, "fileSystemPath": FILE_TEXT}),
     True),
    ("Invalid file format for File metrics collector",
     _mc({"kind": "File"}, {"fileSystemPath": {"path": "/absolute/path", "kind": "File", "format": "invalid"}}), True),
    ("Invalid metrics filer for File metrics collector when file format is `JSON`",
     _mc({"kind": "File"}, {"filter": {}, "fileSystemPath": {"path": "/absolute/path", "kind": "File",
                                                              "format": "JSON"}}), True),
    ("Run validator for correct File metrics collector",
     _mc({"kind": "File"}, {"fileSystemPath": {"path": "/absolute/path", "kind": "File", "format": "JSON"}}), False),
]


@pytest.mark.parametrize("desc,mut,err", METRICS_COLLECTOR_CASES, ids=[c[0] for c in METRICS_COLLECTOR_CASES])
def test_validate_metrics_collector(desc, mut, err):
    inst = fake(mut)
    configured = {"StdOut", "File", "TensorFlowEvent", "PrometheusMetric"}
    if err:
        with pytest.raises(ValidationError):
            _validate_metrics_collector(inst, configured)
    else:
        _validate_metrics_collector(inst, configured)


@pytest.mark.parametrize("desc,kw", [
    ("Get metrics collector config data error", dict(metrics_collectors={"File"})),
    ("Get early stopping config data error", dict(early_stopping_algorithms=set())),
    ("Get suggestion config data error", dict(suggestion_algorithms=set())),
])
def test_validate_config_data(desc, kw):
    """TestValidateConfigData: a kind/algorithm missing from katib-config is an error."""
    args = dict(suggestion_algorithms={"test"}, early_stopping_algorithms={"test"},
                metrics_collectors={"StdOut"})
    args.update(kw)
    with pytest.raises(ValidationError, match="config"):
        validate_experiment(fake(), **args)


# ---- job_util_test.go: GetDeployedJobStatus ----------------------------------------------

SUCCESS = 'status.conditions.#(type=="Complete")#|#(status=="True")#'
FAILURE = 'status.conditions.#(type=="Failed")#|#(status=="True")#'


def _deployed(failed_status="False", complete_status="True"):
    return {"metadata": {"name": "test-job"},
            "status": {"conditions": [
                {"type": "Failed", "status": failed_status, "reason": "test-reason", "message": "test-message"},
                {"type": "Complete", "status": complete_status, "reason": "test-reason", "message": "test-message"}],
                "succeeded": 1}}


@pytest.mark.parametrize("desc,success,job,want", [
    ("Job status is running", SUCCESS, _deployed("False", "False"), {"condition": "Running"}),
    ("Job status is succeeded, reason and message must be returned", SUCCESS, _deployed(),
     {"condition": "Succeeded", "message": "test-message", "reason": "test-reason"}),
    ("Job status is failed, reason and message must be returned", SUCCESS, _deployed("True", "False"),
     {"condition": "Failed", "message": "test-message", "reason": "test-reason"}),
    ("Job status is succeeded because status.succeeded = 1", "status.[@this].#(succeeded==1)", _deployed(),
     {"condition": "Succeeded"}),
])
def test_deployed_job_status(desc, success, job, want):
    assert gjson.deployed_job_status(job, success, FAILURE) == want


def test_deployed_job_status_running_trial_needs_no_update():
    assert gjson.deployed_job_status(_deployed("False", "False"), SUCCESS, FAILURE, trial_running=True) is None


def test_failure_condition_wins_over_success():
    job = _deployed("True", "True")
    assert gjson.deployed_job_status(job, SUCCESS, FAILURE)["condition"] == "Failed"
