"""v1beta1 object model: Experiment / Trial / Suggestion and their sub-types.

Field names, attribute order and (de)serialisation match the reference SDK's
generated models (``sdk/python/v1beta1/kubeflow/katib/models/*.py``) and the CRD
Go types (``pkg/apis/controller/{experiments,trials,suggestions,common}/v1beta1``):

* Python attributes are snake_case; the wire/YAML form is camelCase
  (``attribute_map``), exactly as ``experiment_types.go`` json tags.
* Constructor keyword arguments are in the generated (alphabetical) order, so
  positional calls such as ``V1beta1FeasibleSpace(["a", "b"])``
  (``sdk/.../api/search.py:64``) keep working.
* ``to_dict()`` returns snake_case like the generated models;
  ``to_k8s()`` / ``from_k8s()`` speak the camelCase CRD JSON used by Experiment
  YAML files, the journal and the gRPC converters.

Instead of ~40 generated files, one declarative table drives every model.
"""

from __future__ import annotations

import copy
import datetime as _dt
import pprint
from typing import Any, Dict, List, Optional, Tuple


def _camel(snake: str) -> str:
    head, *rest = snake.split("_")
    return head + "".join(p[:1].upper() + p[1:] for p in rest)


class Model:
    """Base for every v1beta1 model.  Subclasses set ``openapi_types`` and
    ``attribute_map``; everything else is generic."""

    openapi_types: Dict[str, str] = {}
    attribute_map: Dict[str, str] = {}
    _defaults: Dict[str, Any] = {}

    def __init__(self, *args, **kwargs):
        names = list(self.openapi_types)
        kwargs.pop("local_vars_configuration", None)
        if len(args) > len(names):
            raise TypeError(f"{type(self).__name__} takes at most {len(names)} positional args")
        for n in names:
            object.__setattr__(self, n, copy.copy(self._defaults.get(n)))
        for n, v in zip(names, args):
            object.__setattr__(self, n, v)
        for k, v in kwargs.items():
            if k not in self.openapi_types:
                raise TypeError(f"{type(self).__name__} got an unexpected keyword argument '{k}'")
            object.__setattr__(self, k, v)

    # -- generic (de)serialisation ------------------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        """snake_case dict, mirrors the generated ``to_dict`` of the reference SDK."""
        out = {}
        for attr in self.openapi_types:
            out[attr] = _to_plain(getattr(self, attr), snake=True)
        return out

    def to_k8s(self) -> Dict[str, Any]:
        """camelCase dict with None/empty omitted (the CRD JSON form)."""
        out = {}
        for attr in self.openapi_types:
            v = getattr(self, attr)
            if v is None:
                continue
            pv = _to_plain(v, snake=False)
            if pv is None or (isinstance(pv, (list, dict)) and len(pv) == 0 and attr not in _KEEP_EMPTY):
                continue
            out[self.attribute_map[attr]] = pv
        return out

    @classmethod
    def from_k8s(cls, data: Optional[Dict[str, Any]]):
        if data is None:
            return None
        if isinstance(data, cls):
            return data
        rev = {v: k for k, v in cls.attribute_map.items()}
        kwargs = {}
        for key, val in data.items():
            attr = rev.get(key)
            if attr is None:
                attr = key if key in cls.openapi_types else None
            if attr is None:
                continue  # unknown field: CRDs preserve them, we drop (x-kubernetes-preserve-unknown-fields)
            kwargs[attr] = _from_plain(cls.openapi_types[attr], val)
        return cls(**kwargs)

    @classmethod
    def from_dict(cls, data):
        """Accepts snake_case or camelCase keys."""
        if data is None:
            return None
        norm = {}
        for k, v in data.items():
            norm[cls.attribute_map.get(k, k)] = v
        return cls.from_k8s(norm)

    def deepcopy(self):
        return copy.deepcopy(self)

    def to_str(self):
        return pprint.pformat(self.to_dict())

    def __repr__(self):
        return self.to_str()

    def __eq__(self, other):
        if not isinstance(other, type(self)):
            return False
        return self.to_dict() == other.to_dict()

    def __ne__(self, other):
        return not self == other


_KEEP_EMPTY = set()


def _to_plain(v, snake: bool):
    if isinstance(v, Model):
        return v.to_dict() if snake else v.to_k8s()
    if isinstance(v, list):
        return [_to_plain(x, snake) for x in v]
    if isinstance(v, dict):
        return {k: _to_plain(x, snake) for k, x in v.items()}
    if isinstance(v, _dt.datetime):
        return format_time(v)
    return v


def _from_plain(type_str: str, val):
    if val is None:
        return None
    if type_str.startswith("list["):
        inner = type_str[5:-1]
        return [_from_plain(inner, x) for x in val]
    if type_str.startswith("dict("):
        inner = type_str[5:-1].split(",", 1)[1].strip()
        return {k: _from_plain(inner, x) for k, x in val.items()}
    if type_str == "datetime":
        if isinstance(val, _dt.datetime):
            return val
        return parse_time(val)
    cls = MODEL_REGISTRY.get(type_str)
    if cls is not None:
        if isinstance(val, Model):
            return val
        return cls.from_k8s(val)
    if type_str == "int" and isinstance(val, str) and val.lstrip("-").isdigit():
        return int(val)
    return val


# --------------------------------------------------------------------------------------
# time helpers (metav1.Time is RFC3339, second precision; observation logs RFC3339Nano)
# --------------------------------------------------------------------------------------
ZERO_TIME = "0001-01-01T00:00:00Z"


def now() -> _dt.datetime:
    return _dt.datetime.now(_dt.timezone.utc)


def format_time(t: Optional[_dt.datetime]) -> Optional[str]:
    if t is None:
        return None
    if t.tzinfo is None:
        t = t.replace(tzinfo=_dt.timezone.utc)
    t = t.astimezone(_dt.timezone.utc)
    return t.strftime("%Y-%m-%dT%H:%M:%SZ")


def parse_time(s) -> Optional[_dt.datetime]:
    if s is None or s == "":
        return None
    if isinstance(s, _dt.datetime):
        return s
    s = str(s)
    if s.endswith("Z"):
        s = s[:-1] + "+00:00"
    # python < 3.11 only accepts up to 6 fractional digits
    if "." in s:
        head, frac = s.split(".", 1)
        tz = ""
        for sep in ("+", "-"):
            if sep in frac:
                i = frac.index(sep)
                frac, tz = frac[:i], frac[i:]
                break
        s = head + "." + (frac + "000000")[:6] + tz
    return _dt.datetime.fromisoformat(s)


# --------------------------------------------------------------------------------------
# declarative model table: name -> [(attr, type)], attrs in generated (alphabetical) order
# --------------------------------------------------------------------------------------
_SPECS: Dict[str, List[Tuple[str, str]]] = {
    # metadata (subset of kubernetes V1ObjectMeta that the framework uses)
    "V1ObjectMeta": [
        ("annotations", "dict(str, str)"), ("creation_timestamp", "datetime"),
        ("deletion_timestamp", "datetime"), ("finalizers", "list[str]"),
        ("generate_name", "str"), ("generation", "int"), ("labels", "dict(str, str)"),
        ("name", "str"), ("namespace", "str"), ("owner_references", "list[object]"),
        ("resource_version", "str"), ("uid", "str"),
    ],
    "V1HTTPGetAction": [("host", "str"), ("path", "str"), ("port", "object"), ("scheme", "str")],
    # common_types.go
    "V1beta1AlgorithmSetting": [("name", "str"), ("value", "str")],
    "V1beta1AlgorithmSpec": [("algorithm_name", "str"), ("algorithm_settings", "list[V1beta1AlgorithmSetting]")],
    "V1beta1EarlyStoppingSetting": [("name", "str"), ("value", "str")],
    "V1beta1EarlyStoppingSpec": [("algorithm_name", "str"), ("algorithm_settings", "list[V1beta1EarlyStoppingSetting]")],
    "V1beta1EarlyStoppingRule": [("comparison", "str"), ("name", "str"), ("start_step", "int"), ("value", "str")],
    "V1beta1MetricStrategy": [("name", "str"), ("value", "str")],
    "V1beta1ObjectiveSpec": [
        ("additional_metric_names", "list[str]"), ("goal", "float"),
        ("metric_strategies", "list[V1beta1MetricStrategy]"), ("objective_metric_name", "str"), ("type", "str"),
    ],
    "V1beta1ParameterAssignment": [("name", "str"), ("value", "str")],
    "V1beta1Metric": [("latest", "str"), ("max", "str"), ("min", "str"), ("name", "str")],
    "V1beta1Observation": [("metrics", "list[V1beta1Metric]")],
    "V1beta1FilterSpec": [("metrics_format", "list[str]")],
    "V1beta1FileSystemPath": [("format", "str"), ("kind", "str"), ("path", "str")],
    "V1beta1SourceSpec": [("file_system_path", "V1beta1FileSystemPath"), ("filter", "V1beta1FilterSpec"),
                          ("http_get", "V1HTTPGetAction")],
    "V1beta1CollectorSpec": [("custom_collector", "object"), ("kind", "str")],
    "V1beta1MetricsCollectorSpec": [("collector", "V1beta1CollectorSpec"), ("source", "V1beta1SourceSpec")],
    # experiment_types.go
    "V1beta1FeasibleSpace": [("list", "list[str]"), ("max", "str"), ("min", "str"), ("step", "str")],
    "V1beta1ParameterSpec": [("feasible_space", "V1beta1FeasibleSpace"), ("name", "str"), ("parameter_type", "str")],
    "V1beta1ConfigMapSource": [("config_map_name", "str"), ("config_map_namespace", "str"), ("template_path", "str")],
    "V1beta1TrialParameterSpec": [("description", "str"), ("name", "str"), ("reference", "str")],
    "V1beta1TrialSource": [("config_map", "V1beta1ConfigMapSource"), ("trial_spec", "object")],
    "V1beta1TrialTemplate": [
        ("config_map", "V1beta1ConfigMapSource"), ("failure_condition", "str"), ("primary_container_name", "str"),
        ("primary_pod_labels", "dict(str, str)"), ("retain", "bool"), ("success_condition", "str"),
        ("trial_parameters", "list[V1beta1TrialParameterSpec]"), ("trial_spec", "object"),
    ],
    "V1beta1GraphConfig": [("input_sizes", "list[int]"), ("num_layers", "int"), ("output_sizes", "list[int]")],
    "V1beta1Operation": [("operation_type", "str"), ("parameters", "list[V1beta1ParameterSpec]")],
    "V1beta1NasConfig": [("graph_config", "V1beta1GraphConfig"), ("operations", "list[V1beta1Operation]")],
    "V1beta1ExperimentSpec": [
        ("algorithm", "V1beta1AlgorithmSpec"), ("early_stopping", "V1beta1EarlyStoppingSpec"),
        ("max_failed_trial_count", "int"), ("max_trial_count", "int"),
        ("metrics_collector_spec", "V1beta1MetricsCollectorSpec"), ("nas_config", "V1beta1NasConfig"),
        ("objective", "V1beta1ObjectiveSpec"), ("parallel_trial_count", "int"),
        ("parameters", "list[V1beta1ParameterSpec]"), ("resume_policy", "str"),
        ("trial_template", "V1beta1TrialTemplate"),
    ],
    "V1beta1ExperimentCondition": [
        ("last_transition_time", "datetime"), ("last_update_time", "datetime"), ("message", "str"),
        ("reason", "str"), ("status", "str"), ("type", "str"),
    ],
    "V1beta1OptimalTrial": [("best_trial_name", "str"), ("observation", "V1beta1Observation"),
                            ("parameter_assignments", "list[V1beta1ParameterAssignment]")],
    "V1beta1ExperimentStatus": [
        ("completion_time", "datetime"), ("conditions", "list[V1beta1ExperimentCondition]"),
        ("current_optimal_trial", "V1beta1OptimalTrial"), ("early_stopped_trial_list", "list[str]"),
        ("failed_trial_list", "list[str]"), ("killed_trial_list", "list[str]"),
        ("last_reconcile_time", "datetime"), ("metrics_unavailable_trial_list", "list[str]"),
        ("pending_trial_list", "list[str]"), ("running_trial_list", "list[str]"), ("start_time", "datetime"),
        ("succeeded_trial_list", "list[str]"), ("trial_metrics_unavailable", "int"), ("trials", "int"),
        ("trials_early_stopped", "int"), ("trials_failed", "int"), ("trials_killed", "int"),
        ("trials_pending", "int"), ("trials_running", "int"), ("trials_succeeded", "int"),
    ],
    "V1beta1Experiment": [("api_version", "str"), ("kind", "str"), ("metadata", "V1ObjectMeta"),
                          ("spec", "V1beta1ExperimentSpec"), ("status", "V1beta1ExperimentStatus")],
    "V1beta1ExperimentList": [("api_version", "str"), ("items", "list[V1beta1Experiment]"), ("kind", "str"),
                              ("metadata", "object")],
    # trial_types.go
    "V1beta1TrialSpec": [
        ("early_stopping_rules", "list[V1beta1EarlyStoppingRule]"), ("failure_condition", "str"),
        ("labels", "dict(str, str)"), ("metrics_collector", "V1beta1MetricsCollectorSpec"),
        ("objective", "V1beta1ObjectiveSpec"), ("parameter_assignments", "list[V1beta1ParameterAssignment]"),
        ("primary_container_name", "str"), ("primary_pod_labels", "dict(str, str)"), ("retain_run", "bool"),
        ("run_spec", "object"), ("success_condition", "str"),
    ],
    "V1beta1TrialCondition": [
        ("last_transition_time", "datetime"), ("last_update_time", "datetime"), ("message", "str"),
        ("reason", "str"), ("status", "str"), ("type", "str"),
    ],
    "V1beta1TrialStatus": [("completion_time", "datetime"), ("conditions", "list[V1beta1TrialCondition]"),
                           ("last_reconcile_time", "datetime"), ("observation", "V1beta1Observation"),
                           ("start_time", "datetime")],
    "V1beta1Trial": [("api_version", "str"), ("kind", "str"), ("metadata", "V1ObjectMeta"),
                     ("spec", "V1beta1TrialSpec"), ("status", "V1beta1TrialStatus")],
    "V1beta1TrialList": [("api_version", "str"), ("items", "list[V1beta1Trial]"), ("kind", "str"),
                         ("metadata", "object")],
    # suggestion_types.go
    "V1beta1SuggestionSpec": [("algorithm", "V1beta1AlgorithmSpec"), ("early_stopping", "V1beta1EarlyStoppingSpec"),
                              ("requests", "int"), ("resume_policy", "str")],
    "V1beta1TrialAssignment": [("early_stopping_rules", "list[V1beta1EarlyStoppingRule]"),
                               ("labels", "dict(str, str)"), ("name", "str"),
                               ("parameter_assignments", "list[V1beta1ParameterAssignment]")],
    "V1beta1SuggestionCondition": [
        ("last_transition_time", "datetime"), ("last_update_time", "datetime"), ("message", "str"),
        ("reason", "str"), ("status", "str"), ("type", "str"),
    ],
    "V1beta1SuggestionStatus": [
        ("algorithm_settings", "list[V1beta1AlgorithmSetting]"), ("completion_time", "datetime"),
        ("conditions", "list[V1beta1SuggestionCondition]"), ("last_reconcile_time", "datetime"),
        ("start_time", "datetime"), ("suggestion_count", "int"), ("suggestions", "list[V1beta1TrialAssignment]"),
    ],
    "V1beta1Suggestion": [("api_version", "str"), ("kind", "str"), ("metadata", "V1ObjectMeta"),
                          ("spec", "V1beta1SuggestionSpec"), ("status", "V1beta1SuggestionStatus")],
    "V1beta1SuggestionList": [("api_version", "str"), ("items", "list[V1beta1Suggestion]"), ("kind", "str"),
                              ("metadata", "object")],
}

_CONDITION_DEFAULTS = {"status": "", "type": ""}

MODEL_REGISTRY: Dict[str, type] = {}


def _make(name: str, fields: List[Tuple[str, str]]):
    attrs = {
        "openapi_types": {a: t for a, t in fields},
        "attribute_map": {a: _camel(a) for a, _ in fields},
        "_defaults": dict(_CONDITION_DEFAULTS) if name.endswith("Condition") else {},
        "__doc__": f"{name} (v1beta1 model, see katib_amd.api.models)",
    }
    if name == "V1ObjectMeta":
        attrs["attribute_map"]["owner_references"] = "ownerReferences"
    cls = type(name, (Model,), attrs)
    MODEL_REGISTRY[name] = cls
    return cls


for _n, _f in _SPECS.items():
    globals()[_n] = _make(_n, _f)

# explicit names for static analysis / IDEs
V1ObjectMeta = MODEL_REGISTRY["V1ObjectMeta"]
V1HTTPGetAction = MODEL_REGISTRY["V1HTTPGetAction"]
V1beta1AlgorithmSetting = MODEL_REGISTRY["V1beta1AlgorithmSetting"]
V1beta1AlgorithmSpec = MODEL_REGISTRY["V1beta1AlgorithmSpec"]
V1beta1EarlyStoppingSetting = MODEL_REGISTRY["V1beta1EarlyStoppingSetting"]
V1beta1EarlyStoppingSpec = MODEL_REGISTRY["V1beta1EarlyStoppingSpec"]
V1beta1EarlyStoppingRule = MODEL_REGISTRY["V1beta1EarlyStoppingRule"]
V1beta1MetricStrategy = MODEL_REGISTRY["V1beta1MetricStrategy"]
V1beta1ObjectiveSpec = MODEL_REGISTRY["V1beta1ObjectiveSpec"]
V1beta1ParameterAssignment = MODEL_REGISTRY["V1beta1ParameterAssignment"]
V1beta1Metric = MODEL_REGISTRY["V1beta1Metric"]
V1beta1Observation = MODEL_REGISTRY["V1beta1Observation"]
V1beta1FilterSpec = MODEL_REGISTRY["V1beta1FilterSpec"]
V1beta1FileSystemPath = MODEL_REGISTRY["V1beta1FileSystemPath"]
V1beta1SourceSpec = MODEL_REGISTRY["V1beta1SourceSpec"]
V1beta1CollectorSpec = MODEL_REGISTRY["V1beta1CollectorSpec"]
V1beta1MetricsCollectorSpec = MODEL_REGISTRY["V1beta1MetricsCollectorSpec"]
V1beta1FeasibleSpace = MODEL_REGISTRY["V1beta1FeasibleSpace"]
V1beta1ParameterSpec = MODEL_REGISTRY["V1beta1ParameterSpec"]
V1beta1ConfigMapSource = MODEL_REGISTRY["V1beta1ConfigMapSource"]
V1beta1TrialParameterSpec = MODEL_REGISTRY["V1beta1TrialParameterSpec"]
V1beta1TrialSource = MODEL_REGISTRY["V1beta1TrialSource"]
V1beta1TrialTemplate = MODEL_REGISTRY["V1beta1TrialTemplate"]
V1beta1GraphConfig = MODEL_REGISTRY["V1beta1GraphConfig"]
V1beta1Operation = MODEL_REGISTRY["V1beta1Operation"]
V1beta1NasConfig = MODEL_REGISTRY["V1beta1NasConfig"]
V1beta1ExperimentSpec = MODEL_REGISTRY["V1beta1ExperimentSpec"]
V1beta1ExperimentCondition = MODEL_REGISTRY["V1beta1ExperimentCondition"]
V1beta1OptimalTrial = MODEL_REGISTRY["V1beta1OptimalTrial"]
V1beta1ExperimentStatus = MODEL_REGISTRY["V1beta1ExperimentStatus"]
V1beta1Experiment = MODEL_REGISTRY["V1beta1Experiment"]
V1beta1ExperimentList = MODEL_REGISTRY["V1beta1ExperimentList"]
V1beta1TrialSpec = MODEL_REGISTRY["V1beta1TrialSpec"]
V1beta1TrialCondition = MODEL_REGISTRY["V1beta1TrialCondition"]
V1beta1TrialStatus = MODEL_REGISTRY["V1beta1TrialStatus"]
V1beta1Trial = MODEL_REGISTRY["V1beta1Trial"]
V1beta1TrialList = MODEL_REGISTRY["V1beta1TrialList"]
V1beta1SuggestionSpec = MODEL_REGISTRY["V1beta1SuggestionSpec"]
V1beta1TrialAssignment = MODEL_REGISTRY["V1beta1TrialAssignment"]
V1beta1SuggestionCondition = MODEL_REGISTRY["V1beta1SuggestionCondition"]
V1beta1SuggestionStatus = MODEL_REGISTRY["V1beta1SuggestionStatus"]
V1beta1Suggestion = MODEL_REGISTRY["V1beta1Suggestion"]
V1beta1SuggestionList = MODEL_REGISTRY["V1beta1SuggestionList"]

# trialSpec and customCollector are free-form unstructured objects: keep as plain dicts.
__all__ = [n for n in MODEL_REGISTRY] + ["Model", "MODEL_REGISTRY", "parse_time", "format_time", "now", "ZERO_TIME"]
