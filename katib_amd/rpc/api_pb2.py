"""Protobuf messages of the Katib gRPC API ``api.v1.beta1`` and ``grpc.health.v1``.

``protoc``/``grpc_tools`` are not available in this environment, so instead of a
generated ``api_pb2.py`` the file descriptor is assembled in code from a compact
schema table. Package names, message names, field names, field numbers and enum
values are identical to the reference ``pkg/apis/manager/v1beta1/api.proto:11-370``
and ``pkg/apis/manager/health/health.proto:1-20`` so the wire format is
compatible with any Katib client or server.

Usage mirrors a generated module: ``api_pb2.GetSuggestionsRequest(...)``,
``api_pb2.ParameterType.Value("DOUBLE")``, ``api_pb2.DOUBLE``.
"""

from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto

# type aliases
_T = {
    "string": _F.TYPE_STRING, "int32": _F.TYPE_INT32, "double": _F.TYPE_DOUBLE, "bool": _F.TYPE_BOOL,
}

# (name, [fields], nested messages, nested enums)
# field: (name, number, type, label) where type is a scalar name, "msg:.pkg.Type" or "enum:.pkg.Type";
# label "r" repeated, "" optional, "map" -> map<string,string>
PKG = "api.v1.beta1"

_ENUMS = {
    "ParameterType": [("UNKNOWN_TYPE", 0), ("DOUBLE", 1), ("INT", 2), ("DISCRETE", 3), ("CATEGORICAL", 4)],
    "ObjectiveType": [("UNKNOWN", 0), ("MINIMIZE", 1), ("MAXIMIZE", 2)],
    "ComparisonType": [("UNKNOWN_COMPARISON", 0), ("EQUAL", 1), ("LESS", 2), ("GREATER", 3)],
}

_TRIAL_CONDITION = [("CREATED", 0), ("RUNNING", 1), ("SUCCEEDED", 2), ("KILLED", 3), ("FAILED", 4),
                    ("METRICSUNAVAILABLE", 5), ("EARLYSTOPPED", 6), ("UNKNOWN", 7)]


def _m(t):
    return "msg:." + PKG + "." + t


def _e(t):
    return "enum:." + PKG + "." + t


_MESSAGES = [
    ("Experiment", [("name", 1, "string", ""), ("spec", 2, _m("ExperimentSpec"), "")], [], []),
    ("ExperimentSpec", [
        ("parameter_specs", 1, _m("ExperimentSpec.ParameterSpecs"), ""),
        ("objective", 2, _m("ObjectiveSpec"), ""),
        ("algorithm", 3, _m("AlgorithmSpec"), ""),
        ("early_stopping", 4, _m("EarlyStoppingSpec"), ""),
        ("parallel_trial_count", 5, "int32", ""),
        ("max_trial_count", 6, "int32", ""),
        ("nas_config", 7, _m("NasConfig"), ""),
    ], [("ParameterSpecs", [("parameters", 1, _m("ParameterSpec"), "r")], [], [])], []),
    ("ParameterSpec", [("name", 1, "string", ""), ("parameter_type", 2, _e("ParameterType"), ""),
                       ("feasible_space", 3, _m("FeasibleSpace"), "")], [], []),
    ("FeasibleSpace", [("max", 1, "string", ""), ("min", 2, "string", ""), ("list", 3, "string", "r"),
                       ("step", 4, "string", "")], [], []),
    ("ObjectiveSpec", [("type", 1, _e("ObjectiveType"), ""), ("goal", 2, "double", ""),
                       ("objective_metric_name", 3, "string", ""),
                       ("additional_metric_names", 4, "string", "r")], [], []),
    ("AlgorithmSpec", [("algorithm_name", 1, "string", ""),
                       ("algorithm_settings", 2, _m("AlgorithmSetting"), "r")], [], []),
    ("AlgorithmSetting", [("name", 1, "string", ""), ("value", 2, "string", "")], [], []),
    ("EarlyStoppingSpec", [("algorithm_name", 1, "string", ""),
                           ("algorithm_settings", 2, _m("EarlyStoppingSetting"), "r")], [], []),
    ("EarlyStoppingSetting", [("name", 1, "string", ""), ("value", 2, "string", "")], [], []),
    ("NasConfig", [("graph_config", 1, _m("GraphConfig"), ""), ("operations", 2, _m("NasConfig.Operations"), "")],
     [("Operations", [("operation", 1, _m("Operation"), "r")], [], [])], []),
    ("GraphConfig", [("num_layers", 1, "int32", ""), ("input_sizes", 2, "int32", "r"),
                     ("output_sizes", 3, "int32", "r")], [], []),
    ("Operation", [("operation_type", 1, "string", ""),
                   ("parameter_specs", 2, _m("Operation.ParameterSpecs"), "")],
     [("ParameterSpecs", [("parameters", 1, _m("ParameterSpec"), "r")], [], [])], []),
    ("Trial", [("name", 1, "string", ""), ("spec", 2, _m("TrialSpec"), ""), ("status", 3, _m("TrialStatus"), "")],
     [], []),
    ("TrialSpec", [("objective", 2, _m("ObjectiveSpec"), ""),
                   ("parameter_assignments", 3, _m("TrialSpec.ParameterAssignments"), ""),
                   ("labels", 4, "string", "map")],
     [("ParameterAssignments", [("assignments", 1, _m("ParameterAssignment"), "r")], [], [])], []),
    ("ParameterAssignment", [("name", 1, "string", ""), ("value", 2, "string", "")], [], []),
    ("TrialStatus", [("start_time", 1, "string", ""), ("completion_time", 2, "string", ""),
                     ("condition", 3, _e("TrialStatus.TrialConditionType"), ""),
                     ("observation", 4, _m("Observation"), "")], [], [("TrialConditionType", _TRIAL_CONDITION)]),
    ("Observation", [("metrics", 1, _m("Metric"), "r")], [], []),
    ("Metric", [("name", 1, "string", ""), ("value", 2, "string", "")], [], []),
    ("ReportObservationLogRequest", [("trial_name", 1, "string", ""),
                                     ("observation_log", 2, _m("ObservationLog"), "")], [], []),
    ("ReportObservationLogReply", [], [], []),
    ("ObservationLog", [("metric_logs", 1, _m("MetricLog"), "r")], [], []),
    ("MetricLog", [("time_stamp", 1, "string", ""), ("metric", 2, _m("Metric"), "")], [], []),
    ("GetObservationLogRequest", [("trial_name", 1, "string", ""), ("metric_name", 2, "string", ""),
                                  ("start_time", 3, "string", ""), ("end_time", 4, "string", "")], [], []),
    ("GetObservationLogReply", [("observation_log", 1, _m("ObservationLog"), "")], [], []),
    ("DeleteObservationLogRequest", [("trial_name", 1, "string", "")], [], []),
    ("DeleteObservationLogReply", [], [], []),
    ("GetSuggestionsRequest", [("experiment", 1, _m("Experiment"), ""), ("trials", 2, _m("Trial"), "r"),
                               ("current_request_number", 4, "int32", ""),
                               ("total_request_number", 5, "int32", "")], [], []),
    ("GetSuggestionsReply", [
        ("parameter_assignments", 1, _m("GetSuggestionsReply.ParameterAssignments"), "r"),
        ("algorithm", 2, _m("AlgorithmSpec"), ""),
        ("early_stopping_rules", 3, _m("EarlyStoppingRule"), "r"),
    ], [("ParameterAssignments", [("assignments", 1, _m("ParameterAssignment"), "r"),
                                  ("trial_name", 2, "string", ""), ("labels", 3, "string", "map")], [], [])], []),
    ("ValidateAlgorithmSettingsRequest", [("experiment", 1, _m("Experiment"), "")], [], []),
    ("ValidateAlgorithmSettingsReply", [], [], []),
    ("GetEarlyStoppingRulesRequest", [("experiment", 1, _m("Experiment"), ""), ("trials", 2, _m("Trial"), "r"),
                                      ("db_manager_address", 3, "string", "")], [], []),
    ("GetEarlyStoppingRulesReply", [("early_stopping_rules", 1, _m("EarlyStoppingRule"), "r")], [], []),
    ("EarlyStoppingRule", [("name", 1, "string", ""), ("value", 2, "string", ""),
                           ("comparison", 3, _e("ComparisonType"), ""), ("start_step", 4, "int32", "")], [], []),
    ("ValidateEarlyStoppingSettingsRequest", [("early_stopping", 1, _m("EarlyStoppingSpec"), "")], [], []),
    ("ValidateEarlyStoppingSettingsReply", [], [], []),
    ("SetTrialStatusRequest", [("trial_name", 1, "string", "")], [], []),
    ("SetTrialStatusReply", [], [], []),
]

_SERVICES = [
    ("DBManager", [("ReportObservationLog", "ReportObservationLogRequest", "ReportObservationLogReply"),
                   ("GetObservationLog", "GetObservationLogRequest", "GetObservationLogReply"),
                   ("DeleteObservationLog", "DeleteObservationLogRequest", "DeleteObservationLogReply")]),
    ("Suggestion", [("GetSuggestions", "GetSuggestionsRequest", "GetSuggestionsReply"),
                    ("ValidateAlgorithmSettings", "ValidateAlgorithmSettingsRequest",
                     "ValidateAlgorithmSettingsReply")]),
    ("EarlyStopping", [("GetEarlyStoppingRules", "GetEarlyStoppingRulesRequest", "GetEarlyStoppingRulesReply"),
                       ("SetTrialStatus", "SetTrialStatusRequest", "SetTrialStatusReply"),
                       ("ValidateEarlyStoppingSettings", "ValidateEarlyStoppingSettingsRequest",
                        "ValidateEarlyStoppingSettingsReply")]),
]


def _camel(s):
    return "".join(p[:1].upper() + p[1:] for p in s.split("_"))


def _fill_message(mp: descriptor_pb2.DescriptorProto, name, fields, nested, enums, scope):
    mp.name = name
    full = scope + "." + name
    for en, vals in enums:
        ep = mp.enum_type.add()
        ep.name = en
        for vn, vv in vals:
            v = ep.value.add()
            v.name = vn
            v.number = vv
    for nn, nf, nnest, nenum in nested:
        _fill_message(mp.nested_type.add(), nn, nf, nnest, nenum, full)
    for fname, num, ftype, label in fields:
        f = mp.field.add()
        f.name = fname
        f.number = num
        f.json_name = fname[0] + _camel(fname)[1:]
        if label == "map":
            entry_name = _camel(fname) + "Entry"
            ent = mp.nested_type.add()
            ent.name = entry_name
            ent.options.map_entry = True
            for i, kn in enumerate(("key", "value"), start=1):
                kf = ent.field.add()
                kf.name = kn
                kf.number = i
                kf.type = _F.TYPE_STRING
                kf.label = _F.LABEL_OPTIONAL
                kf.json_name = kn
            f.type = _F.TYPE_MESSAGE
            f.type_name = full + "." + entry_name
            f.label = _F.LABEL_REPEATED
            continue
        f.label = _F.LABEL_REPEATED if label == "r" else _F.LABEL_OPTIONAL
        if ftype.startswith("msg:"):
            f.type = _F.TYPE_MESSAGE
            f.type_name = ftype[4:]
        elif ftype.startswith("enum:"):
            f.type = _F.TYPE_ENUM
            f.type_name = ftype[5:]
        else:
            f.type = _T[ftype]


def _build_api():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "api.proto"
    fdp.package = PKG
    fdp.syntax = "proto3"
    for en, vals in _ENUMS.items():
        ep = fdp.enum_type.add()
        ep.name = en
        for vn, vv in vals:
            v = ep.value.add()
            v.name = vn
            v.number = vv
    for name, fields, nested, enums in _MESSAGES:
        _fill_message(fdp.message_type.add(), name, fields, nested, enums, "." + PKG)
    for sname, methods in _SERVICES:
        sp = fdp.service.add()
        sp.name = sname
        for mname, req, rep in methods:
            m = sp.method.add()
            m.name = mname
            m.input_type = "." + PKG + "." + req
            m.output_type = "." + PKG + "." + rep
    return fdp


def _build_health():
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "health.proto"
    fdp.package = "grpc.health.v1"
    fdp.syntax = "proto3"
    req = fdp.message_type.add()
    req.name = "HealthCheckRequest"
    f = req.field.add()
    f.name, f.number, f.type, f.label = "service", 1, _F.TYPE_STRING, _F.LABEL_OPTIONAL
    rep = fdp.message_type.add()
    rep.name = "HealthCheckResponse"
    e = rep.enum_type.add()
    e.name = "ServingStatus"
    for vn, vv in (("UNKNOWN", 0), ("SERVING", 1), ("NOT_SERVING", 2)):
        v = e.value.add()
        v.name, v.number = vn, vv
    f = rep.field.add()
    f.name, f.number, f.type, f.label = "status", 1, _F.TYPE_ENUM, _F.LABEL_OPTIONAL
    f.type_name = ".grpc.health.v1.HealthCheckResponse.ServingStatus"
    sp = fdp.service.add()
    sp.name = "Health"
    m = sp.method.add()
    m.name, m.input_type, m.output_type = "Check", ".grpc.health.v1.HealthCheckRequest", \
        ".grpc.health.v1.HealthCheckResponse"
    return fdp


POOL = descriptor_pool.DescriptorPool()
FILE_DESCRIPTOR = POOL.Add(_build_api())
HEALTH_FILE_DESCRIPTOR = POOL.Add(_build_health())
DESCRIPTOR = POOL.FindFileByName("api.proto")


def _cls(full):
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(full))


class _EnumWrapper:
    def __init__(self, ed):
        self._ed = ed
        for v in ed.values:
            setattr(self, v.name, v.number)

    def Value(self, name):
        return self._ed.values_by_name[name].number

    def Name(self, number):
        return self._ed.values_by_number[number].name

    def keys(self):
        return [v.name for v in self._ed.values]

    def values(self):
        return [v.number for v in self._ed.values]

    def items(self):
        return [(v.name, v.number) for v in self._ed.values]


_g = globals()
for _name, *_ in _MESSAGES:
    _g[_name] = _cls(PKG + "." + _name)
for _en in _ENUMS:
    _w = _EnumWrapper(POOL.FindEnumTypeByName(PKG + "." + _en))
    _g[_en] = _w
    for _vn, _vv in _ENUMS[_en]:
        _g[_vn] = _vv

HealthCheckRequest = _cls("grpc.health.v1.HealthCheckRequest")
HealthCheckResponse = _cls("grpc.health.v1.HealthCheckResponse")

SERVICES = {s: [(m, PKG + "." + rq, PKG + "." + rp) for m, rq, rp in ms] for s, ms in _SERVICES}

# enum values nested in messages are reachable as in generated code:
#   api_pb2.TrialStatus.SUCCEEDED, api_pb2.TrialStatus.TrialConditionType.Value("FAILED")
