"""OpenAPI (Swagger 2.0) document of the v1beta1 API, generated from the model table.

The reference generates ``pkg/apis/v1beta1/swagger.json`` from its Go types
(``hack/swagger/main.go:1-84`` over ``pkg/apis/v1beta1/openapi_generated.go``) and the Python
SDK models from that document (``hack/gen-python-sdk/gen-sdk.sh``). Here the direction is
reversed: the declarative model table of :mod:`katib_amd.api.models` (which already is the
SDK model set, one class per definition) is the single source, and this module renders the
Swagger document from it with the reference's definition names (``v1beta1.X``; the trial
and suggestion types under ``.v1beta1.X``, as the reference's generator emits them), wire
(camelCase) property names and type mapping:

* ``str`` -> ``string``, ``int`` -> ``integer`` (int32), ``bool`` -> ``boolean``,
* ``datetime`` -> ``$ref v1.Time``, ``object`` -> free-form object,
* ``list[X]`` -> ``array`` of X, ``dict(str, str)`` -> ``additionalProperties: string``,
* model types -> ``$ref`` to their definition.

``python -m katib_amd openapi`` prints it; the HTTP API serves it at ``/openapi/v2``.
"""

from __future__ import annotations

import json
import re
from typing import Dict

from . import models as M

# definitions the reference's generator emits with a leading dot (trials / suggestions packages)
_DOTTED = {"Suggestion", "SuggestionCondition", "SuggestionList", "SuggestionSpec", "SuggestionStatus", "Trial",
           "TrialAssignment", "TrialCondition", "TrialList", "TrialSpec", "TrialStatus"}
_K8S = {"V1ObjectMeta": "v1.ObjectMeta", "V1HTTPGetAction": "v1.HTTPGetAction"}


def definition_name(model: str) -> str:
    if model in _K8S:
        return _K8S[model]
    short = model[len("V1beta1"):]
    return (".v1beta1." if short in _DOTTED else "v1beta1.") + short


def _schema(type_str: str) -> Dict:
    if type_str == "str":
        return {"type": "string"}
    if type_str == "int":
        return {"type": "integer", "format": "int32"}
    if type_str == "bool":
        return {"type": "boolean"}
    if type_str == "float":
        return {"type": "number", "format": "double"}
    if type_str == "datetime":
        return {"$ref": "#/definitions/v1.Time"}
    if type_str == "object":
        return {"type": "object"}
    m = re.fullmatch(r"list\[(.+)\]", type_str)
    if m:
        return {"type": "array", "items": _schema(m.group(1))}
    m = re.fullmatch(r"dict\((\w+), (.+)\)", type_str)
    if m:
        return {"type": "object", "additionalProperties": _schema(m.group(2))}
    if type_str in M.MODEL_REGISTRY:
        return {"$ref": "#/definitions/" + definition_name(type_str)}
    raise ValueError("no OpenAPI mapping for model type %r" % type_str)


def document(include_k8s: bool = False) -> Dict:
    """The Swagger 2.0 document (``info`` as in the reference's ``swagger.json``)."""
    defs = {}
    for name, cls in M.MODEL_REGISTRY.items():
        if name in _K8S and not include_k8s:
            continue
        props = {}
        for attr, t in cls.openapi_types.items():
            props[cls.attribute_map[attr]] = _schema(t)
        defs[definition_name(name)] = {"type": "object", "properties": dict(sorted(props.items())),
                                       "description": "%s (katib_amd.api.models.%s)" % (definition_name(name), name)}
    if include_k8s:
        defs["v1.Time"] = {"type": "string", "format": "date-time"}
    return {"swagger": "2.0",
            "info": {"title": "Katib", "description": "Swagger description for Katib", "version": "v1beta1-0.1"},
            "paths": {}, "definitions": dict(sorted(defs.items()))}


def dumps(indent: int = 2, include_k8s: bool = False) -> str:
    return json.dumps(document(include_k8s), indent=indent, sort_keys=False)
