"""Experiment YAML / JSON (de)serialisation.

Accepts the same documents as ``kubectl apply -f`` on the reference examples
(``examples/v1beta1/**``): ``apiVersion: kubeflow.org/v1beta1``, ``kind:
Experiment`` with the camelCase CRD fields. Multi-document files are supported;
ConfigMaps in the same file are returned separately (trial-template ConfigMaps).
"""

from __future__ import annotations

import json
from typing import Dict, List, Tuple

import yaml

from . import constants as C
from .models import V1beta1Experiment, V1beta1Suggestion, V1beta1Trial, V1ObjectMeta

_KINDS = {C.KIND_EXPERIMENT: V1beta1Experiment, C.KIND_TRIAL: V1beta1Trial, C.KIND_SUGGESTION: V1beta1Suggestion}


def load_documents(text: str) -> Tuple[List, List[Dict]]:
    objs, cms = [], []
    for doc in yaml.safe_load_all(text):
        if not doc:
            continue
        kind = doc.get("kind")
        if kind == "ConfigMap":
            cms.append(doc)
            continue
        cls = _KINDS.get(kind)
        if cls is None:
            raise ValueError("unsupported kind %r" % kind)
        objs.append(cls.from_k8s(doc))
    return objs, cms


def load_experiment(path_or_text: str) -> V1beta1Experiment:
    text = path_or_text
    if "\n" not in path_or_text and not path_or_text.lstrip().startswith("{"):
        with open(path_or_text) as f:
            text = f.read()
    objs, _ = load_documents(text)
    exps = [o for o in objs if isinstance(o, V1beta1Experiment)]
    if not exps:
        raise ValueError("no Experiment document found")
    e = exps[0]
    if e.metadata is None:
        e.metadata = V1ObjectMeta()
    return e


def dump_yaml(obj) -> str:
    return yaml.safe_dump(obj.to_k8s(), sort_keys=False)


def dump_json(obj) -> str:
    return json.dumps(obj.to_k8s(), indent=2)
