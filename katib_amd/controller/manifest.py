"""Trial-template rendering: the manifest generator
(reference ``pkg/controller.v1beta1/experiment/manifest/generator.go:37-215``).

``${trialParameters.X}`` placeholders resolve either to a parameter assignment
(``reference`` = parameter name) or to trial metadata
(``${trialSpec.Name|Namespace|Kind|APIVersion|Labels[k]|Annotations[k]}``). The
template is serialised to JSON, substituted by the native renderer and parsed
back, then ``metadata.name/namespace`` are set to the trial's.
"""

from __future__ import annotations

import json
import re
from typing import Dict, List, Optional, Tuple

import yaml

from ..api import constants as C
from .. import native

_META_RE = re.compile(C.TRIAL_TEMPLATE_META_REPLACE_REGEX)
_META_PARSE_RE = re.compile(C.TRIAL_TEMPLATE_META_PARSE_REGEX)


class ConfigMapStore:
    """Stand-in for ConfigMaps holding trial templates (label
    ``katib.kubeflow.org/component=trial-templates``)."""

    def __init__(self):
        self._maps: Dict[Tuple[str, str], Dict] = {}

    def put(self, namespace: str, name: str, data: Dict[str, str], labels: Optional[Dict[str, str]] = None):
        self._maps[(namespace, name)] = {"data": dict(data), "labels": dict(labels or {})}

    def put_manifest(self, doc: Dict):
        md = doc.get("metadata", {})
        self.put(md.get("namespace", "default"), md["name"], doc.get("data", {}), md.get("labels"))

    def get(self, namespace: str, name: str) -> Dict[str, str]:
        if (namespace, name) not in self._maps:
            raise KeyError("configmaps \"%s\" not found" % name)
        return self._maps[(namespace, name)]["data"]

    def delete(self, namespace: str, name: str):
        self._maps.pop((namespace, name), None)

    def list(self, label_selector: Optional[Dict[str, str]] = None):
        out = []
        for (ns, name), v in self._maps.items():
            if label_selector and any(v["labels"].get(k) != val for k, val in label_selector.items()):
                continue
            out.append((ns, name, v["data"]))
        return out

    def trial_templates(self):
        return self.list({C.LABEL_TRIAL_TEMPLATE_CONFIGMAP_NAME: C.LABEL_TRIAL_TEMPLATE_CONFIGMAP_VALUE})


def parse_unstructured(s: str) -> Dict:
    try:
        return json.loads(s)
    except ValueError:
        return yaml.safe_load(s)


class Generator:
    def __init__(self, configmaps: ConfigMapStore):
        self.configmaps = configmaps

    def get_trial_template(self, experiment) -> str:
        src = experiment.spec.trial_template
        if src.trial_spec is not None:
            return json.dumps(src.trial_spec)
        cm = src.config_map
        data = self.configmaps.get(cm.config_map_namespace, cm.config_map_name)
        if cm.template_path not in data:
            raise KeyError("TemplatePath: %s not found in configMap: %s" % (cm.template_path, data))
        return data[cm.template_path]

    def apply_parameters(self, experiment, trial_name: str, trial_namespace: str, assignments) -> str:
        tpl = self.get_trial_template(experiment)
        trial_spec = experiment.spec.trial_template.trial_spec
        if trial_spec is None:
            trial_spec = parse_unstructured(tpl)
        amap = {a.name: a.value for a in assignments}
        values: Dict[str, str] = {}
        non_meta = 0
        md = trial_spec.get("metadata") or {}
        for p in experiment.spec.trial_template.trial_parameters or []:
            m = _META_RE.search(p.reference)
            if not m:
                if p.reference in amap:
                    values[p.name] = amap[p.reference]
                    non_meta += 1
                    continue
                raise ValueError("Unable to find parameter: %s in parameter assignment %s" % (p.reference, amap))
            key, idx = m.group(1), None
            sub = _META_PARSE_RE.search(key)
            if sub:
                key, idx = sub.group(1), sub.group(2)
            if key == "Name":
                values[p.name] = trial_name
            elif key == "Namespace":
                values[p.name] = trial_namespace
            elif key == "Kind":
                values[p.name] = trial_spec.get("kind", "")
            elif key == "APIVersion":
                values[p.name] = trial_spec.get("apiVersion", "")
            elif key == "Annotations":
                ann = md.get("annotations") or {}
                if idx not in ann:
                    raise ValueError("illegal reference of trial metadata: %s; failed to fetch Annotation: %s"
                                     % (p.reference, idx))
                values[p.name] = ann[idx]
            elif key == "Labels":
                lab = md.get("labels") or {}
                if idx not in lab:
                    raise ValueError("illegal reference of trial metadata: %s; failed to fetch Label: %s"
                                     % (p.reference, idx))
                values[p.name] = lab[idx]
            else:
                raise ValueError("illegal reference of trial metadata: %s" % p.reference)
        if len(list(assignments)) != non_meta:
            raise ValueError("Number of TrialAssignment: %d != number of nonMetaTrialParameters in TrialSpec: %d"
                             % (len(list(assignments)), non_meta))
        # raw textual replacement, like strings.Replace in the reference (values such as the
        # DARTS/ENAS JSON strings already had their double quotes swapped for single quotes)
        return native.load().render_template(tpl, {k: str(v) for k, v in values.items()})

    def run_spec(self, experiment, trial_name: str, trial_namespace: str, assignments) -> Dict:
        rendered = self.apply_parameters(experiment, trial_name, trial_namespace, assignments)
        spec = parse_unstructured(rendered)
        spec.setdefault("metadata", {})
        spec["metadata"]["name"] = trial_name
        spec["metadata"]["namespace"] = trial_namespace
        return spec
