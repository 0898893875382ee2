"""katib-config.yaml: schema defaults and lookups.

Defaulting follows ``pkg/apis/config/v1beta1/defaults.go:61-270`` (controller and
cert-generator init config; image pull policy, resource requests/limits with the
``-1`` "nuke" convention, suggestion volume settings) and the getters follow
``pkg/util/v1beta1/katibconfig/config.go:44-175`` (error cases included).

Configs are handled in their manifest form (camelCase dicts, quantities as strings)
so a user's existing katib-config.yaml is read unchanged. On the node-local MI355X
scheduler a suggestion runs in-process, so an entry may name a ``service`` instead
of a container ``image``; either one satisfies the "image is required" rule.
"""

from __future__ import annotations

import copy
import os
import re
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

import yaml

KATIB_CONFIG_MAP_NAME = "katib-config"
KATIB_CONFIG_TAG = "katib-config.yaml"
DEFAULT_KATIB_NAMESPACE = "kubeflow"

DEFAULT_EXPERIMENT_SUGGESTION_NAME = "default"
DEFAULT_METRICS_ADDR = ":8080"
DEFAULT_HEALTHZ_ADDR = ":18080"
DEFAULT_LEADER_ELECTION_ID = "3fbc96e9.katib.kubeflow.org"
DEFAULT_SUGGESTION_VOLUME_MOUNT_PATH = "/opt/katib/data"
DEFAULT_SUGGESTION_VOLUME_ACCESS_MODE = "ReadWriteOnce"
DEFAULT_SUGGESTION_VOLUME_STORAGE = "1Gi"
DEFAULT_IMAGE_PULL_POLICY = "IfNotPresent"
DEFAULT_CPU_LIMIT = "500m"
DEFAULT_CPU_REQUEST = "50m"
DEFAULT_MEM_LIMIT = "100Mi"
DEFAULT_MEM_REQUEST = "10Mi"
DEFAULT_DISK_LIMIT = "5Gi"
DEFAULT_DISK_REQUEST = "500Mi"
DEFAULT_WEBHOOK_SERVICE_NAME = "katib-controller"
DEFAULT_WEBHOOK_SECRET_NAME = "katib-webhook-cert"
DEFAULT_ENABLE_GRPC_PROBE_IN_SUGGESTION = True
DEFAULT_WEBHOOK_PORT = 8443
DEFAULT_TRIAL_RESOURCES = ["Job.v1.batch"]
PULL_POLICIES = ("Always", "IfNotPresent", "Never")


class KatibConfigError(ValueError):
    pass


ERR_KATIB_CONFIG_NIL = "failed to parse katib-config.yaml in ConfigMap: %s" % KATIB_CONFIG_MAP_NAME
ERR_INVALID_GVK_FORMAT = "invalid GroupVersionKinds"
ERR_TRIAL_RESOURCES_ARE_EMPTY = "trialResources are empty"

_QTY = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+))(?:([eE][+-]?\d+)|(Ki|Mi|Gi|Ti|Pi|Ei|n|u|m|k|M|G|T|P|E))?$")
_SUFFIX = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
           "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
           "P": Fraction(10 ** 15), "E": Fraction(10 ** 18), "Ki": Fraction(2 ** 10), "Mi": Fraction(2 ** 20),
           "Gi": Fraction(2 ** 30), "Ti": Fraction(2 ** 40), "Pi": Fraction(2 ** 50), "Ei": Fraction(2 ** 60)}


def parse_quantity(q) -> Fraction:
    """resource.ParseQuantity: exact value of a Kubernetes quantity string."""
    if isinstance(q, (int, float)):
        return Fraction(q)
    m = _QTY.match(str(q).strip())
    if not m:
        raise KatibConfigError("quantities must match the regular expression '%s': %r" % (_QTY.pattern, q))
    v = Fraction(m.group(1))
    if m.group(2):
        v *= Fraction(10) ** int(m.group(2)[1:])
    return v * _SUFFIX[m.group(3) or ""]


def _qty(q) -> Fraction:
    return Fraction(0) if q in (None, "") else parse_quantity(q)


def set_image_pull_policy(policy: Optional[str]) -> str:
    return policy if policy in PULL_POLICIES else DEFAULT_IMAGE_PULL_POLICY


def set_resource_requirements(res: Optional[Dict]) -> Dict:
    """setResourceRequirements (defaults.go:194-270): zero entries take the defaults,
    negative ones are removed ("nuke")."""
    res = dict(res or {})
    req = dict(res.get("requests") or {})
    lim = dict(res.get("limits") or {})
    for store, defaults in ((req, (("cpu", DEFAULT_CPU_REQUEST), ("memory", DEFAULT_MEM_REQUEST),
                                   ("ephemeral-storage", DEFAULT_DISK_REQUEST))),
                            (lim, (("cpu", DEFAULT_CPU_LIMIT), ("memory", DEFAULT_MEM_LIMIT),
                                   ("ephemeral-storage", DEFAULT_DISK_LIMIT)))):
        for key, dflt in defaults:
            v = _qty(store.get(key))
            if v == 0:
                store[key] = dflt
            elif v < 0:
                del store[key]
    res["requests"], res["limits"] = req, lim
    return res


def set_controller_config(c: Dict) -> Dict:
    if not c.get("experimentSuggestionName"):
        c["experimentSuggestionName"] = DEFAULT_EXPERIMENT_SUGGESTION_NAME
    if not c.get("metricsAddr"):
        c["metricsAddr"] = DEFAULT_METRICS_ADDR
    if not c.get("healthzAddr"):
        c["healthzAddr"] = DEFAULT_HEALTHZ_ADDR
    if c.get("enableGRPCProbeInSuggestion") is None:
        c["enableGRPCProbeInSuggestion"] = DEFAULT_ENABLE_GRPC_PROBE_IN_SUGGESTION
    if not c.get("trialResources"):
        c["trialResources"] = list(DEFAULT_TRIAL_RESOURCES)
    if c.get("webhookPort") is None:
        c["webhookPort"] = DEFAULT_WEBHOOK_PORT
    if not c.get("leaderElectionID"):
        c["leaderElectionID"] = DEFAULT_LEADER_ELECTION_ID
    return c


def set_cert_generator_config(c: Dict) -> Dict:
    if c.get("webhookServiceName") or c.get("webhookSecretName"):
        c["enable"] = True
    if c.get("enable") and not c.get("webhookServiceName"):
        c["webhookServiceName"] = DEFAULT_WEBHOOK_SERVICE_NAME
    if c.get("enable") and not c.get("webhookSecretName"):
        c["webhookSecretName"] = DEFAULT_WEBHOOK_SECRET_NAME
    return c


def set_suggestion_config(s: Dict) -> Dict:
    s["imagePullPolicy"] = set_image_pull_policy(s.get("imagePullPolicy"))
    s["resources"] = set_resource_requirements(s.get("resources"))
    if not s.get("volumeMountPath"):
        s["volumeMountPath"] = DEFAULT_SUGGESTION_VOLUME_MOUNT_PATH
    pvc = dict(s.get("persistentVolumeClaimSpec") or {})
    if not pvc.get("accessModes"):
        pvc["accessModes"] = [DEFAULT_SUGGESTION_VOLUME_ACCESS_MODE]
    pres = dict(pvc.get("resources") or {})
    if not pres.get("requests"):
        pres["requests"] = {"storage": DEFAULT_SUGGESTION_VOLUME_STORAGE}
    pvc["resources"] = pres
    s["persistentVolumeClaimSpec"] = pvc
    if s.get("persistentVolumeSpec"):  # only an explicitly configured PV gets reclaimPolicy Delete
        s["persistentVolumeSpec"] = dict(s["persistentVolumeSpec"], persistentVolumeReclaimPolicy="Delete")
    return s


def set_collector_config(m: Dict) -> Dict:
    """Early-stopping and metrics-collector entries: pull policy and resources."""
    m["imagePullPolicy"] = set_image_pull_policy(m.get("imagePullPolicy"))
    m["resources"] = set_resource_requirements(m.get("resources"))
    return m


def set_defaults(cfg: Optional[Dict]) -> Optional[Dict]:
    """SetDefaults_KatibConfig (defaults.go:61-67); mutates and returns ``cfg``."""
    if cfg is None:
        return None
    init = cfg.setdefault("init", {}) or {}
    cfg["init"] = init
    init["controller"] = set_controller_config(dict(init.get("controller") or {}))
    init["certGenerator"] = set_cert_generator_config(dict(init.get("certGenerator") or {}))
    rt = cfg.get("runtime") or {}
    cfg["runtime"] = rt
    for key, fn in (("suggestions", set_suggestion_config), ("metricsCollectors", set_collector_config),
                    ("earlyStoppings", set_collector_config)):
        if rt.get(key):
            rt[key] = [fn(dict(e)) for e in rt[key]]
    return cfg


def trial_resources_to_gvks(resources: List[str]) -> List[Tuple[str, str, str]]:
    """TrialResourcesToGVKs (config.go:44-57): ``Kind.version.group`` -> (group, version, kind)."""
    if not resources:
        raise KatibConfigError(ERR_TRIAL_RESOURCES_ARE_EMPTY)
    out = []
    for r in resources:
        if r.count(".") < 2:  # schema.ParseKindArg needs Kind.version.group
            raise KatibConfigError(ERR_INVALID_GVK_FORMAT)
        kind, version, group = r.split(".", 2)
        out.append((group, version, kind))
    return out


def _decode(text: str) -> Dict:
    try:
        cfg = yaml.safe_load(text) or {}
    except yaml.YAMLError as e:
        raise KatibConfigError("%s: %s" % (ERR_KATIB_CONFIG_NIL, e))
    if not isinstance(cfg, dict):
        raise KatibConfigError("%s: not a mapping" % ERR_KATIB_CONFIG_NIL)
    return set_defaults(cfg)


def from_config_map(configmaps) -> Dict:
    """fromConfigMap (config.go:162-175); ``configmaps`` is a ConfigMapStore-like
    object (``get(namespace, name) -> data``)."""
    if configmaps is None:
        raise KatibConfigError('configmaps "%s" not found' % KATIB_CONFIG_MAP_NAME)
    try:
        data = configmaps.get(DEFAULT_KATIB_NAMESPACE, KATIB_CONFIG_MAP_NAME)
    except KeyError as e:
        raise KatibConfigError(str(e).strip("'\""))
    if KATIB_CONFIG_TAG not in data:
        raise KatibConfigError("failed to find katib-config.yaml in ConfigMap: %s" % KATIB_CONFIG_MAP_NAME)
    return _decode(data[KATIB_CONFIG_TAG])


def _has_image(entry: Dict) -> bool:
    return bool(str(entry.get("image") or "").strip() or str(entry.get("service") or "").strip())


def _find(entries, key, value):
    hit = None
    for e in entries or []:
        if e.get(key) == value:
            hit = e  # last match wins, as the reference loop
    return hit


def get_suggestion_config_data(algorithm: str, configmaps) -> Dict:
    cfg = from_config_map(configmaps)
    s = _find(cfg["runtime"].get("suggestions"), "algorithmName", algorithm)
    if s is None:
        raise KatibConfigError("failed to find suggestion config for algorithm: %s in ConfigMap: %s"
                               % (algorithm, KATIB_CONFIG_MAP_NAME))
    if not _has_image(s):
        raise KatibConfigError("required value for image configuration of algorithm name: %s" % algorithm)
    return s


def get_early_stopping_config_data(algorithm: str, configmaps) -> Dict:
    cfg = from_config_map(configmaps)
    s = _find(cfg["runtime"].get("earlyStoppings"), "algorithmName", algorithm)
    if s is None:
        raise KatibConfigError("failed to find early stopping config for algorithm: %s in ConfigMap: %s"
                               % (algorithm, KATIB_CONFIG_MAP_NAME))
    if not _has_image(s):
        raise KatibConfigError("required value for image configuration of algorithm name: %s" % algorithm)
    return s


def get_metrics_collector_config_data(kind: str, configmaps) -> Dict:
    cfg = from_config_map(configmaps)
    s = _find(cfg["runtime"].get("metricsCollectors"), "kind", kind)
    if s is None:
        raise KatibConfigError("failed to find metrics collector config for kind: %s in ConfigMap: %s"
                               % (kind, KATIB_CONFIG_MAP_NAME))
    if not _has_image(s):
        raise KatibConfigError("required value for image configuration of metrics collector kind: %s" % kind)
    return s


def get_init_config_data(path: str) -> Dict:
    """GetInitConfigData (config.go:140-147): defaulted ``init`` section of the file
    (all defaults for an empty path)."""
    if not path:
        return set_defaults({})["init"]
    try:
        with open(path) as f:
            text = f.read()
    except OSError as e:
        raise KatibConfigError("%s: %s" % (ERR_KATIB_CONFIG_NIL, e))
    return _decode(text)["init"]


def katib_config_map(cfg: Optional[Dict]) -> Dict:
    """The ``katib-config`` ConfigMap manifest holding ``cfg`` (as the reference installs it)."""
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": KATIB_CONFIG_MAP_NAME, "namespace": DEFAULT_KATIB_NAMESPACE},
            "data": {KATIB_CONFIG_TAG: yaml.safe_dump(copy.deepcopy(cfg or {}))}}


def load_file(path: str) -> Dict:
    if not os.path.exists(path):
        raise KatibConfigError("%s: %s not found" % (ERR_KATIB_CONFIG_NIL, path))
    with open(path) as f:
        return _decode(f.read())
