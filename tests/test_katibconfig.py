"""katib-config defaults and lookups: ports of the reference
``pkg/apis/config/v1beta1/defaults_test.go`` and
``pkg/util/v1beta1/katibconfig/config_test.go`` (same fakes and cases)."""
import copy

import pytest
import yaml

from katib_amd.api import katibconfig as KC
from katib_amd.controller.config import KatibConfig
from katib_amd.controller.manifest import ConfigMapStore

DEFAULT_RES = {"requests": {"cpu": KC.DEFAULT_CPU_REQUEST, "memory": KC.DEFAULT_MEM_REQUEST,
                            "ephemeral-storage": KC.DEFAULT_DISK_REQUEST},
               "limits": {"cpu": KC.DEFAULT_CPU_LIMIT, "memory": KC.DEFAULT_MEM_LIMIT,
                          "ephemeral-storage": KC.DEFAULT_DISK_LIMIT}}
CUSTOM_RES = {"requests": {"cpu": "25m", "memory": "200Mi", "ephemeral-storage": "550Mi"},
              "limits": {"cpu": "250m", "memory": "2Gi", "ephemeral-storage": "15Gi"}}


def fake_suggestion(name="test-suggestion", **kw):
    s = {"algorithmName": name, "image": "suggestion-image", "imagePullPolicy": KC.DEFAULT_IMAGE_PULL_POLICY,
         "resources": copy.deepcopy(DEFAULT_RES), "volumeMountPath": KC.DEFAULT_SUGGESTION_VOLUME_MOUNT_PATH,
         "persistentVolumeClaimSpec": {"accessModes": [KC.DEFAULT_SUGGESTION_VOLUME_ACCESS_MODE],
                                       "resources": {"requests": {"storage": KC.DEFAULT_SUGGESTION_VOLUME_STORAGE}}},
         "persistentVolumeSpec": {"persistentVolumeReclaimPolicy": "Delete"}}
    s.update(copy.deepcopy(kw))
    return s


def fake_early_stopping(name="test-early-stopping", **kw):
    s = {"algorithmName": name, "image": "early-stopping-image", "imagePullPolicy": KC.DEFAULT_IMAGE_PULL_POLICY,
         "resources": copy.deepcopy(DEFAULT_RES)}
    s.update(copy.deepcopy(kw))
    return s


def fake_collector(kind="testCollector", **kw):
    s = {"kind": kind, "image": "metrics-collector-image", "imagePullPolicy": KC.DEFAULT_IMAGE_PULL_POLICY,
         "resources": copy.deepcopy(DEFAULT_RES)}
    s.update(copy.deepcopy(kw))
    return s


# ---- defaults_test.go ------------------------------------------------------------------

@pytest.mark.parametrize("desc,config,want", [
    ("All parameters correctly are specified", fake_suggestion(imagePullPolicy="Always", resources=CUSTOM_RES),
     fake_suggestion(imagePullPolicy="Always", resources=CUSTOM_RES)),
    ("sets IfNotPresent to imagePullPolicy", fake_suggestion(imagePullPolicy=""), fake_suggestion()),
    ("sets resource.requests and resource.limits for the suggestion service", fake_suggestion(resources={}),
     fake_suggestion()),
    ("sets /opt/katib/data to volumeMountPath", fake_suggestion(volumeMountPath=""), fake_suggestion()),
    ("sets accessMode and resource.requests for PVC", fake_suggestion(persistentVolumeClaimSpec={}),
     fake_suggestion()),
    ("does not set Delete to persistentVolumeReclaimPolicy", fake_suggestion(persistentVolumeSpec={}),
     fake_suggestion(persistentVolumeSpec={})),
])
def test_set_suggestion_configs(desc, config, want):
    kc = KC.set_defaults({"runtime": {"suggestions": [config]}})
    assert kc["runtime"]["suggestions"] == [want]


@pytest.mark.parametrize("desc,config,want", [
    ("All parameters correctly are specified", fake_early_stopping(imagePullPolicy="IfNotPresent"),
     fake_early_stopping(imagePullPolicy="IfNotPresent")),
    ("sets IfNotPresent to imagePullPolicy", fake_early_stopping(imagePullPolicy=""), fake_early_stopping()),
])
def test_set_early_stopping_configs(desc, config, want):
    kc = KC.set_defaults({"runtime": {"earlyStoppings": [config]}})
    assert kc["runtime"]["earlyStoppings"] == [want]


NUKE = {"cpu": "-1", "memory": "-1", "ephemeral-storage": "-1"}


@pytest.mark.parametrize("desc,config,want", [
    ("All parameters correctly are specified", fake_collector(imagePullPolicy="Never"),
     fake_collector(imagePullPolicy="Never")),
    ("sets IfNotPresent to imagePullPolicy", fake_collector(imagePullPolicy=""), fake_collector()),
    ("nukes resource.requests and resource.limits for the metrics collector",
     fake_collector(resources={"requests": NUKE, "limits": NUKE}),
     fake_collector(resources={"requests": {}, "limits": {}})),
])
def test_set_metrics_collector_configs(desc, config, want):
    kc = KC.set_defaults({"runtime": {"metricsCollectors": [config]}})
    assert kc["runtime"]["metricsCollectors"] == [want]


FULL_CONTROLLER = {"experimentSuggestionName": "test", "metricsAddr": ":8081", "healthzAddr": ":18081",
                   "injectSecurityContext": True, "enableGRPCProbeInSuggestion": False,
                   "trialResources": ["Job.v1.batch", "TFJob.v1.kubeflow.org"], "webhookPort": 18443,
                   "enableLeaderElection": True, "leaderElectionID": "xyz0123"}
DEFAULT_CONTROLLER = {"experimentSuggestionName": KC.DEFAULT_EXPERIMENT_SUGGESTION_NAME,
                      "metricsAddr": KC.DEFAULT_METRICS_ADDR, "healthzAddr": KC.DEFAULT_HEALTHZ_ADDR,
                      "enableGRPCProbeInSuggestion": True, "trialResources": ["Job.v1.batch"],
                      "webhookPort": KC.DEFAULT_WEBHOOK_PORT, "leaderElectionID": KC.DEFAULT_LEADER_ELECTION_ID}


@pytest.mark.parametrize("desc,config,want", [
    ("All parameters correctly are specified", FULL_CONTROLLER, FULL_CONTROLLER),
    ("ControllerConfig is empty", {}, DEFAULT_CONTROLLER),
])
def test_set_controller_config(desc, config, want):
    kc = KC.set_defaults({"init": {"controller": copy.deepcopy(config)}})
    assert kc["init"]["controller"] == want


@pytest.mark.parametrize("desc,config,want", [
    ("All parameters correctly are specified",
     {"enable": True, "webhookServiceName": "test", "webhookSecretName": "katib-test"},
     {"enable": True, "webhookServiceName": "test", "webhookSecretName": "katib-test"}),
    ("CertGeneratorConfig is empty", {}, {}),
    ("Enable is true and serviceName is empty", {"enable": True},
     {"enable": True, "webhookServiceName": KC.DEFAULT_WEBHOOK_SERVICE_NAME,
      "webhookSecretName": KC.DEFAULT_WEBHOOK_SECRET_NAME}),
    ("cert-generator is forcefully enabled due to set webhookSecretName", {"webhookSecretName": "katib-test"},
     {"enable": True, "webhookServiceName": KC.DEFAULT_WEBHOOK_SERVICE_NAME, "webhookSecretName": "katib-test"}),
    ("cert-generator is forcefully enabled due to set webhookServiceName", {"webhookServiceName": "katib-test"},
     {"enable": True, "webhookServiceName": "katib-test", "webhookSecretName": KC.DEFAULT_WEBHOOK_SECRET_NAME}),
])
def test_set_cert_generator_config(desc, config, want):
    kc = KC.set_defaults({"init": {"certGenerator": copy.deepcopy(config)}})
    assert kc["init"]["certGenerator"] == want


@pytest.mark.parametrize("q,v", [("500m", 0.5), ("1Gi", 2 ** 30), ("100Mi", 100 * 2 ** 20), ("-1", -1), ("1e3", 1000),
                                 ("2k", 2000), (".5", 0.5), ("0", 0)])
def test_parse_quantity(q, v):
    assert float(KC.parse_quantity(q)) == v


def test_parse_quantity_rejects_garbage():
    with pytest.raises(KC.KatibConfigError):
        KC.parse_quantity("12 cores")


# ---- config_test.go ------------------------------------------------------------------

@pytest.mark.parametrize("desc,resources,want,err", [
    ("All GVKs are appropriate", ["Job.v1.batch", "TFJob.v1.kubeflow.org"],
     [("batch", "v1", "Job"), ("kubeflow.org", "v1", "TFJob")], None),
    ("TrialResources are empty", [], None, KC.ERR_TRIAL_RESOURCES_ARE_EMPTY),
    ("GVK with invalid schema", ["invalid;;invalid"], None, KC.ERR_INVALID_GVK_FORMAT),
])
def test_trial_resources_to_gvks(desc, resources, want, err):
    if err:
        with pytest.raises(KC.KatibConfigError, match=err):
            KC.trial_resources_to_gvks(resources)
    else:
        assert KC.trial_resources_to_gvks(resources) == want


def _store(cfg):
    if cfg is None:
        return ConfigMapStore()
    st = ConfigMapStore()
    st.put_manifest(KC.katib_config_map(cfg))
    return st


def _lookup_cases(key, fake, name, invalid):
    return [
        ("All parameters correctly are specified", {"runtime": {key: [fake]}}, name, fake),
        ("There is not katib-config.", None, name, None),
        ("There is not the %s field in katib-config configMap" % key, {}, name, None),
        ("There is not the AlgorithmName", {"runtime": {key: [fake]}}, invalid, None),
        ("Image filed is empty in katib-config configMap", {"runtime": {key: [dict(fake, image="")]}}, name, None),
    ]


@pytest.mark.parametrize("desc,cfg,name,want", _lookup_cases(
    "suggestions", fake_suggestion(imagePullPolicy="Always", resources=CUSTOM_RES), "test-suggestion",
    "invalid-algorithm-name"))
def test_get_suggestion_config_data(desc, cfg, name, want):
    if want is None:
        with pytest.raises(KC.KatibConfigError):
            KC.get_suggestion_config_data(name, _store(cfg))
    else:
        assert KC.get_suggestion_config_data(name, _store(cfg)) == want


@pytest.mark.parametrize("desc,cfg,name,want", _lookup_cases(
    "earlyStoppings", fake_early_stopping(), "test-early-stopping", "invalid-algorithm-name"))
def test_get_early_stopping_config_data(desc, cfg, name, want):
    if want is None:
        with pytest.raises(KC.KatibConfigError):
            KC.get_early_stopping_config_data(name, _store(cfg))
    else:
        assert KC.get_early_stopping_config_data(name, _store(cfg)) == want


@pytest.mark.parametrize("desc,cfg,name,want", _lookup_cases(
    "metricsCollectors", fake_collector(imagePullPolicy="Never"), "testCollector", "invalidCollector"))
def test_get_metrics_collector_config_data(desc, cfg, name, want):
    if want is None:
        with pytest.raises(KC.KatibConfigError):
            KC.get_metrics_collector_config_data(name, _store(cfg))
    else:
        assert KC.get_metrics_collector_config_data(name, _store(cfg)) == want


def test_suggestion_service_counts_as_image():
    """An in-process suggestion may name a service instead of an image."""
    cfg = {"runtime": {"suggestions": [{"algorithmName": "tpe", "service": "hyperopt"}]}}
    assert KC.get_suggestion_config_data("tpe", _store(cfg))["service"] == "hyperopt"


FULL_INIT = """
apiVersion: config.kubeflow.org/v1beta1
kind: KatibConfig
init:
  certGenerator:
    enable: true
    webhookServiceName: katib-test
    webhookSecretName: katib-test-secret
  controller:
    experimentSuggestionName: test
    metricsAddr: :8081
    healthzAddr: :18081
    injectSecurityContext: true
    enableGRPCProbeInSuggestion: false
    trialResources:
    - Job.v1.batch
    - TFJob.v1.kubeflow.org
    - PyTorchJob.v1.kubeflow.org
    - MPIJob.v1.kubeflow.org
    - XGBoostJob.v1.kubeflow.org
    - MXJob.v1.kubeflow.org
    webhookPort: 18443
    enableLeaderElection: true
    leaderElectionID: xyz0123
runtime:
  suggestions:
  - algorithmName: random
    image: docker.io/kubeflowkatib/suggestion-hyperopt:latest
"""


def test_get_init_config_data(tmp_path):
    assert KC.get_init_config_data("") == {"controller": DEFAULT_CONTROLLER, "certGenerator": {}}
    with pytest.raises(KC.KatibConfigError, match="failed to parse katib-config.yaml"):
        KC.get_init_config_data(str(tmp_path / "invalid"))
    p = tmp_path / "full.yaml"
    p.write_text(FULL_INIT)
    got = KC.get_init_config_data(str(p))
    assert got["certGenerator"] == {"enable": True, "webhookServiceName": "katib-test",
                                    "webhookSecretName": "katib-test-secret"}
    want = dict(FULL_CONTROLLER, trialResources=["Job.v1.batch", "TFJob.v1.kubeflow.org", "PyTorchJob.v1.kubeflow.org",
                                                 "MPIJob.v1.kubeflow.org", "XGBoostJob.v1.kubeflow.org",
                                                 "MXJob.v1.kubeflow.org"])
    assert got["controller"] == want


def test_scheduler_config_applies_reference_defaults():
    cfg = KatibConfig.from_dict(yaml.safe_load(FULL_INIT))
    assert cfg.suggestions["random"] == "hyperopt"
    s = cfg.raw["runtime"]["suggestions"][0]
    assert s["imagePullPolicy"] == "IfNotPresent" and s["resources"] == DEFAULT_RES
    with pytest.raises(KC.KatibConfigError, match="invalid GroupVersionKinds"):
        KatibConfig.from_dict({"init": {"controller": {"trialResources": ["bad"]}}})


def test_reference_install_config_loads():
    path = "/root/reference/manifests/v1beta1/installs/katib-standalone/katib-config.yaml"
    import os

    if not os.path.exists(path):
        pytest.skip("reference manifests not mounted")
    docs = [d for d in yaml.safe_load_all(open(path)) if d]
    text = docs[0]["data"][KC.KATIB_CONFIG_TAG] if docs[0].get("kind") == "ConfigMap" else yaml.safe_dump(docs[0])
    st = ConfigMapStore()
    st.put(KC.DEFAULT_KATIB_NAMESPACE, KC.KATIB_CONFIG_MAP_NAME, {KC.KATIB_CONFIG_TAG: text})
    for algo in ("random", "tpe", "grid", "hyperband", "bayesianoptimization", "cmaes", "enas", "darts", "pbt"):
        assert KC.get_suggestion_config_data(algo, st)["image"]
    assert KC.get_early_stopping_config_data("medianstop", st)["image"]
    for kind in ("StdOut", "File", "TensorFlowEvent"):
        assert KC.get_metrics_collector_config_data(kind, st)["resources"]["limits"]
