"""v1beta1 API: models, YAML round trip of the reference examples, defaults, validation
(reference validator_test.go / experiment_defaults)."""
import glob
import os

import pytest
import yaml

from katib_amd.api import constants as C
from katib_amd.api.defaults import set_default
from katib_amd.api.models import (V1beta1Experiment, V1beta1FeasibleSpace, V1beta1ParameterSpec,
                                  V1beta1ObjectiveSpec)
from katib_amd.api.validation import ValidationError, validate_experiment
from katib_amd.api.yaml_io import load_documents, load_experiment
from katib_amd.controller.manifest import ConfigMapStore, Generator

REF = "/root/reference/examples/v1beta1"
EXAMPLES = sorted(glob.glob(REF + "/hp-tuning/*.yaml") + glob.glob(REF + "/early-stopping/*.yaml")
                  + glob.glob(REF + "/nas/*.yaml") + glob.glob(REF + "/metrics-collector/*.yaml")
                  + glob.glob(REF + "/resume-experiment/*.yaml"))


def test_positional_feasible_space():
    fs = V1beta1FeasibleSpace(["a", "b"])  # search.py:64 calls it positionally
    assert fs.list == ["a", "b"] and fs.min is None


@pytest.mark.skipif(not EXAMPLES, reason="reference examples not mounted")
@pytest.mark.parametrize("path", EXAMPLES, ids=lambda p: os.path.relpath(p, REF))
def test_reference_examples_roundtrip_default_validate(path):
    with open(path) as f:
        text = f.read()
    objs, cms = load_documents(text)
    for e in objs:
        if not isinstance(e, V1beta1Experiment):
            continue
        raw = [d for d in yaml.safe_load_all(text) if d and d.get("kind") == "Experiment"][0]
        assert e.to_k8s()["spec"] == raw["spec"]
        set_default(e)
        gen = Generator(ConfigMapStore())
        for cm in cms:
            gen.configmaps.put_manifest(cm)
        if e.spec.trial_template.config_map is not None:
            continue  # ConfigMap lives in the reference install manifests
        try:
            validate_experiment(e, template_getter=gen.get_trial_template)
        except ValidationError as err:
            # simple-pbt.yaml sets maxFailedTrialCount(3) > maxTrialCount(2): the reference
            # webhook (validator.go:86-89) rejects it as well
            assert "maxFailedTrialCount should be less than or equal" in str(err), str(err)
        assert e.spec.parallel_trial_count is not None
        strategies = {s.name: s.value for s in e.spec.objective.metric_strategies}
        assert e.spec.objective.objective_metric_name in strategies


def _exp(**kw):
    e = load_experiment(os.path.join(os.path.dirname(__file__), "..", "examples", "hp-tuning",
                                     "random-quadratic.yaml"))
    for k, v in kw.items():
        setattr(e.spec, k, v)
    return set_default(e)


def test_defaults():
    e = load_experiment(os.path.join(os.path.dirname(__file__), "..", "examples", "hp-tuning",
                                     "random-quadratic.yaml"))
    e.spec.parallel_trial_count = None
    e.spec.objective.additional_metric_names = ["loss"]
    set_default(e)
    assert e.spec.parallel_trial_count == 3 and e.spec.resume_policy == "Never"
    assert [(s.name, s.value) for s in e.spec.objective.metric_strategies] == [("result", "max"), ("loss", "max")]
    assert e.spec.trial_template.success_condition == C.DEFAULT_JOB_SUCCESS_CONDITION
    assert e.spec.metrics_collector_spec.collector.kind == "StdOut"


@pytest.mark.parametrize("mut,msg", [
    (dict(max_trial_count=0), "spec.maxTrialCount must be greater than 0"),
    (dict(parallel_trial_count=0), "spec.parallelTrialCount must be greater than 0"),
    (dict(max_failed_trial_count=-1), "spec.maxFailedTrialCount should not be less than 0"),
    (dict(max_failed_trial_count=20), "spec.maxFailedTrialCount should be less than or equal to spec.maxTrialCount"),
    (dict(parallel_trial_count=20), "spec.paralelTrialCount should be less than or equal to spec.maxTrialCount"),
    (dict(resume_policy="Sometimes"), "invalid ResumePolicyType Sometimes"),
])
def test_validation_counts(mut, msg):
    with pytest.raises(ValidationError, match=msg.replace(".", r"\.")):
        validate_experiment(_exp(**mut))


def test_validation_objective_and_params():
    e = _exp()
    e.spec.objective.type = "up"
    with pytest.raises(ValidationError, match="spec.objective.type must be minimize or maximize"):
        validate_experiment(e)
    e = _exp()
    e.spec.objective.additional_metric_names = ["result"]
    with pytest.raises(ValidationError, match="should not contain"):
        validate_experiment(e)
    e = _exp()
    e.spec.parameters.append(V1beta1ParameterSpec(name="c", parameter_type="categorical",
                                                  feasible_space=V1beta1FeasibleSpace(list=["a"], max="3")))
    with pytest.raises(ValidationError, match=r"feasibleSpace \.max, \.min and \.step is not supported"):
        validate_experiment(e)
    e = _exp()
    e.spec.algorithm.algorithm_name = "nope"
    with pytest.raises(ValidationError, match="unable to get Suggestion config data"):
        validate_experiment(e, suggestion_algorithms={"random"})


def test_validation_trial_template():
    e = _exp()
    e.spec.trial_template.trial_parameters[0].reference = "zzz"
    with pytest.raises(ValidationError, match="parameter reference zzz does not exist"):
        validate_experiment(e)
    e = _exp()
    e.spec.trial_template.trial_parameters.pop()
    with pytest.raises(ValidationError, match="not found in spec.trialParameters"):
        validate_experiment(e)
    e = _exp()
    e.spec.trial_template.trial_spec["metadata"] = {"name": "x"}
    with pytest.raises(ValidationError, match="must be omitted"):
        validate_experiment(e)


def test_validation_edit_rules():
    old = _exp()
    old.metadata.name = "random-quadratic"
    new = old.deepcopy()
    new.spec.max_trial_count = 20
    validate_experiment(new, old)
    new.spec.objective.goal = 1.0
    with pytest.raises(ValidationError, match="only spec.parallelTrialCount"):
        validate_experiment(new, old)


def test_metrics_collector_validation():
    from katib_amd.api.models import V1beta1CollectorSpec, V1beta1MetricsCollectorSpec, V1beta1SourceSpec, \
        V1beta1FilterSpec

    e = _exp()
    e.spec.metrics_collector_spec = V1beta1MetricsCollectorSpec(collector=V1beta1CollectorSpec(kind="File"))
    set_default(e)
    validate_experiment(e)
    e.spec.metrics_collector_spec.source.filter = V1beta1FilterSpec(metrics_format=["(only-one)"])
    with pytest.raises(ValidationError, match="two top subexpressions are required"):
        validate_experiment(e)
    e.spec.metrics_collector_spec.collector.kind = "Bogus"
    with pytest.raises(ValidationError, match="invalid metrics collector kind"):
        validate_experiment(e)


def test_manifest_generator_meta_refs():
    e = _exp()
    e.spec.trial_template.trial_parameters.append(
        type(e.spec.trial_template.trial_parameters[0])(name="trialName", reference="${trialSpec.Name}"))
    e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]["command"].append(
        "--name=${trialParameters.trialName}")
    from katib_amd.api.models import V1beta1ParameterAssignment as PA

    spec = Generator(ConfigMapStore()).run_spec(e, "t-1", "ns", [PA(name="a", value="1"), PA(name="b", value="2")])
    cmd = spec["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[-1] == "--name=t-1" and "a=1; b=2" in cmd[2]
    assert spec["metadata"] == {"name": "t-1", "namespace": "ns"}
    with pytest.raises(ValueError, match="Number of TrialAssignment"):
        Generator(ConfigMapStore()).run_spec(e, "t", "ns", [PA(name="a", value="1"), PA(name="b", value="2"),
                                                            PA(name="c", value="3")])
