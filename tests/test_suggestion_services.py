"""Suggestion / early-stopping service unit tests, mirroring the reference's Python unit tier
(reference test/unit/v1beta1/{suggestion,earlystopping,metricscollector}/*.py): the same
request fixtures go through our servicers, and the reply counts, gRPC status codes and
validation messages are checked.

The reference drives each servicer through ``grpc_testing`` (not installed here); the
servicers take ``(request, context)`` exactly like gRPC handlers, so a recording context
stands in for it. ``tests/test_cli.py::test_suggestion_server_grpc`` covers the real
gRPC server path.
"""
import json
import os

import grpc
import pytest

from katib_amd.rpc import api_pb2 as api


class Ctx:
    """Records what a gRPC handler reports (grpc.ServicerContext subset)."""

    def __init__(self):
        self.code = grpc.StatusCode.OK
        self.details = ""

    def set_code(self, code):
        self.code = code

    def set_details(self, details):
        self.details = details


def call(method, request):
    ctx = Ctx()
    reply = method(request, ctx)
    return reply, ctx.code, ctx.details


def validate(service, spec):
    return call(service.ValidateAlgorithmSettings,
                api.ValidateAlgorithmSettingsRequest(experiment=api.Experiment(name="validation-test", spec=spec)))


def P(name, ptype, **fs):
    return api.ParameterSpec(name=name, parameter_type=ptype, feasible_space=api.FeasibleSpace(**fs))


HP_PARAMS = [P("param-1", api.INT, max="5", min="1", list=[]),
             P("param-2", api.CATEGORICAL, list=["cat1", "cat2", "cat3"]),
             P("param-3", api.DISCRETE, list=["3", "2", "6"]),
             P("param-4", api.DOUBLE, max="5", min="1", list=[])]


def hp_trials(values=(("2", "cat1", "2", "3.44", "435", "5643"), ("3", "cat2", "6", "4.44", "123", "3028")),
              metric="metric-2", names=("test-asfjh", "test-234hs"), assignments=None, cond=api.TrialStatus.SUCCEEDED):
    out = []
    for i, (v, n) in enumerate(zip(values, names)):
        pas = assignments[i] if assignments is not None else [
            api.ParameterAssignment(name="param-%d" % (k + 1), value=v[k]) for k in range(4)]
        out.append(api.Trial(
            name=n,
            spec=api.TrialSpec(objective=api.ObjectiveSpec(type=api.MAXIMIZE, objective_metric_name=metric, goal=0.9),
                               parameter_assignments=api.TrialSpec.ParameterAssignments(assignments=pas)),
            status=api.TrialStatus(condition=cond, observation=api.Observation(metrics=[
                api.Metric(name="metric-1", value=v[4]), api.Metric(name="metric-2", value=v[5])]))))
    return out


def hp_experiment(algorithm, settings, params=HP_PARAMS, max_trial_count=0):
    return api.Experiment(name="test", spec=api.ExperimentSpec(
        algorithm=api.AlgorithmSpec(algorithm_name=algorithm, algorithm_settings=[
            api.AlgorithmSetting(name=k, value=v) for k, v in settings.items()]),
        objective=api.ObjectiveSpec(type=api.MAXIMIZE, goal=0.9, objective_metric_name="metric-2"),
        max_trial_count=max_trial_count,
        parameter_specs=api.ExperimentSpec.ParameterSpecs(parameters=params)))


# ------------------------------------------------------------------------------------ hyperopt
def test_hyperopt_get_suggestion():
    """test_hyperopt_service.py:36-202: TPE with two completed trials, 2 new assignments."""
    from katib_amd.algorithms.hpo import HyperoptService

    exp = hp_experiment("tpe", {"random_state": "10", "gamma": "0.25", "prior_weight": "1.0",
                                "n_EI_candidates": "24"})
    reply, code, _ = call(HyperoptService().GetSuggestions,
                          api.GetSuggestionsRequest(experiment=exp, trials=hp_trials(), current_request_number=2))
    assert code == grpc.StatusCode.OK
    assert len(reply.parameter_assignments) == 2
    for pa in reply.parameter_assignments:
        vals = {a.name: a.value for a in pa.assignments}
        assert 1 <= int(vals["param-1"]) <= 5 and vals["param-2"] in ("cat1", "cat2", "cat3")
        assert vals["param-3"] in ("3", "2", "6") and 1.0 <= float(vals["param-4"]) <= 5.0


@pytest.mark.parametrize("algorithm,settings,details", [
    ("tpe", {"random_state": "10", "gamma": "0.25", "prior_weight": "1.0", "n_EI_candidates": "24"}, None),
    ("unknown", {}, "unknown algorithm name unknown"),
    ("random", {"unknown_conf": "1111"}, "unknown setting unknown_conf for algorithm random"),
    ("tpe", {"gamma": "1.5"}, "gamma should be in the range of (0, 1)"),
    ("tpe", {"n_EI_candidates": "0"}, "n_EI_candidates should be great than zero"),
    ("tpe", {"random_state": "-1"}, "random_state should be great or equal than zero"),
    ("tpe", {"prior_weight": "aaa"}, "failed to validate prior_weight(aaa)"),
])
def test_hyperopt_validate_algorithm_settings(algorithm, settings, details):
    """test_hyperopt_service.py:204-313 (same settings, codes and messages)."""
    from katib_amd.algorithms.hpo import HyperoptService

    _, code, got = validate(HyperoptService(), hp_experiment(algorithm, settings, params=[]).spec)
    if details is None:
        assert code == grpc.StatusCode.OK, got
    else:
        assert code == grpc.StatusCode.INVALID_ARGUMENT
        assert got.startswith(details), got


# ------------------------------------------------------------------------------------ optuna
OPTUNA_PARAMS = HP_PARAMS[:3] + [P("param-4", api.DOUBLE, max="5", min="1", step="1", list=[])]


@pytest.mark.parametrize("algorithm,settings", [
    ("tpe", {"n_startup_trials": "20", "n_ei_candidates": "10", "random_state": "71"}),
    ("multivariate-tpe", {"n_startup_trials": "20", "n_ei_candidates": "10", "random_state": "71"}),
    ("cmaes", {"restart_strategy": "ipop", "sigma": "2", "random_state": "71"}),
    ("random", {"random_state": "71"}),
    ("grid", {"random_state": "71"}),
])
def test_optuna_get_suggestion(algorithm, settings):
    """test_optuna_service.py:33-193: first call without trials, second call with the first
    call's assignments as completed trials; 2 assignments each time."""
    from katib_amd.algorithms.hpo import OptunaService

    svc = OptunaService()
    exp = hp_experiment(algorithm, settings, params=OPTUNA_PARAMS)
    reply, code, details = call(svc.GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, trials=[], current_request_number=2))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 2
    trials = hp_trials(assignments=[reply.parameter_assignments[0].assignments,
                                    reply.parameter_assignments[1].assignments])
    reply, code, details = call(svc.GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, trials=trials, current_request_number=2))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 2


TWO_INTS = [P("param-1", api.INT, max="5", min="1", list=[]), P("param-2", api.INT, max="10", min="9", list=[])]
OK, BAD = grpc.StatusCode.OK, grpc.StatusCode.INVALID_ARGUMENT


@pytest.mark.parametrize("algorithm,settings,max_trials,params,result", [
    ("invalid", {}, 1, [], BAD),
    ("tpe", {"n_startup_trials": "5", "n_ei_candidates": "24", "random_state": "1"}, 100, [], OK),
    ("tpe", {"invalid": "5"}, 100, [], BAD),
    ("tpe", {"n_startup_trials": "-1"}, 100, [], BAD),
    ("tpe", {"n_ei_candidate": "-1"}, 100, [], BAD),
    ("tpe", {"random_state": "-1"}, 100, [], BAD),
    ("multivariate-tpe", {"n_startup_trials": "5", "n_ei_candidates": "24", "random_state": "1"}, 100, [], OK),
    ("cmaes", {"restart_strategy": "ipop", "sigma": "0.1", "random_state": "10"}, 20, TWO_INTS, OK),
    ("cmaes", {"invalid": "invalid", "sigma": "0.1"}, 100, TWO_INTS, BAD),
    ("cmaes", {"restart_strategy": "invalid", "sigma": "0.1"}, 15, TWO_INTS, BAD),
    ("cmaes", {"restart_strategy": "None", "sigma": "-10"}, 55, TWO_INTS, BAD),
    ("cmaes", {"sigma": "0.2", "random_state": "-20"}, 25, TWO_INTS, BAD),
    ("cmaes", {"sigma": "0.2"}, 5, TWO_INTS[:1], BAD),
    ("random", {"random_state": "10"}, 23, TWO_INTS, OK),
    ("random", {"invalid": "invalid"}, 33, [], BAD),
    ("random", {"random_state": "-1"}, 33, [], BAD),
    ("grid", {"random_state": "10"}, 5, TWO_INTS[:1], OK),
    ("grid", {"invalid": "invalid"}, 33, [], BAD),
    ("grid", {"random_state": "-1"}, 10, [], BAD),
    ("grid", {"random_state": "1"}, 26, [P("param-1", api.DOUBLE, max="5", min="1", list=[])], BAD),
    ("grid", {"random_state": "1"}, 26, [TWO_INTS[0], P("param-2", api.DOUBLE, max="5", min="1", step="1", list=[])],
     BAD),
])
def test_optuna_validate_algorithm_settings(algorithm, settings, max_trials, params, result):
    """test_optuna_service.py:195-497 (all 21 cases)."""
    from katib_amd.algorithms.hpo import OptunaService

    _, code, details = validate(OptunaService(), hp_experiment(algorithm, settings, params, max_trials).spec)
    assert code == result, details


# ------------------------------------------------------------------------------------ skopt
def test_skopt_get_suggestion():
    """test_skopt_service.py:36-190."""
    from katib_amd.algorithms.hpo import SkoptService

    exp = hp_experiment("bayesianoptimization", {"random_state": "10"})
    reply, code, details = call(SkoptService().GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, trials=hp_trials(), current_request_number=2))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 2


@pytest.mark.parametrize("algorithm,settings,details", [
    ("bayesianoptimization", {"random_state": "10"}, None),
    ("unknown", {}, "unknown algorithm name unknown"),
    ("bayesianoptimization", {"unknown_conf": "1111"},
     "unknown setting unknown_conf for algorithm bayesianoptimization"),
    ("bayesianoptimization", {"base_estimator": "unknown estimator"},
     "base_estimator unknown estimator is not supported in Bayesian optimization"),
    ("bayesianoptimization", {"n_initial_points": "-1"}, "n_initial_points should be great or equal than zero"),
    ("bayesianoptimization", {"acq_func": "unknown"}, "acq_func unknown is not supported in Bayesian optimization"),
    ("bayesianoptimization", {"acq_optimizer": "unknown"},
     "acq_optimizer unknown is not supported in Bayesian optimization"),
    ("bayesianoptimization", {"random_state": "-1"}, "random_state should be great or equal than zero"),
])
def test_skopt_validate_algorithm_settings(algorithm, settings, details):
    """test_skopt_service.py:192-311 (same messages)."""
    from katib_amd.algorithms.hpo import SkoptService

    _, code, got = validate(SkoptService(), hp_experiment(algorithm, settings, params=[]).spec)
    if details is None:
        assert code == grpc.StatusCode.OK, got
    else:
        assert code == grpc.StatusCode.INVALID_ARGUMENT and got == details, got


# ------------------------------------------------------------------------------------ goptuna
@pytest.mark.parametrize("algorithm,settings", [
    ("cmaes", {"random_state": "71", "sigma": "0.2"}), ("sobol", {}), ("tpe", {"random_state": "71"}),
    ("random", {"random_state": "71"})])
def test_goptuna_get_suggestion(algorithm, settings):
    """reference pkg/suggestion/v1beta1/goptuna/service_test.go: 2 continuous dims, two rounds."""
    from katib_amd.algorithms.hpo import GoptunaService

    params = [P("param-1", api.DOUBLE, max="5", min="1", list=[]), P("param-2", api.DOUBLE, max="10", min="9", list=[])]
    svc = GoptunaService()
    exp = hp_experiment(algorithm, settings, params=params)
    reply, code, details = call(svc.GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, trials=[], current_request_number=2))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 2
    trials = hp_trials(assignments=[pa.assignments for pa in reply.parameter_assignments])
    reply, code, details = call(svc.GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, trials=trials, current_request_number=3))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 3
    for pa in reply.parameter_assignments:
        v = {a.name: float(a.value) for a in pa.assignments}
        assert 1 <= v["param-1"] <= 5 and 9 <= v["param-2"] <= 10


# ------------------------------------------------------------------------------------ hyperband
def test_hyperband_get_suggestion():
    """test_hyperband_service.py:34-192: r_l=10 over --num-epochs, 2 assignments; the
    algorithm state round-trips through the reply's algorithm settings."""
    from katib_amd.algorithms.hyperband import HyperbandService

    exp = hp_experiment("hyperband", {"r_l": "10", "resource_name": "--num-epochs"})
    trials = hp_trials(cond=api.TrialStatus.RUNNING)
    reply, code, details = call(HyperbandService().GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, trials=trials, current_request_number=2))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 2
    state = {s.name: s.value for s in reply.algorithm.algorithm_settings}
    assert {"eta", "s_max", "r_l", "b_l", "r", "n", "current_s", "current_i", "resource_name"} <= set(state)
    assert state["resource_name"] == "--num-epochs" and float(state["r_l"]) == 10


@pytest.mark.parametrize("settings,parallel,ok", [
    ({"r_l": "9", "resource_name": "epochs", "eta": "3"}, 9, True),
    ({"resource_name": "epochs"}, 9, False),                      # r_l missing
    ({"r_l": "9"}, 9, False),                                     # resource_name missing
    ({"r_l": "9", "resource_name": "epochs", "eta": "3"}, 2, False),  # parallelTrialCount < eta^s_max
])
def test_hyperband_validate_algorithm_settings(settings, parallel, ok):
    """hyperband/service.py:199-243 validation rules."""
    from katib_amd.algorithms.hyperband import HyperbandService

    params = [P("lr", api.DOUBLE, max="0.1", min="0.01", list=[]), P("epochs", api.INT, max="9", min="1", list=[])]
    exp = hp_experiment("hyperband", settings, params=params)
    exp.spec.parallel_trial_count = parallel
    _, code, details = validate(HyperbandService(), exp.spec)
    assert (code == grpc.StatusCode.OK) == ok, details


# ------------------------------------------------------------------------------------ NAS common / DARTS
def _op(op_type, *params):
    return api.Operation(operation_type=op_type, parameter_specs=api.Operation.ParameterSpecs(parameters=list(params)))


@pytest.mark.parametrize("ops,valid", [
    ([_op("separable_convolution", P("filter_size", api.CATEGORICAL, list=["3", "5"]),
          P("pool_size", api.INT, max="2", min="3", step="1", list=[]),
          P("valid_type_double_example", api.DOUBLE, max="1.0", min="3.0", step="0.1", list=[]))], True),
    ([api.Operation(parameter_specs=api.Operation.ParameterSpecs(parameters=[
        P("filter_size", api.CATEGORICAL, list=["3", "5"])]))], False),            # no operation type
    ([api.Operation(operation_type="separable_convolution", parameter_specs=api.Operation.ParameterSpecs())], False),
    ([_op("separable_convolution", P("", api.CATEGORICAL, list=["3", "5"]))], False),  # empty name
    ([_op("separable_convolution", api.ParameterSpec(name="filter_size", feasible_space=api.FeasibleSpace(
        list=["3", "5"])))], False),                                                 # no parameter type
    ([_op("separable_convolution", P("filter_size", api.CATEGORICAL, max="1", min="2"))], False),  # no list
    ([_op("separable_convolution", P("pool_size", api.INT, list=["1", "2"]))], False),             # no min/max
    ([_op("separable_convolution", P("invalid_type_double_example", api.DOUBLE, max="1.0", min="3.0"))], False),
])
def test_nas_validate_operations(ops, valid):
    """test_nas_common.py:23-176 (all 8 cases)."""
    from katib_amd.algorithms.nas import validate_operations

    assert validate_operations(ops)[0] is valid


DARTS_VALID = {"num_epoch": "10", "w_lr": "0.01", "w_lr_min": "0.01", "alpha_lr": "0.01", "w_weight_decay": "0.25",
               "alpha_weight_decay": "0.25", "w_momentum": "0.9", "w_grad_clip": "5.0", "batch_size": "100",
               "num_workers": "0", "init_channels": "1", "print_step": "100", "num_nodes": "4", "stem_multiplier": "3"}


@pytest.mark.parametrize("settings,valid", [
    (DARTS_VALID, True), ({"num_epochs": "0"}, False), ({"w_lr": "-0.1"}, False),
    ({"alpha_weight_decay": "-0.02"}, False), ({"w_momentum": "-0.8"}, False), ({"batch_size": "0"}, False),
    ({"batch_size": "None"}, True), ({"print_step": "0"}, False)])
def test_darts_validate_algorithm_settings(settings, valid):
    """test_darts_service.py:116-171."""
    from katib_amd.algorithms.nas import validate_darts_settings

    assert validate_darts_settings([api.AlgorithmSetting(name=k, value=v) for k, v in settings.items()])[0] is valid


def test_darts_get_suggestion():
    """test_darts_service.py:35-114: one assignment carrying the user's settings over the
    defaults, num-layers and the expanded search space."""
    from katib_amd.algorithms.nas import DartsService

    exp = api.Experiment(name="darts-experiment", spec=api.ExperimentSpec(
        algorithm=api.AlgorithmSpec(algorithm_name="darts",
                                    algorithm_settings=[api.AlgorithmSetting(name="num_epoch", value="10")]),
        objective=api.ObjectiveSpec(type=api.MAXIMIZE, objective_metric_name="Best-Genotype"),
        parallel_trial_count=1, max_trial_count=1,
        nas_config=api.NasConfig(graph_config=api.GraphConfig(num_layers=3), operations=api.NasConfig.Operations(
            operation=[_op("separable_convolution", P("filter_size", api.CATEGORICAL, list=["3", "5"]))]))))
    reply, code, details = call(DartsService().GetSuggestions,
                                api.GetSuggestionsRequest(experiment=exp, current_request_number=1))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 1
    got = {a.name: a.value for a in reply.parameter_assignments[0].assignments}
    settings = json.loads(got["algorithm-settings"].replace("'", '"'))
    assert settings["num_epoch"] == "10"
    assert int(got["num-layers"]) == 3
    assert json.loads(got["search-space"].replace("'", '"')) == ["separable_convolution_3x3",
                                                                  "separable_convolution_5x5"]


# ------------------------------------------------------------------------------------ ENAS
ENAS_OPS = [
    _op("convolution", P("filter_size", api.CATEGORICAL, list=["5"]), P("num_filter", api.CATEGORICAL, list=["128"]),
        P("stride", api.CATEGORICAL, list=["1", "2"])),
    _op("reduction", P("reduction_type", api.CATEGORICAL, list=["max_pooling"]),
        P("pool_size", api.INT, min="2", max="3", step="1", list=[])),
]


def enas_request(trials, n=2, settings=None, num_layers=4):
    """test_enas_service.py:37-195 fixture: 4 layers, input 32x32x8, conv + reduction ops."""
    exp = api.Experiment(name="enas-experiment", spec=api.ExperimentSpec(
        algorithm=api.AlgorithmSpec(algorithm_name="enas", algorithm_settings=[
            api.AlgorithmSetting(name=k, value=v) for k, v in (settings or {}).items()]),
        objective=api.ObjectiveSpec(type=api.MAXIMIZE, goal=0.9, objective_metric_name="Validation-Accuracy"),
        parallel_trial_count=2, max_trial_count=10,
        nas_config=api.NasConfig(graph_config=api.GraphConfig(num_layers=num_layers, input_sizes=[32, 32, 8],
                                                             output_sizes=[10]),
                                 operations=api.NasConfig.Operations(operation=ENAS_OPS))))
    archs = ["[[3], [0, 1], [0, 0, 1], [2, 1, 0, 0]]", "[[1], [0, 1], [2, 1, 1], [2, 1, 1, 0]]"]
    tr = []
    for i, (name, acc) in enumerate(trials):
        tr.append(api.Trial(
            name=name,
            spec=api.TrialSpec(objective=api.ObjectiveSpec(type=api.MAXIMIZE, objective_metric_name="Validation-Accuracy",
                                                           goal=0.99),
                               parameter_assignments=api.TrialSpec.ParameterAssignments(assignments=[
                                   api.ParameterAssignment(name="architecture", value=archs[i % 2]),
                                   api.ParameterAssignment(name="nn_config", value="{'num_layers': 4}")])),
            status=api.TrialStatus(condition=api.TrialStatus.SUCCEEDED, observation=api.Observation(
                metrics=[api.Metric(name="Validation-Accuracy", value=str(acc))]))))
    return api.GetSuggestionsRequest(experiment=exp, trials=tr, current_request_number=n)


def test_enas_get_suggestion(tmp_path, monkeypatch):
    """test_enas_service.py:37-195 (first call samples; a call with succeeded trials trains the
    controller for controller_train_steps and samples again); torch backend on the CPU."""
    from katib_amd.algorithms.nas import EnasService

    monkeypatch.setenv("KATIB_AMD_ENAS_BACKEND", "torch")
    svc = EnasService(cache_dir=str(tmp_path), seed=1)
    reply, code, details = call(svc.GetSuggestions, enas_request([("first-trial", 0.88), ("second-trial", 0.84)]))
    assert code == grpc.StatusCode.OK, details
    assert len(reply.parameter_assignments) == 2
    for pa in reply.parameter_assignments:
        got = {a.name: a.value for a in pa.assignments}
        arch = json.loads(got["architecture"].replace("'", '"'))
        assert [len(layer) for layer in arch] == [1, 2, 3, 4]
        cfg = json.loads(got["nn_config"].replace("'", '"'))
        assert cfg["num_layers"] == 4 and cfg["input_sizes"] == [32, 32, 8] and cfg["output_sizes"] == [10]
    reply, code, _ = call(svc.GetSuggestions, enas_request([("first-trial", 0.88), ("second-trial", 0.84)], n=3))
    assert code == grpc.StatusCode.OK and len(reply.parameter_assignments) == 3
    assert svc.controller.train_step == 50
    assert os.path.exists(os.path.join(str(tmp_path), "enas-experiment.pt"))


def test_enas_all_trials_failed_returns_empty(tmp_path, monkeypatch):
    """nas/enas/service.py:294-301: no succeeded trial after the first call -> empty reply."""
    from katib_amd.algorithms.nas import EnasService

    monkeypatch.setenv("KATIB_AMD_ENAS_BACKEND", "torch")
    svc = EnasService(cache_dir=str(tmp_path), seed=1)
    call(svc.GetSuggestions, enas_request([]))
    reply, code, _ = call(svc.GetSuggestions, enas_request([]))
    assert code == grpc.StatusCode.OK and len(reply.parameter_assignments) == 0


@pytest.mark.parametrize("settings,ok", [
    ({"controller_hidden_size": "64", "controller_temperature": "5", "controller_tanh_const": "2.25"}, True),
    ({"controller_temperature": "None", "controller_tanh_const": "None"}, True),
    ({"controller_hidden_size": "0"}, False), ({"controller_learning_rate": "-1"}, False),
    ({"controller_unknown": "1"}, False), ({"controller_train_steps": "abc"}, False)])
def test_enas_validate_algorithm_settings(settings, ok):
    """nas/enas/service.py validation (AlgorithmSettings.py ranges)."""
    from katib_amd.algorithms.nas import EnasService

    req = enas_request([], settings=settings)
    _, code, details = validate(EnasService(), req.experiment.spec)
    assert (code == grpc.StatusCode.OK) == ok, details


def test_enas_controller_reinforce_learns_a_bandit():
    """REINFORCE direction (Controller.py:200-222, loss = CE * (R - b)): per-sample rewards
    for one op raise its probability (torch oracle; the HIP kernel is checked against it in
    tests/test_gpu_enas.py)."""
    from katib_amd.models.enas_controller import EnasController

    c = EnasController(num_layers=2, num_operations=4, hidden_size=32, seed=1, learning_rate=0.05,
                       entropy_weight=None, skip_weight=None)
    with __import__("torch").no_grad():
        hits0 = sum(c.sample_arc()[0] == 2 for _ in range(300)) / 300
    for _ in range(150):
        arc = c.sample_arc()
        c.train_once(1.0 if arc[0] == 2 else 0.0, forced=arc)
    with __import__("torch").no_grad():
        hits1 = sum(c.sample_arc()[0] == 2 for _ in range(300)) / 300
    assert hits1 > max(0.6, hits0 + 0.3), (hits0, hits1)


# ------------------------------------------------------------------------------------ medianstop
def ms_spec(algorithm="medianstop", **settings):
    return api.EarlyStoppingSpec(algorithm_name=algorithm, algorithm_settings=[
        api.EarlyStoppingSetting(name=k, value=v) for k, v in settings.items()])


@pytest.mark.parametrize("spec,details", [
    (ms_spec(min_trials_required="2", start_step="5"), None),
    (ms_spec("unknown"), "unknown algorithm name unknown"),
    (ms_spec(unknown_conf="100"), "unknown setting unknown_conf for algorithm medianstop"),
    (ms_spec(min_trials_required="0"), "min_trials_required must be greater than zero (>0)"),
    (ms_spec(start_step="0"), "start_step must be greater or equal than one (>=1)"),
])
def test_medianstop_validate_early_stopping_settings(spec, details):
    """test_medianstop_service.py:38-111 (same messages)."""
    from katib_amd.earlystopping.medianstop import MedianStopService

    _, code, got = call(MedianStopService().ValidateEarlyStoppingSettings,
                        api.ValidateEarlyStoppingSettingsRequest(early_stopping=spec))
    if details is None:
        assert code == grpc.StatusCode.OK, got
    else:
        assert code == grpc.StatusCode.INVALID_ARGUMENT and got == details, got


def test_medianstop_get_early_stopping_rules():
    """test_medianstop_service.py:113-139 plus the rule itself: the mean of the first
    start_step values of the succeeded trials, LESS for maximize."""
    from katib_amd.earlystopping.medianstop import MedianStopService

    logs = {"t1": ["0.5", "0.7", "0.9"], "t2": ["0.1", "0.3", "0.2"]}

    class Store:  # observation store: get_observation_log(trial, metric) -> [(time, metric, value)]
        def __init__(self, d):
            self.d = d

        def get_observation_log(self, trial, metric):
            return [("2024-01-01T00:00:0%dZ" % i, metric, v) for i, v in enumerate(self.d.get(trial, []))]

    svc = MedianStopService(log_source=Store(logs))
    exp = api.Experiment(name="test", spec=api.ExperimentSpec(
        objective=api.ObjectiveSpec(type=api.MAXIMIZE, objective_metric_name="acc"),
        early_stopping=ms_spec(min_trials_required="2", start_step="2")))
    trials = [api.Trial(name=n, status=api.TrialStatus(condition=api.TrialStatus.SUCCEEDED)) for n in logs]
    reply, code, _ = call(svc.GetEarlyStoppingRules, api.GetEarlyStoppingRulesRequest(
        experiment=exp, trials=trials, db_manager_address="katib-db-manager.kubeflow:6789"))
    assert code == grpc.StatusCode.OK
    assert len(reply.early_stopping_rules) == 1
    r = reply.early_stopping_rules[0]
    assert r.name == "acc" and r.comparison == api.LESS and r.start_step == 2
    assert float(r.value) == pytest.approx((0.6 + 0.2) / 2)
    # the reference's smoke case: bare trials, no rules yet
    reply, code, _ = call(MedianStopService(log_source=Store({})).GetEarlyStoppingRules,
                          api.GetEarlyStoppingRulesRequest(experiment=api.Experiment(name="test"),
                                                           trials=[api.Trial(name="test-asfjh"),
                                                                   api.Trial(name="test-234hs")]))
    assert code == grpc.StatusCode.OK and len(reply.early_stopping_rules) == 0


# ------------------------------------------------------------------------------------ TF events
def test_tfevent_collector_parse_file(tmp_path):
    """test_tfevent_metricscollector.py:20-41: metrics named {dir}/{tag} across train/ and
    test/ subdirectories (20 logs), and bare tag names inside one directory (10 logs). The
    reference's fixture is produced by running its TF MNIST example; ours writes the same
    layout (5 steps x accuracy/loss x train/test) with the built-in event writer."""
    from katib_amd.metricscollector.tfevent import EventWriter, collect

    for sub in ("train", "test"):
        w = EventWriter(str(tmp_path / sub))
        for step in range(5):
            w.add_scalar("accuracy", 0.5 + 0.1 * step, step)
            w.add_scalar("loss", 1.0 - 0.1 * step, step)
        w.close()
    names = ["train/accuracy", "train/loss", "test/loss", "test/accuracy"]
    logs = collect(str(tmp_path), names)
    assert len(logs) == 20 and {n for _, n, _ in logs} == set(names)
    logs = collect(str(tmp_path / "train"), ["accuracy", "loss"])
    assert len(logs) == 10 and {n for _, n, _ in logs} == {"accuracy", "loss"}
