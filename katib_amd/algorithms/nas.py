"""Neural-architecture-search suggestion services: DARTS and ENAS.

* :class:`DartsService` (reference ``pkg/suggestion/v1beta1/nas/darts/service.py:26-201``):
  no search logic - emits ``current_request_number`` identical assignments
  ``algorithm-settings`` (JSON with defaults), ``search-space`` (primitive names
  ``<op>_<k>x<k>`` / ``skip_connection``) and ``num-layers``; double quotes are
  swapped for single quotes. The supernet search itself runs inside the trial
  (:mod:`katib_amd.models.darts`).
* :class:`EnasService` (reference ``nas/enas/service.py:32-431``): LSTM controller
  (:class:`katib_amd.models.enas_controller.EnasController`); first call samples
  random arcs from the initial controller, later calls compute the reward as the
  mean objective of succeeded trials (negated for minimise), run
  ``controller_train_steps`` REINFORCE steps and sample new arcs. The controller
  state is kept in memory and checkpointed to ``<cache_dir>/<experiment>.pt``.
"""

from __future__ import annotations

import itertools
import json
import os
from typing import Dict, List

import numpy as np

from ..rpc import api_pb2 as api
from .internal import SuggestionService, abort

DARTS_DEFAULT_SETTINGS = {
    "num_epochs": 50, "w_lr": 0.025, "w_lr_min": 0.001, "w_momentum": 0.9, "w_weight_decay": 3e-4,
    "w_grad_clip": 5., "alpha_lr": 3e-4, "alpha_weight_decay": 1e-3, "batch_size": 128, "num_workers": 4,
    "init_channels": 16, "print_step": 50, "num_nodes": 4, "stem_multiplier": 3,
}


# ------------------------------------------------------------------------------- common validation
def validate_operations(operations, parameterless=()) -> (bool, str):
    """``nas/common/validation.py:18-63``. ``parameterless``: operation types accepted
    without parameters - documented divergence for DARTS' ``skip_connection``, which the
    reference's own darts examples declare without parameters but its shared validator
    rejects ("Missing ParameterConfigs")."""
    for op in operations:
        if not op.operation_type:
            return False, "Missing operationType in Operation:\n{}".format(op)
        if not op.parameter_specs.parameters and op.operation_type in parameterless:
            continue
        if not op.parameter_specs.parameters:
            return False, "Missing ParameterConfigs in Operation:\n{}".format(op)
        for p in op.parameter_specs.parameters:
            if not p.name:
                return False, "Missing Name in ParameterConfig:\n{}".format(p)
            if not p.parameter_type:
                return False, "Missing ParameterType in ParameterConfig:\n{}".format(p)
            if p.parameter_type in (api.CATEGORICAL, api.DISCRETE):
                if not p.feasible_space.list:
                    return False, "Missing List in ParameterConfig.feasibleSpace:\n{}".format(p)
            elif p.parameter_type in (api.INT, api.DOUBLE):
                if not p.feasible_space.min and not p.feasible_space.max:
                    return False, "Missing Max and Min in ParameterConfig.feasibleSpace:\n{}".format(p)
                try:
                    if p.parameter_type == api.DOUBLE and (not p.feasible_space.step
                                                           or float(p.feasible_space.step) <= 0):
                        return False, "Step parameter should be > 0 in ParameterConfig.feasibleSpace:\n{}".format(p)
                except Exception as e:
                    return False, "failed to validate ParameterConfig.feasibleSpace \n{parameter}):\n{exception}".format(
                        parameter=p, exception=e)
    return True, ""


def validate_darts_settings(settings) -> (bool, str):
    for s in settings:
        try:
            if s.name == "num_epochs" and not int(s.value) > 0:
                return False, "{} should be greater than zero".format(s.name)
            if s.name in {"w_lr", "w_lr_min", "alpha_lr", "w_weight_decay", "alpha_weight_decay", "w_momentum",
                          "w_grad_clip"} and not float(s.value) >= 0.0:
                return False, "{} should be greater than or equal to zero".format(s.name)
            if s.name == "batch_size" and s.value != "None" and not int(s.value) >= 1:
                return False, "batch_size should be greater than or equal to one"
            if s.name == "num_workers" and not int(s.value) >= 0:
                return False, "num_workers should be greater than or equal to zero"
            if s.name in {"init_channels", "print_step", "num_nodes", "stem_multiplier"} and not int(s.value) >= 1:
                return False, "{} should be greater than or equal to one".format(s.name)
        except Exception as e:
            return False, "failed to validate {name}({value}): {exception}".format(name=s.name, value=s.value,
                                                                                   exception=e)
    return True, ""


# ------------------------------------------------------------------------------- DARTS
def darts_search_space(operations) -> List[str]:
    out = []
    for op in operations.operation:
        if op.operation_type == "skip_connection":
            out.append(op.operation_type)
        else:
            spec = list(op.parameter_specs.parameters)[0]
            for fs in spec.feasible_space.list:
                out.append(op.operation_type + "_{}x{}".format(fs, fs))
    return out


def darts_algorithm_settings(settings_raw) -> Dict:
    d = dict(DARTS_DEFAULT_SETTINGS)
    for s in settings_raw:
        d[s.name] = None if s.value == "None" else s.value
    return d


class DartsService(SuggestionService):
    algorithm_names = ("darts",)

    def ValidateAlgorithmSettings(self, request, context=None):
        spec = request.experiment.spec
        ok, msg = validate_operations(spec.nas_config.operations.operation, parameterless=("skip_connection",))
        if ok:
            ok, msg = validate_darts_settings(spec.algorithm.algorithm_settings)
        if not ok:
            abort(context, "INVALID_ARGUMENT", msg)
        return api.ValidateAlgorithmSettingsReply()

    def GetSuggestions(self, request, context=None):
        nas = request.experiment.spec.nas_config
        num_layers = str(nas.graph_config.num_layers)
        ss = json.dumps(darts_search_space(nas.operations)).replace('"', "'")
        st = json.dumps(darts_algorithm_settings(request.experiment.spec.algorithm.algorithm_settings)).replace('"', "'")
        pas = [api.GetSuggestionsReply.ParameterAssignments(assignments=[
            api.ParameterAssignment(name="algorithm-settings", value=st),
            api.ParameterAssignment(name="search-space", value=ss),
            api.ParameterAssignment(name="num-layers", value=num_layers)])
            for _ in range(request.current_request_number)]
        return api.GetSuggestionsReply(parameter_assignments=pas)


# ------------------------------------------------------------------------------- ENAS
ENAS_SETTINGS = {
    "controller_hidden_size": (int, [1, "inf"], 64),
    "controller_temperature": (float, [0, "inf"], 5.0),
    "controller_tanh_const": (float, [0, "inf"], 2.25),
    "controller_entropy_weight": (float, [0.0, "inf"], 1e-5),
    "controller_baseline_decay": (float, [0.0, 1.0], 0.999),
    "controller_learning_rate": (float, [0.0, 1.0], 5e-5),
    "controller_skip_target": (float, [0.0, 1.0], 0.4),
    "controller_skip_weight": (float, [0.0, "inf"], 0.8),
    "controller_train_steps": (int, [1, "inf"], 50),
    "controller_log_every_steps": (int, [1, "inf"], 10),
}
ENAS_NONE_OK = ("controller_temperature", "controller_tanh_const", "controller_entropy_weight",
                "controller_skip_weight")


def enas_operations(operations) -> List[Dict]:
    """Expand every operation's parameter product into op ids (``enas/Operation.py:42-91``)."""
    out, oid = [], 0
    for op in operations.operation:
        space = {}
        for sp in op.parameter_specs.parameters:
            if sp.parameter_type == api.CATEGORICAL:
                space[sp.name] = list(sp.feasible_space.list)
            elif sp.parameter_type == api.INT:
                space[sp.name] = list(range(int(sp.feasible_space.min), int(sp.feasible_space.max) + 1,
                                            int(sp.feasible_space.step)))
            elif sp.parameter_type == api.DOUBLE:
                lo, hi, st = float(sp.feasible_space.min), float(sp.feasible_space.max), float(sp.feasible_space.step)
                vals = np.arange(lo, hi + st, st)
                if vals[-1] > hi:
                    vals = vals[:-1]
                space[sp.name] = [float(v) for v in vals]
        keys = list(space)
        for combo in itertools.product(*space.values()):
            out.append({"opt_id": oid, "opt_type": op.operation_type, "opt_params": dict(zip(keys, combo))})
            oid += 1
    return out


def parse_enas_settings(settings_raw) -> Dict:
    d = {k: v[2] for k, v in ENAS_SETTINGS.items()}
    for s in settings_raw:
        d[s.name] = None if s.value == "None" else ENAS_SETTINGS[s.name][0](s.value)
    return d


class EnasService(SuggestionService):
    algorithm_names = ("enas",)

    def __init__(self, cache_dir: str = None, seed=None):
        self.cache_dir = cache_dir or os.environ.get("KATIB_AMD_ENAS_CACHE", "/tmp/katib-amd/ctrl_cache")
        self.controller = None
        self.first = True
        self.suggestion_step = 0
        self.seed = seed
        self.last_train_log = []

    def ValidateAlgorithmSettings(self, request, context=None):
        nas = request.experiment.spec.nas_config
        gc = nas.graph_config

        def bad(msg):
            abort(context, "INVALID_ARGUMENT", msg)
            return api.ValidateAlgorithmSettingsReply()

        if not gc.input_sizes:
            return bad("Missing InputSizes in GraphConfig:\n{}".format(gc))
        if not gc.output_sizes:
            return bad("Missing OutputSizes in GraphConfig:\n{}".format(gc))
        if not gc.num_layers:
            return bad("Missing NumLayers in GraphConfig:\n{}".format(gc))
        ok, msg = validate_operations(nas.operations.operation)
        if not ok:
            return bad(msg)
        for s in request.experiment.spec.algorithm.algorithm_settings:
            if s.name not in ENAS_SETTINGS:
                return bad("Unknown Algorithm Setting name: {}".format(s.name))
            if s.name in ENAS_NONE_OK and s.value == "None":
                continue
            typ, rng, _ = ENAS_SETTINGS[s.name]
            try:
                v = typ(s.value)
            except Exception as e:
                return bad("Algorithm Setting {} must be {} type: exception {}".format(s.name, typ.__name__, e))
            if typ == float:
                if v <= rng[0] or (rng[1] != "inf" and v > rng[1]):
                    return bad("Algorithm Setting {}: {} with {} type must be in range ({}, {}]".format(
                        s.name, v, typ.__name__, rng[0], rng[1]))
            elif v < rng[0]:
                return bad("Algorithm Setting {}: {} with {} type must be in range [{}, {})".format(
                    s.name, v, typ.__name__, rng[0], rng[1]))
        return api.ValidateAlgorithmSettingsReply()

    def _setup(self, exp):
        import torch  # noqa: F401
        from ..models.enas_controller import make_controller

        nas = exp.spec.nas_config
        self.num_layers = int(nas.graph_config.num_layers)
        self.input_sizes = list(map(int, nas.graph_config.input_sizes))
        self.output_sizes = list(map(int, nas.graph_config.output_sizes))
        self.search_space = enas_operations(nas.operations)
        self.settings = parse_enas_settings(exp.spec.algorithm.algorithm_settings)
        s = self.settings
        self.controller = make_controller(
            num_layers=self.num_layers, num_operations=len(self.search_space),
            hidden_size=s["controller_hidden_size"], temperature=s["controller_temperature"],
            tanh_const=s["controller_tanh_const"], entropy_weight=s["controller_entropy_weight"],
            baseline_decay=s["controller_baseline_decay"], learning_rate=s["controller_learning_rate"],
            skip_target=s["controller_skip_target"], skip_weight=s["controller_skip_weight"], seed=self.seed)
        self.opt_direction = exp.spec.objective.type
        self.experiment_name = exp.name

    def _ckpt(self):
        import torch

        os.makedirs(self.cache_dir, exist_ok=True)
        torch.save(self.controller.state(), os.path.join(self.cache_dir, f"{self.experiment_name}.pt"))

    @staticmethod
    def evaluation_result(trials):
        done = {}
        for t in trials:
            if t.status.condition == api.TrialStatus.SUCCEEDED:
                val = None
                for m in t.status.observation.metrics:
                    if m.name == t.spec.objective.objective_metric_name:
                        val = m.value
                        break
                try:
                    done[t.name] = float(val)
                except (TypeError, ValueError):
                    continue
        if done:
            return sum(done.values()) / len(done)
        return None

    def GetSuggestions(self, request, context=None):
        if self.controller is None:
            self._setup(request.experiment)
        n = request.current_request_number if request.current_request_number > 0 else 1
        if self.first:
            cands = self.controller.sample_arcs(n)
            self.first = False
        else:
            result = self.evaluation_result(request.trials)
            if result is None:
                # every spawned trial failed: the reference returns [] (service.py:294-301)
                return api.GetSuggestionsReply()
            if self.opt_direction == api.MINIMIZE:
                result = -result
            # all controller_train_steps REINFORCE steps (one kernel launch on the HIP backend)
            self.last_train_log = self.controller.train(result, self.settings["controller_train_steps"],
                                                        self.settings["controller_log_every_steps"])
            cands = self.controller.sample_arcs(n)
        self._ckpt()
        pas = []
        for arc in cands:
            organized, rec = [], 0
            for layer in range(self.num_layers):
                organized.append(arc[rec: rec + layer + 1])
                rec += layer + 1
            nn_config = {"num_layers": self.num_layers, "input_sizes": self.input_sizes,
                         "output_sizes": self.output_sizes, "embedding": {}}
            for layer in range(self.num_layers):
                op = organized[layer][0]
                nn_config["embedding"][op] = self.search_space[op]
            pas.append(api.GetSuggestionsReply.ParameterAssignments(assignments=[
                api.ParameterAssignment(name="architecture", value=json.dumps(organized).replace('"', "'")),
                api.ParameterAssignment(name="nn_config", value=json.dumps(nn_config).replace('"', "'"))]))
        self.suggestion_step += 1
        return api.GetSuggestionsReply(parameter_assignments=pas)
