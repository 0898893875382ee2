"""Hyperparameter-optimisation suggestion services.

Four service classes keep the *settings surface and validation messages* of the
reference services, all running on the shared samplers of
:mod:`katib_amd.algorithms.samplers`:

* :class:`HyperoptService` - ``random``, ``tpe`` (``pkg/suggestion/v1beta1/hyperopt/service.py:28-137``)
* :class:`OptunaService`   - ``tpe``, ``multivariate-tpe``, ``cmaes``, ``random``, ``grid``
  (``pkg/suggestion/v1beta1/optuna/service.py:30-270``)
* :class:`GoptunaService`  - ``cmaes``, ``sobol``, ``tpe``, ``random``
  (``pkg/suggestion/v1beta1/goptuna/service.go``, ``converter.go:69-184``)
* :class:`SkoptService`    - ``bayesianoptimization`` (``pkg/suggestion/v1beta1/skopt/service.py:60-140``)

Every service is stateful in memory, re-receives all trials on each call and
records a completed trial exactly once (by name), like the reference.
Divergence (documented): a completed trial whose assignments were not produced by
this service instance is accepted as an external observation instead of raising
"An unknown trial has been passed" (optuna/base_service.py:83-87) - needed to
resume an experiment from its journal after a scheduler restart.
"""

from __future__ import annotations

import itertools
import threading
from typing import Dict

from ..rpc import api_pb2 as api
from .internal import (MAX_GOAL, AlgorithmError, SearchSpace, SuggestionService, abort, convert_trials,
                       make_reply_assignments, numeric_losses, settings_dict)
from .samplers import (BayesOptSampler, CmaEsSampler, GridSampler, RandomSampler, SobolSampler, Study,
                       TpeSampler)


class _StudyService(SuggestionService):
    """ask/tell engine shared by the services below."""

    def __init__(self):
        self.lock = threading.Lock()
        self.study = None
        self.sampler = None
        self.space = None

    # subclasses: build sampler from (algorithm name, settings)
    def make_sampler(self, name: str, settings: Dict[str, str], space: SearchSpace, request):
        raise NotImplementedError

    def _ensure(self, request):
        if self.study is None:
            self.space = SearchSpace.convert(request.experiment)
            alg = request.experiment.spec.algorithm
            self.sampler = self.make_sampler(alg.algorithm_name, settings_dict(alg), self.space, request)
            self.study = Study(self.space)

    def _tell_all(self, request):
        trials = convert_trials(request.trials)
        for t in trials:
            v = t.objective()
            if v is None:
                continue
            loss = -v if self.space.goal == MAX_GOAL else v
            params = self.study.tell(t.name, t.assignments, loss)
            if params is not None:
                self.sampler.on_tell(self.study, params, loss)

    def GetSuggestions(self, request, context=None):
        with self.lock:
            try:
                self._ensure(request)
                self._tell_all(request)
                out = []
                n = request.current_request_number
                for _ in range(n):
                    params = self.sampler.sample(self.study, n)
                    self.study.register_ask(params)
                    out.append({k: v for k, v in params.items() if not k.startswith("__")})
                # keep spec parameter order in the reply
                order = [p.name for p in self.space.params]
                out = [[(k, a[k]) for k in order if k in a] for a in out]
                return api.GetSuggestionsReply(parameter_assignments=make_reply_assignments(out))
            except AlgorithmError as e:
                abort(context, e.code, e.message)
                return api.GetSuggestionsReply()

    def is_exhausted(self) -> bool:
        return isinstance(self.sampler, GridSampler) and self.sampler.exhausted()

    # validation helpers ---------------------------------------------------------------
    def _invalid(self, context, message):
        abort(context, "INVALID_ARGUMENT", message)
        return api.ValidateAlgorithmSettingsReply()


def _check(settings, rules, algo):
    """rules: name -> (parser, predicate, message). Returns None when every setting is
    valid, else the reference's error message (which may be the empty string, as for a
    negative random_state in optuna/service.py:226-229). ``message`` may be a callable of
    (name, value) for messages that quote the offending value."""
    for name, value in settings:
        if name not in rules:
            return "unknown setting {} for algorithm {}".format(name, algo)
        parse, pred, msg = rules[name]
        try:
            if not pred(parse(value)):
                return msg(name, value) if callable(msg) else msg
        except Exception as e:
            return "failed to validate {name}({value}): {exception}".format(name=name, value=value, exception=e)
    return None


def _pairs(request):
    return [(s.name, s.value) for s in request.experiment.spec.algorithm.algorithm_settings]


def _count_continuous(request):
    return sum(1 for p in request.experiment.spec.parameter_specs.parameters
               if p.parameter_type in (api.DOUBLE, api.INT))


# ==================================================================================== hyperopt
class HyperoptService(_StudyService):
    algorithm_names = ("random", "tpe")

    def make_sampler(self, name, s, space, request):
        seed = int(s["random_state"]) if "random_state" in s else None
        if name == "random":
            return RandomSampler(space, seed)
        if name == "tpe":
            return TpeSampler(space, seed, mode="hyperopt", gamma=float(s.get("gamma", 0.25)),
                              prior_weight=float(s.get("prior_weight", 1.0)),
                              n_ei_candidates=int(s.get("n_EI_candidates", 24)))
        raise AlgorithmError("unknown algorithm name {}".format(name))

    def ValidateAlgorithmSettings(self, request, context=None):
        name = request.experiment.spec.algorithm.algorithm_name
        if name == "tpe":
            err = _check(_pairs(request), {
                "gamma": (float, lambda v: 1 > v > 0, "gamma should be in the range of (0, 1)"),
                "prior_weight": (float, lambda v: v > 0, "prior_weight should be great than zero"),
                "n_EI_candidates": (int, lambda v: v > 0, "n_EI_candidates should be great than zero"),
                "random_state": (int, lambda v: v >= 0, "random_state should be great or equal than zero"),
            }, "tpe")
        elif name == "random":
            err = _check(_pairs(request), {
                "random_state": (int, lambda v: v >= 0, "random_state should be great or equal than zero")},
                "random")
        else:
            err = "unknown algorithm name {}".format(name)
        if err is not None:
            return self._invalid(context, err)
        return api.ValidateAlgorithmSettingsReply()


# ==================================================================================== optuna
class OptunaService(_StudyService):
    algorithm_names = ("tpe", "multivariate-tpe", "cmaes", "random", "grid")

    def make_sampler(self, name, s, space, request):
        seed = s.get("seed", s.get("random_state"))
        seed = int(seed) if seed not in (None, "") else None
        if name in ("tpe", "multivariate-tpe"):
            return TpeSampler(space, seed, mode="optuna",
                              n_startup_trials=int(s.get("n_startup_trials", 10)),
                              n_ei_candidates=int(s.get("n_ei_candidates", 24)),
                              multivariate=(name == "multivariate-tpe"), constant_liar=True)
        if name == "cmaes":
            sigma = s.get("sigma", s.get("sigma0"))
            return CmaEsSampler(space, seed, sigma0=float(sigma) if sigma else None,
                                restart_strategy=s.get("restart_strategy"))
        if name == "random":
            return RandomSampler(space, seed)
        if name == "grid":
            return GridSampler(space, seed)
        raise AlgorithmError("unknown algorithm name {}".format(name))

    def ValidateAlgorithmSettings(self, request, context=None):
        """optuna/service.py:118-262: per-algorithm setting rules, CMA-ES needs >= 2
        continuous dimensions, grid needs maxTrialCount <= number of combinations."""
        exp = request.experiment
        name = exp.spec.algorithm.algorithm_name
        pairs = _pairs(request)
        ge0 = lambda k: "{} should be greate or equal than zero".format(k)  # noqa: E731 (reference spelling)
        if name in ("tpe", "multivariate-tpe"):
            err = _check(pairs, {k: (int, lambda v: v >= 0, ge0(k))
                                 for k in ("n_startup_trials", "n_ei_candidates", "random_state")}, name)
        elif name == "cmaes":
            err = _check(pairs, {
                "restart_strategy": (str, lambda v: v in ("ipop", "None", "none"),
                                     lambda k, v: "restart_strategy {} is not supported in CMAES optimization".format(v)),
                "sigma": (float, lambda v: v >= 0, ge0("sigma")),
                "random_state": (int, lambda v: v >= 0, ge0("random_state")),
            }, "cmaes")
            if err is None and _count_continuous(request) < 2:
                err = "cmaes only supports two or more dimensional continuous search space."
        elif name in ("random", "grid"):
            err = _check(pairs, {"random_state": (int, lambda v: v >= 0, "")}, name)
            if err is None and name == "grid":
                space = SearchSpace.convert(exp)
                try:
                    n = 1
                    for v in space.combinations().values():
                        n *= len(v)
                    if exp.spec.max_trial_count > n:
                        err = "Max Trial Count: {max_trial} > all possible search combinations: {combinations}".format(
                            max_trial=exp.spec.max_trial_count, combinations=n)
                except Exception as e:
                    err = "failed to validate parameters({parameters}): {exception}".format(
                        parameters=space.params, exception=e)
        else:
            err = "unknown algorithm name {}".format(name)
        if err is not None:
            return self._invalid(context, err)
        return api.ValidateAlgorithmSettingsReply()


# ==================================================================================== goptuna
class GoptunaService(_StudyService):
    algorithm_names = ("cmaes", "tpe", "random", "sobol")

    def make_sampler(self, name, s, space, request):
        seed = int(s["random_state"]) if s.get("random_state") not in (None, "") else None
        if name == "cmaes":
            rs = s.get("restart_strategy", "none")
            if rs not in ("ipop", "bipop", "none"):
                raise AlgorithmError("invalid restart_strategy: '%s'" % rs, "INTERNAL")
            return CmaEsSampler(space, seed, sigma0=float(s["sigma"]) if s.get("sigma") else None,
                                restart_strategy=None if rs == "none" else rs)
        if name == "tpe":
            return TpeSampler(space, seed, mode="optuna", gamma=0.25,
                              n_startup_trials=int(s.get("n_startup_trials", 10)),
                              n_ei_candidates=int(s.get("n_ei_candidates", 24)))
        if name == "sobol":
            return SobolSampler(space, seed)
        return RandomSampler(space, seed)

    def ValidateAlgorithmSettings(self, request, context=None):
        name = request.experiment.spec.algorithm.algorithm_name
        if name not in self.algorithm_names:
            return self._invalid(context, "unsupported algorithm")
        params = request.experiment.spec.parameter_specs.parameters
        if name == "cmaes" and _count_continuous(request) < 2:
            return self._invalid(context, "CMA-ES only supports two or more dimensional continuous search space.")
        seen = set()
        for p in params:
            if p.name in seen:
                return self._invalid(context, "Detect duplicated parameter name: %s" % p.name)
            seen.add(p.name)
        try:
            space = SearchSpace.convert(request.experiment)
            self.make_sampler(name, settings_dict(request.experiment.spec.algorithm), space, request)
        except Exception as e:
            abort(context, "INTERNAL", "Failed to create goptuna study and search space: %s" % e)
            return api.ValidateAlgorithmSettingsReply()
        return api.ValidateAlgorithmSettingsReply()


# ==================================================================================== skopt
class SkoptService(_StudyService):
    algorithm_names = ("bayesianoptimization",)

    def make_sampler(self, name, s, space, request):
        if name != "bayesianoptimization":
            raise AlgorithmError("unknown algorithm name {}".format(name))
        return BayesOptSampler(space, int(s["random_state"]) if s.get("random_state") else None,
                               base_estimator=s.get("base_estimator", "GP"),
                               n_initial_points=int(s.get("n_initial_points", 10)),
                               acq_func=s.get("acq_func", "gp_hedge"),
                               acq_optimizer=s.get("acq_optimizer", "auto"))

    def ValidateAlgorithmSettings(self, request, context=None):
        name = request.experiment.spec.algorithm.algorithm_name
        if name != "bayesianoptimization":
            return self._invalid(context, "unknown algorithm name {}".format(name))
        unsupported = lambda k, v: "{} {} is not supported in Bayesian optimization".format(k, v)  # noqa: E731
        err = _check(_pairs(request), {
            "base_estimator": (str, lambda v: v in ("GP", "RF", "ET", "GBRT"), unsupported),
            "n_initial_points": (int, lambda v: v >= 0, "n_initial_points should be great or equal than zero"),
            "acq_func": (str, lambda v: v in BayesOptSampler.ACQS, unsupported),
            "acq_optimizer": (str, lambda v: v in ("auto", "sampling", "lbfgs"), unsupported),
            "random_state": (int, lambda v: v >= 0, "random_state should be great or equal than zero"),
        }, "bayesianoptimization")
        if err is not None:
            return self._invalid(context, err)
        return api.ValidateAlgorithmSettingsReply()
