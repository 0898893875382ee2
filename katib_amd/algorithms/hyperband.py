"""HyperBand suggestion service (reference ``pkg/suggestion/v1beta1/hyperband/service.py:35-354``).

Stateless: all state {eta, s_max, r_l, b_l, r, n, current_s, current_i,
resource_name, evaluating_trials} round-trips through
``GetSuggestionsReply.algorithm`` -> ``Suggestion.status.algorithmSettings`` and
comes back overlaid on the experiment's settings in the next request.

Master bracket: ``n`` uniform samples with the resource parameter set to ``r``.
Child bracket: top ``ceil(n_i/eta)`` of the last ``evaluating_trials`` trials
(sorted by start time) with the resource set to ``r*eta^i``.
``n`` is overwritten by ``current_request_number`` (the reference's "hack").

Documented divergence: the reference raises while the previous rung's trials are
still running (``_get_top_trial``) and its controller rejects a reply with fewer
assignments than requested (``suggestionclient.go:124-128``), so a child bracket
smaller than ``parallelTrialCount`` livelocks there. Here a pending rung returns an
empty reply (the scheduler waits; :meth:`finished_on_empty` tells it the outer loop
is not done) and the scheduler accepts short batches from this service
(``partial_batches``), lowering the Suggestion's request count to what was served.
Completed-but-unsuccessful trials of a rung rank last instead of blocking it.
"""

from __future__ import annotations

import math

import numpy as np

from ..rpc import api_pb2 as api
from .internal import SuggestionService, abort, convert_parameter, format_value


class HyperBandParam:
    def __init__(self, eta=3, s_max=-1, r_l=-1, b_l=-1, r=-1, n=-1, current_s=-2, current_i=-1, resource_name="",
                 evaluating_trials=0):
        self.eta, self.s_max, self.r_l, self.b_l, self.r, self.n = eta, s_max, r_l, b_l, r, n
        self.current_s, self.current_i = current_s, current_i
        self.resource_name, self.evaluating_trials = resource_name, evaluating_trials

    @staticmethod
    def generate(p):
        names = ["eta", "s_max", "r_l", "b_l", "r", "n", "current_s", "current_i", "resource_name",
                 "evaluating_trials"]
        return api.AlgorithmSpec(algorithm_settings=[
            api.AlgorithmSetting(name=k, value=(p.resource_name if k == "resource_name" else str(getattr(p, k))))
            for k in names])

    @staticmethod
    def convert(settings):
        p = HyperBandParam()
        for s in settings:
            if s.name == "eta":
                p.eta = float(s.value)
            elif s.name == "r_l":
                p.r_l = float(s.value)
            elif s.name == "b_l":
                p.b_l = float(s.value)
            elif s.name == "n":
                p.n = int(float(s.value))
            elif s.name == "r":
                p.r = int(float(s.value))
            elif s.name == "current_s":
                p.current_s = int(float(s.value))
            elif s.name == "current_i":
                p.current_i = int(float(s.value))
            elif s.name == "s_max":
                p.s_max = int(float(s.value))
            elif s.name == "evaluating_trials":
                p.evaluating_trials = int(float(s.value))
            elif s.name == "resource_name":
                p.resource_name = s.value
        if p.current_s == -1:
            return p  # outer loop finished
        if p.eta <= 0:
            p.eta = 3
        if p.s_max < 0:
            p.s_max = int(math.log(p.r_l) / math.log(p.eta))
        if p.b_l < 0:
            p.b_l = (p.s_max + 1) * p.r_l
        if p.current_s < 0:
            p.current_s = p.s_max
        if p.current_i < 0:
            p.current_i = 0
        if p.n < 0:
            p.n = int(math.ceil(float(p.s_max + 1) * (float(p.eta ** p.current_s) / float(p.current_s + 1))))
        if p.r < 0:
            p.r = p.r_l * p.eta ** (-p.current_s)
        return p


class _RungPending(Exception):
    pass


class HyperbandService(SuggestionService):
    algorithm_names = ("hyperband",)
    partial_batches = True

    def __init__(self, seed=None):
        self.rng = np.random.RandomState(seed)
        self.all_trials = []
        self.finished = False

    def finished_on_empty(self) -> bool:
        return self.finished

    def GetSuggestions(self, request, context=None):
        reply = api.GetSuggestionsReply()
        experiment = request.experiment
        self.all_trials = list(request.trials)
        param = HyperBandParam.convert(experiment.spec.algorithm.algorithm_settings)
        if param.current_s < 0:
            self.finished = True
            return reply  # outer loop finished
        param.n = request.current_request_number
        try:
            specs = self._make_bracket(experiment, param)
        except _RungPending:
            return api.GetSuggestionsReply()  # state unchanged; asked again once the rung completes
        for spec in specs:
            reply.parameter_assignments.add(assignments=spec)
        reply.algorithm.CopyFrom(HyperBandParam.generate(param))
        return reply

    def _update(self, p):
        p.current_i += 1
        if p.current_i > p.current_s:
            self._new(p)

    def _new(self, p):
        p.current_s -= 1
        p.current_i = 0
        if p.current_s >= 0:
            p.n = int(math.ceil(float(p.s_max + 1) * (float(p.eta ** p.current_s) / float(p.current_s + 1))))
            p.r = p.r_l * p.eta ** (-p.current_s)

    def _make_bracket(self, experiment, p):
        specs = self._master(experiment, p) if p.evaluating_trials == 0 else self._child(experiment, p)
        p.evaluating_trials = len(specs) if p.current_i < p.current_s else 0
        if p.evaluating_trials == 0:
            self._new(p)
        return specs

    def _child(self, experiment, p):
        n_i = math.ceil(p.n * p.eta ** (-p.current_i))
        top = int(math.ceil(n_i / p.eta))
        self._update(p)
        r_i = int(p.r * p.eta ** p.current_i)
        last = self._top_trials(p.evaluating_trials, top, experiment)
        out = []
        for t in last:
            out.append([api.ParameterAssignment(name=a.name, value=str(r_i) if a.name == p.resource_name else a.value)
                        for a in t.spec.parameter_assignments.assignments])
        return out

    def _top_trials(self, latest_n, top_n, experiment):
        obj = experiment.spec.objective.objective_metric_name

        rev = experiment.spec.objective.type == api.MAXIMIZE
        worst = float("-inf") if rev else float("inf")

        def value(t):
            if t.status.condition != api.TrialStatus.SUCCEEDED:
                return worst
            for m in t.status.observation.metrics:
                if m.name == obj:
                    try:
                        return float(m.value)
                    except ValueError:
                        return worst
            return worst

        latest = sorted(self.all_trials, key=lambda t: t.status.start_time)
        if len(latest) > latest_n:
            latest = latest[-latest_n:]
        if len(latest) < latest_n or any(t.status.condition in (api.TrialStatus.CREATED, api.TrialStatus.RUNNING)
                                         for t in latest):
            raise _RungPending()
        return sorted(latest, key=value, reverse=rev)[:top_n]

    def _master(self, experiment, p):
        r = int(p.r)
        params = [convert_parameter(x) for x in experiment.spec.parameter_specs.parameters]
        out = []
        for _ in range(p.n):
            row = []
            for prm in params:
                v = str(r) if prm.name == p.resource_name else format_value(prm.sample_uniform(self.rng))
                row.append(api.ParameterAssignment(name=prm.name, value=v))
            out.append(row)
        return out

    def ValidateAlgorithmSettings(self, request, context=None):
        params = request.experiment.spec.parameter_specs.parameters
        sd = {s.name: s.value for s in request.experiment.spec.algorithm.algorithm_settings}

        def bad(msg):
            abort(context, "INVALID_ARGUMENT", msg)
            return api.ValidateAlgorithmSettingsReply()

        if "r_l" not in sd or "resource_name" not in sd:
            return bad("r_l and resource_name must be set.")
        try:
            rl = float(sd["r_l"])
        except Exception:
            return bad("r_l must be a positive float number.")
        if rl < 0:
            return bad("r_l must be a positive float number.")
        eta = int(float(sd["eta"])) if "eta" in sd else 3
        if eta <= 0:
            eta = 3
        smax = int(math.log(rl) / math.log(eta))
        max_parallel = int(math.ceil(eta ** smax))
        if request.experiment.spec.parallel_trial_count < max_parallel:
            return bad("parallelTrialCount must be not less than %d." % max_parallel)
        if not any(p.name == sd["resource_name"] for p in params):
            return bad("value of resource_name setting must be in parameters.")
        return api.ValidateAlgorithmSettingsReply()
