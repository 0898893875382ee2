"""Shared helpers for every suggestion service (reference
``pkg/suggestion/v1beta1/internal/{search_space,trial,constant}.py``).

* :class:`SearchSpace` parses ``experiment.spec.parameter_specs`` once into typed
  :class:`Param` objects (INT step defaults to 1; DOUBLE step optional) and maps
  values to/from a numeric *internal* coordinate (float, index for categorical /
  discrete) used by the model-based samplers.
* :func:`convert_trials` keeps SUCCEEDED and EARLYSTOPPED trials that carry the
  objective metric (``internal/trial.py:34-71``).
* :func:`make_reply_assignments` builds ``GetSuggestionsReply.ParameterAssignments``
  with optional ``trial_name`` / ``labels`` (``internal/trial.py:87-114``).
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..rpc import api_pb2 as api

MAX_GOAL = "MAXIMIZE"
MIN_GOAL = "MINIMIZE"
INTEGER = "INTEGER"
DOUBLE = "DOUBLE"
CATEGORICAL = "CATEGORICAL"
DISCRETE = "DISCRETE"


class AlgorithmError(Exception):
    """Raised by services; ``code`` is a grpc.StatusCode name."""

    def __init__(self, message: str, code: str = "INVALID_ARGUMENT"):
        super().__init__(message)
        self.code = code
        self.message = message


def format_value(v) -> str:
    """Value -> assignment string: ints as ints, floats with Go 'f' shortest-repr."""
    if isinstance(v, (bool, np.bool_)):
        return str(v)
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        f = float(v)
        r = repr(f)
        if "e" in r or "E" in r:
            # strconv.FormatFloat(f, 'f', -1, 64): no exponent
            r = np.format_float_positional(f, trim="-")
        return r
    return str(v)


@dataclass
class Param:
    name: str
    type: str
    min: float = 0.0
    max: float = 0.0
    step: Optional[float] = None
    list: List[str] = field(default_factory=list)
    raw_min: str = ""
    raw_max: str = ""
    raw_step: str = ""

    @property
    def is_numeric(self) -> bool:
        return self.type in (INTEGER, DOUBLE)

    # ---- internal coordinates -------------------------------------------------------
    def to_internal(self, value: str) -> float:
        if self.type == INTEGER:
            return float(int(float(value)))
        if self.type == DOUBLE:
            return float(value)
        try:
            return float(self.list.index(str(value)))
        except ValueError:
            return float("nan")

    def from_internal(self, x: float):
        if self.type == INTEGER:
            step = int(self.step or 1)
            lo, hi = int(self.min), int(self.max)
            k = int(round((x - lo) / step))
            v = lo + k * step
            while v > hi:
                v -= step
            return max(v, lo)
        if self.type == DOUBLE:
            x = min(max(float(x), self.min), self.max)
            if self.step:
                k = round((x - self.min) / self.step)
                x = min(self.min + k * self.step, self.max)
            return float(x)
        idx = int(round(x))
        idx = min(max(idx, 0), len(self.list) - 1)
        return self.list[idx]

    def grid(self) -> list:
        """Enumerated values (convert_to_combinations, search_space.py:45-66)."""
        if self.type == INTEGER:
            return list(range(int(self.min), int(self.max) + 1, int(self.step or 1)))
        if self.type == DOUBLE:
            if not self.step:
                raise AlgorithmError(
                    "Param {} step is nil; For discrete search space, all parameters must include step".format(
                        self.name))
            vals = np.arange(self.min, self.max + self.step, self.step)
            if len(vals) and vals[-1] > self.max:
                vals = vals[:-1]
            return [float(v) for v in vals]
        return list(self.list)

    def sample_uniform(self, rng: np.random.RandomState):
        if self.type == INTEGER:
            step = int(self.step or 1)
            n = (int(self.max) - int(self.min)) // step
            return int(self.min) + step * int(rng.randint(0, n + 1))
        if self.type == DOUBLE:
            if self.step:
                n = int(math.floor((self.max - self.min) / self.step + 1e-9))
                return float(self.min + self.step * rng.randint(0, n + 1))
            return float(rng.uniform(self.min, self.max))
        return self.list[int(rng.randint(0, len(self.list)))]


class SearchSpace:
    def __init__(self, goal: str, params: List[Param]):
        self.goal = goal
        self.params = params

    @staticmethod
    def convert(experiment) -> "SearchSpace":
        goal = ""
        if experiment.spec.objective.type == api.MAXIMIZE:
            goal = MAX_GOAL
        elif experiment.spec.objective.type == api.MINIMIZE:
            goal = MIN_GOAL
        return SearchSpace(goal, [convert_parameter(p) for p in experiment.spec.parameter_specs.parameters])

    def names(self) -> List[str]:
        return [p.name for p in self.params]

    def __len__(self):
        return len(self.params)

    def combinations(self) -> Dict[str, list]:
        return {p.name: p.grid() for p in self.params}


def convert_parameter(p) -> Param:
    fs = p.feasible_space
    if p.parameter_type == api.INT:
        step = fs.step if fs.step not in (None, "") else "1"
        return Param(p.name, INTEGER, float(int(float(fs.min))), float(int(float(fs.max))), float(int(float(step))),
                     raw_min=fs.min, raw_max=fs.max, raw_step=step)
    if p.parameter_type == api.DOUBLE:
        return Param(p.name, DOUBLE, float(fs.min), float(fs.max), float(fs.step) if fs.step else None,
                     raw_min=fs.min, raw_max=fs.max, raw_step=fs.step)
    if p.parameter_type == api.CATEGORICAL:
        return Param(p.name, CATEGORICAL, list=[str(e) for e in fs.list])
    if p.parameter_type == api.DISCRETE:
        return Param(p.name, DISCRETE, list=[str(e) for e in fs.list])
    raise AlgorithmError("Cannot get the type for the parameter: {} ({})".format(p.name, p.parameter_type))


@dataclass
class Metric:
    name: str
    value: str


@dataclass
class Trial:
    name: str
    assignments: Dict[str, str]
    target_metric: Metric
    metric_name: str
    additional_metrics: List[Metric]
    labels: Dict[str, str]
    condition: int = 0

    def objective(self) -> Optional[float]:
        try:
            return float(self.target_metric.value)
        except (TypeError, ValueError):
            return None


def convert_trials(trials, include_states=(api.TrialStatus.SUCCEEDED, api.TrialStatus.EARLYSTOPPED)) -> List[Trial]:
    out = []
    for t in trials:
        if t.status.condition not in include_states:
            continue
        name = t.spec.objective.objective_metric_name
        target, extra = None, []
        for m in t.status.observation.metrics:
            if m.name == name:
                target = Metric(m.name, m.value)
            else:
                extra.append(Metric(m.name, m.value))
        if target is None:
            continue
        out.append(Trial(t.name, {a.name: a.value for a in t.spec.parameter_assignments.assignments},
                         target, name, extra, dict(t.spec.labels), t.status.condition))
    return out


def numeric_losses(trials: Sequence[Trial], goal: str):
    """(trials, losses) with non-numeric objectives dropped; maximisation negated."""
    keep, losses = [], []
    for t in trials:
        v = t.objective()
        if v is None or math.isnan(v):
            continue
        keep.append(t)
        losses.append(-v if goal == MAX_GOAL else v)
    return keep, losses


def make_reply_assignments(list_of_assignments, trial_names=None, labels=None):
    if trial_names is not None and len(list_of_assignments) != len(trial_names):
        raise RuntimeError("Assignment and trial list length mismatch")
    res = []
    for n, assignments in enumerate(list_of_assignments):
        items = assignments.items() if isinstance(assignments, dict) else assignments
        buf = [api.ParameterAssignment(name=k, value=format_value(v)) for k, v in items]
        kwargs = {"assignments": buf}
        if trial_names is not None:
            kwargs["trial_name"] = trial_names[n]
        if labels is not None:
            kwargs["labels"] = {k: str(v) for k, v in labels[n].items()}
        res.append(api.GetSuggestionsReply.ParameterAssignments(**kwargs))
    return res


def settings_dict(algorithm_spec) -> Dict[str, str]:
    return {s.name: s.value for s in algorithm_spec.algorithm_settings}


def seed_from(settings: Dict[str, str], key: str = "random_state") -> Optional[int]:
    v = settings.get(key)
    if v is None or v == "":
        return None
    return int(v)


class SuggestionService:
    """Base class of in-process suggestion services.

    Method names and request/reply types are those of the gRPC ``Suggestion``
    service, so the same object is served in-process by the scheduler and over
    gRPC by :mod:`katib_amd.rpc.server` (``context`` is optional)."""

    algorithm_names: Sequence[str] = ()

    def GetSuggestions(self, request, context=None):
        raise NotImplementedError

    def ValidateAlgorithmSettings(self, request, context=None):
        return api.ValidateAlgorithmSettingsReply()

    # algorithms that run out of configurations (grid) report exhaustion here
    def is_exhausted(self) -> bool:
        return False

    # an empty GetSuggestions reply means "search finished" unless a service overrides this
    def finished_on_empty(self) -> bool:
        return True


def abort(context, code: str, message: str):
    """Report an error the gRPC way when a context exists, else raise."""
    if context is not None and hasattr(context, "set_code"):
        import grpc

        context.set_code(getattr(grpc.StatusCode, code))
        context.set_details(message)
        return None
    raise AlgorithmError(message, code)
