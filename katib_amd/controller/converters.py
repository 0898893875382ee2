"""CRD <-> gRPC converters (reference ``suggestionclient.go:297-555``, ``nas.go:24-61``,
``algorithm_settings.go:28-68``)."""

from __future__ import annotations

from typing import List

from ..api import constants as C
from ..api.conditions import TrialConditions as TC
from ..api.models import format_time
from ..rpc import api_pb2 as api

_PTYPE = {C.PARAMETER_DOUBLE: api.DOUBLE, C.PARAMETER_INT: api.INT, C.PARAMETER_DISCRETE: api.DISCRETE,
          C.PARAMETER_CATEGORICAL: api.CATEGORICAL}
_OTYPE = {C.OBJECTIVE_MAXIMIZE: api.MAXIMIZE, C.OBJECTIVE_MINIMIZE: api.MINIMIZE}
_TCOND = {C.TRIAL_CREATED: api.TrialStatus.CREATED, C.TRIAL_RUNNING: api.TrialStatus.RUNNING,
          C.TRIAL_SUCCEEDED: api.TrialStatus.SUCCEEDED, C.TRIAL_KILLED: api.TrialStatus.KILLED,
          C.TRIAL_FAILED: api.TrialStatus.FAILED, C.TRIAL_EARLY_STOPPED: api.TrialStatus.EARLYSTOPPED}
_CMP_FROM_PB = {api.EQUAL: C.COMPARISON_EQUAL, api.LESS: C.COMPARISON_LESS, api.GREATER: C.COMPARISON_GREATER}


def convert_parameters(params) -> List:
    out = []
    for p in params or []:
        fs = p.feasible_space
        out.append(api.ParameterSpec(
            name=p.name or "", parameter_type=_PTYPE.get(p.parameter_type, api.UNKNOWN_TYPE),
            feasible_space=api.FeasibleSpace(max=fs.max or "", min=fs.min or "", list=list(fs.list or []),
                                             step=fs.step or "") if fs else None))
    return out


def convert_nas_config(nas):
    gc = nas.graph_config
    ops = []
    for o in nas.operations or []:
        ops.append(api.Operation(operation_type=o.operation_type or "",
                                 parameter_specs=api.Operation.ParameterSpecs(
                                     parameters=convert_parameters(o.parameters))))
    return api.NasConfig(graph_config=api.GraphConfig(num_layers=(gc.num_layers or 0) if gc else 0,
                                                      input_sizes=list((gc.input_sizes or []) if gc else []),
                                                      output_sizes=list((gc.output_sizes or []) if gc else [])),
                         operations=api.NasConfig.Operations(operation=ops))


def convert_experiment(e, extra_settings=None):
    """``extra_settings`` (Suggestion.status.algorithmSettings) overwrite/append the
    experiment's algorithm settings (appendAlgorithmSettingsFromSuggestion)."""
    s = e.spec
    settings = [(x.name, x.value) for x in (s.algorithm.algorithm_settings or [])]
    for es in extra_settings or []:
        for i, (n, _) in enumerate(settings):
            if n == es.name:
                settings[i] = (n, es.value)
                break
        else:
            settings.append((es.name, es.value))
    obj = s.objective
    spec = api.ExperimentSpec(
        algorithm=api.AlgorithmSpec(algorithm_name=s.algorithm.algorithm_name,
                                    algorithm_settings=[api.AlgorithmSetting(name=n, value=v or "")
                                                        for n, v in settings]),
        objective=api.ObjectiveSpec(type=_OTYPE.get(obj.type, api.UNKNOWN),
                                    objective_metric_name=obj.objective_metric_name or "",
                                    additional_metric_names=list(obj.additional_metric_names or [])),
        parameter_specs=api.ExperimentSpec.ParameterSpecs(parameters=convert_parameters(s.parameters)))
    if obj.goal is not None:
        spec.objective.goal = float(obj.goal)
    if s.nas_config is not None:
        spec.nas_config.CopyFrom(convert_nas_config(s.nas_config))
    if s.parallel_trial_count is not None:
        spec.parallel_trial_count = s.parallel_trial_count
    if s.max_trial_count is not None:
        spec.max_trial_count = s.max_trial_count
    if s.early_stopping is not None:
        spec.early_stopping.CopyFrom(api.EarlyStoppingSpec(
            algorithm_name=s.early_stopping.algorithm_name,
            algorithm_settings=[api.EarlyStoppingSetting(name=x.name, value=x.value or "")
                                for x in s.early_stopping.algorithm_settings or []]))
    return api.Experiment(name=e.metadata.name, spec=spec)


def _observation(strategies, obs):
    smap = {x.name: x.value for x in strategies or []}
    out = api.Observation()
    if obs is not None and obs.metrics:
        for m in obs.metrics:
            st = smap.get(m.name)
            if st == C.STRATEGY_MIN:
                v = m.latest if m.min == C.UNAVAILABLE_METRIC_VALUE else m.min
            elif st == C.STRATEGY_MAX:
                v = m.latest if m.max == C.UNAVAILABLE_METRIC_VALUE else m.max
            elif st == C.STRATEGY_LATEST:
                v = m.latest
            else:
                v = ""
            out.metrics.add(name=m.name, value=v or "")
    return out


def convert_trials(trials) -> List:
    out = []
    for t in trials:
        if TC.is_metrics_unavailable(t):
            continue
        if not TC.is_observation_available(t) and TC.is_early_stopped(t):
            continue
        obj = t.spec.objective
        pt = api.Trial(name=t.metadata.name, spec=api.TrialSpec(
            objective=api.ObjectiveSpec(type=_OTYPE.get(obj.type, api.UNKNOWN),
                                        objective_metric_name=obj.objective_metric_name or "",
                                        additional_metric_names=list(obj.additional_metric_names or [])),
            parameter_assignments=api.TrialSpec.ParameterAssignments(
                assignments=[api.ParameterAssignment(name=a.name, value=a.value or "")
                             for a in t.spec.parameter_assignments or []])))
        if t.spec.labels:
            for k, v in t.spec.labels.items():
                pt.spec.labels[k] = v
        if obj.goal is not None:
            pt.spec.objective.goal = float(obj.goal)
        st = t.status
        pt.status.start_time = format_time(st.start_time) if st and st.start_time else ""
        pt.status.completion_time = format_time(st.completion_time) if st and st.completion_time else ""
        pt.status.observation.CopyFrom(_observation(obj.metric_strategies, st.observation if st else None))
        if st and st.conditions:
            pt.status.condition = _TCOND.get(st.conditions[-1].type, api.TrialStatus.UNKNOWN)
        out.append(pt)
    return out


def comparison_from_pb(c) -> str:
    return _CMP_FROM_PB.get(c, C.COMPARISON_EQUAL)
