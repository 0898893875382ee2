"""Experiment defaulting: the ``/mutate-experiment`` webhook's ``SetDefault()``
(reference ``pkg/apis/controller/experiments/v1beta1/experiment_defaults.go:27-178``)."""

from __future__ import annotations

import copy

from . import constants as C
from .models import (V1beta1CollectorSpec, V1beta1Experiment, V1beta1FileSystemPath, V1beta1MetricStrategy,
                     V1beta1MetricsCollectorSpec, V1beta1SourceSpec, V1HTTPGetAction)


def _default_strategy(obj_type: str) -> str:
    if obj_type == C.OBJECTIVE_MINIMIZE:
        return C.STRATEGY_MIN
    if obj_type == C.OBJECTIVE_MAXIMIZE:
        return C.STRATEGY_MAX
    return C.STRATEGY_LATEST


def set_default(e: V1beta1Experiment) -> V1beta1Experiment:
    spec = e.spec
    # parallel trial count
    if spec.parallel_trial_count is None:
        spec.parallel_trial_count = C.DEFAULT_TRIAL_PARALLEL_COUNT
    # resume policy
    if not spec.resume_policy:
        spec.resume_policy = C.DEFAULT_RESUME_POLICY
    # objective metric strategies
    obj = spec.objective
    if obj is not None:
        if obj.metric_strategies is None:
            obj.metric_strategies = []
        has_obj = False
        named = set()
        for s in obj.metric_strategies:
            if s.name == obj.objective_metric_name:
                has_obj = True
                continue
            named.add(s.name)
        if not has_obj:
            obj.metric_strategies.append(V1beta1MetricStrategy(name=obj.objective_metric_name,
                                                               value=_default_strategy(obj.type)))
        for m in obj.additional_metric_names or []:
            if m not in named:
                obj.metric_strategies.append(V1beta1MetricStrategy(name=m, value=_default_strategy(obj.type)))
    # trial template success / failure conditions
    t = spec.trial_template
    if t is not None and t.trial_spec is not None:
        kind = t.trial_spec.get("kind", "")
        if kind in (C.JOB_KIND_JOB, C.JOB_KIND_LOCAL):
            if not t.success_condition:
                t.success_condition = C.DEFAULT_JOB_SUCCESS_CONDITION
            if not t.failure_condition:
                t.failure_condition = C.DEFAULT_JOB_FAILURE_CONDITION
        elif kind in C.KUBEFLOW_JOB_KINDS:
            if not t.success_condition:
                t.success_condition = C.DEFAULT_KUBEFLOW_JOB_SUCCESS_CONDITION
            if not t.failure_condition:
                t.failure_condition = C.DEFAULT_KUBEFLOW_JOB_FAILURE_CONDITION
            if not t.primary_pod_labels:
                t.primary_pod_labels = copy.deepcopy(C.DEFAULT_KUBEFLOW_JOB_PRIMARY_POD_LABELS)
    # metrics collector
    if spec.metrics_collector_spec is None:
        spec.metrics_collector_spec = V1beta1MetricsCollectorSpec()
    mc = spec.metrics_collector_spec
    if mc.collector is None:
        mc.collector = V1beta1CollectorSpec(kind=C.COLLECTOR_STDOUT)
    kind = mc.collector.kind
    if kind == C.COLLECTOR_PROMETHEUS:
        if mc.source is None:
            mc.source = V1beta1SourceSpec()
        if mc.source.http_get is None:
            mc.source.http_get = V1HTTPGetAction()
        if not mc.source.http_get.path:
            mc.source.http_get.path = C.DEFAULT_PROMETHEUS_PATH
        if mc.source.http_get.port in (None, 0, "0", ""):
            mc.source.http_get.port = C.DEFAULT_PROMETHEUS_PORT
    elif kind == C.COLLECTOR_FILE:
        if mc.source is None:
            mc.source = V1beta1SourceSpec()
        if mc.source.file_system_path is None:
            mc.source.file_system_path = V1beta1FileSystemPath()
        fsp = mc.source.file_system_path
        if not fsp.kind:
            fsp.kind = C.FS_KIND_FILE
        if not fsp.path:
            fsp.path = C.DEFAULT_FILE_PATH
        if not fsp.format:
            fsp.format = C.FORMAT_TEXT
    elif kind == C.COLLECTOR_TFEVENT:
        if mc.source is None:
            mc.source = V1beta1SourceSpec()
        if mc.source.file_system_path is None:
            mc.source.file_system_path = V1beta1FileSystemPath()
        fsp = mc.source.file_system_path
        if not fsp.kind:
            fsp.kind = C.FS_KIND_DIRECTORY
        if not fsp.path:
            fsp.path = C.DEFAULT_TFEVENT_DIR_PATH
    return e
