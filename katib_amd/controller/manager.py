"""The node-local Katib control plane.

One :class:`Manager` per MI355X node replaces katib-controller (experiment,
suggestion and trial reconcilers), the admission webhooks, the per-experiment
suggestion Deployments, katib-db-manager and the metrics-collector sidecars
(SURVEY §1 "MI355X mapping"). It owns:

* the object store of Experiments / Trials / Suggestions (v1beta1 models),
* the native observation store and trial runtime (``katib_amd._native``),
* the GPU slot pool and the warm per-GPU worker processes,
* in-process suggestion and early-stopping services.

A single-threaded event loop (:meth:`step`) owns all mutable state; SDK calls
from other threads take the same lock. Reconcile semantics follow the reference
controllers line by line - see the citations on each method.
"""

from __future__ import annotations

import json
import logging
import os
import random
import shutil
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from .. import native
from ..algorithms.internal import AlgorithmError
from ..algorithms.registry import create_early_stopping, create_service
from ..api import constants as C
from ..api.conditions import ExperimentConditions as EC
from ..api.conditions import SuggestionConditions as SC
from ..api.conditions import TrialConditions as TC
from ..api.defaults import set_default
from ..api.models import (V1beta1AlgorithmSetting, V1beta1EarlyStoppingRule, V1beta1Experiment,
                          V1beta1ExperimentStatus, V1beta1Metric, V1beta1Observation, V1beta1OptimalTrial,
                          V1beta1ParameterAssignment, V1beta1Suggestion, V1beta1SuggestionSpec,
                          V1beta1SuggestionStatus, V1beta1Trial, V1beta1TrialAssignment, V1beta1TrialSpec,
                          V1beta1TrialStatus, V1ObjectMeta, now)
from ..api.validation import ValidationError, validate_experiment
from ..rpc import api_pb2 as api
from ..utils.prometheus import Registry
from ..utils.tracing import Tracer
from . import gjson
from . import status_engine as SE
from .config import KatibConfig
from .converters import comparison_from_pb, convert_experiment, convert_trials
from .jobs import JobSpecError, LaunchPlan, assign_ports, job_status, make_plan, map_paths, path_mapping
from .manifest import ConfigMapStore, Generator

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
log = logging.getLogger("katib_amd.controller")

_RAND_ALPHABET = "bcdfghjklmnpqrstvwxz2456789"  # k8s utilrand.String alphabet
_KIND_CODES = {C.COLLECTOR_STDOUT: 0, C.COLLECTOR_FILE: 1, C.COLLECTOR_TFEVENT: 2, C.COLLECTOR_NONE: 3,
               C.COLLECTOR_CUSTOM: 4, C.COLLECTOR_PROMETHEUS: 5}
_CMP_CODES = {C.COMPARISON_EQUAL: 0, C.COMPARISON_LESS: 1, C.COMPARISON_GREATER: 2}

Key = Tuple[str, str]


@dataclass
class TrialRun:
    """Runtime bookkeeping of a trial's job (the 'Job object')."""
    plan: Optional[LaunchPlan] = None
    devices: List[int] = field(default_factory=list)
    cpu_slot: bool = False
    phase: str = "Pending"  # Pending | Launching | Running | Succeeded | Failed
    reason: str = ""
    message: str = ""
    attempt: int = 0
    worker: Optional[int] = None
    aux: List[str] = field(default_factory=list)
    trial_dir: str = ""
    early_stopped: bool = False
    started: float = 0.0
    finished: float = 0.0
    collector: Dict = field(default_factory=dict)
    path_map: Dict[str, str] = field(default_factory=dict)
    deleted: bool = False
    scraper: Optional[object] = None  # PrometheusMetric collector (metricscollector/prometheus.py)
    prom_final: str = ""  # KATIB_PROMETHEUS_FINAL snapshot path
    launcher: str = ""  # "exec" (fork + exec) or "zygote" (forked from the fork server)


@dataclass
class WorkerInfo:
    wid: int
    device_key: str
    busy: Optional[str] = None
    ready: bool = False
    pending: Optional[Tuple] = None  # (trial key, payload, log, collector, deadline)


class Manager:
    def __init__(self, config: Optional[KatibConfig] = None, state_dir: Optional[str] = None,
                 namespace: str = "default", num_devices: Optional[int] = None, journal: bool = True):
        self.config = config or KatibConfig()
        if state_dir:
            self.config.amd.state_dir = state_dir
        if num_devices is not None:
            self.config.amd.num_devices = num_devices
        self.state_dir = self.config.amd.state_dir
        os.makedirs(self.state_dir, exist_ok=True)
        self.namespace = namespace
        self.N = native.load()
        self.store = self.N.ObservationStore()
        self._journal = journal
        if journal:
            jpath = os.path.join(self.state_dir, "observations.jsonl")
            if os.path.exists(jpath):
                self.store.load_journal(jpath)
            self.store.open_journal(jpath)
        self.runtime = self.N.TrialRuntime(self.store)
        self.n_devices = self.config.devices()
        self.slots = self.N.SlotPool(self.n_devices, self.config.amd.slots_per_device)
        self.cpu_slots_used = 0
        self.configmaps = ConfigMapStore()
        self.generator = Generator(self.configmaps)
        self.metrics = Registry()
        self.events: List[Dict] = []
        self.experiments: Dict[Key, V1beta1Experiment] = {}
        self.trials: Dict[Key, V1beta1Trial] = {}
        self.suggestions: Dict[Key, V1beta1Suggestion] = {}
        self.services: Dict[Key, object] = {}
        self.es_services: Dict[Key, object] = {}
        self.runs: Dict[Key, TrialRun] = {}
        self.workers: Dict[int, WorkerInfo] = {}
        self._proc_to_trial: Dict[str, Key] = {}
        self._lock = threading.RLock()
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._zygote = None  # fork server for cold Python trials (controller/zygote.py)
        self._zygote_failed = False
        self._zygote_thread: Optional[threading.Thread] = None
        self._t0 = time.time()
        self._completed = 0
        self.fault_injector: Optional[Callable[[str, Key], bool]] = None
        self.tracer = Tracer()  # trial / suggestion timeline (utils/tracing.py)
        self._install_default_templates()

    # ============================================================== public API (apiserver)
    def _key(self, name: str, namespace: Optional[str] = None) -> Key:
        return (namespace or self.namespace, name)

    def create_experiment(self, exp: V1beta1Experiment, namespace: Optional[str] = None) -> V1beta1Experiment:
        with self._lock:
            exp = exp.deepcopy()
            if exp.metadata is None:
                exp.metadata = V1ObjectMeta()
            exp.metadata.namespace = exp.metadata.namespace or namespace or self.namespace
            exp.api_version = exp.api_version or C.API_VERSION
            exp.kind = exp.kind or C.KIND_EXPERIMENT
            key = (exp.metadata.namespace, exp.metadata.name)
            if key in self.experiments:
                raise ValueError('experiments.kubeflow.org "%s" already exists' % exp.metadata.name)
            set_default(exp)  # /mutate-experiment
            self._validate(exp)  # /validate-experiment
            exp.metadata.creation_timestamp = now()
            exp.metadata.uid = "%032x" % random.getrandbits(128)
            exp.metadata.generation = 1
            exp.status = exp.status or V1beta1ExperimentStatus()
            self.experiments[key] = exp
            self._event(exp, "Normal", "Created", "Experiment created")
            self._persist(key)
            return exp.deepcopy()

    def _validate(self, exp, old=None):
        validate_experiment(exp, old, suggestion_algorithms=set(self.config.suggestions),
                            early_stopping_algorithms=set(self.config.early_stoppings),
                            template_getter=self.generator.get_trial_template,
                            metrics_collectors=set(self.config.metrics_collectors))

    def update_experiment(self, exp: V1beta1Experiment) -> V1beta1Experiment:
        with self._lock:
            key = (exp.metadata.namespace or self.namespace, exp.metadata.name)
            old = self.experiments.get(key)
            if old is None:
                raise KeyError('experiments.kubeflow.org "%s" not found' % exp.metadata.name)
            new = exp.deepcopy()
            new.status = old.status
            new.metadata = old.metadata
            set_default(new)
            self._validate(new, old.deepcopy())
            new.metadata.generation = (old.metadata.generation or 1) + 1
            self.experiments[key] = new
            self._persist(key)
            return new.deepcopy()

    def get_experiment(self, name: str, namespace: Optional[str] = None) -> V1beta1Experiment:
        with self._lock:
            e = self.experiments.get(self._key(name, namespace))
            if e is None:
                raise KeyError('experiments.kubeflow.org "%s" not found' % name)
            return e.deepcopy()

    def list_experiments(self, namespace: Optional[str] = None) -> List[V1beta1Experiment]:
        with self._lock:
            ns = namespace or self.namespace
            return [e.deepcopy() for (n, _), e in sorted(self.experiments.items()) if n == ns]

    def delete_experiment(self, name: str, namespace: Optional[str] = None):
        with self._lock:
            key = self._key(name, namespace)
            exp = self.experiments.get(key)
            if exp is None:
                raise KeyError('experiments.kubeflow.org "%s" not found' % name)
            for tkey in [k for k, t in self.trials.items() if self._owner(t) == key]:
                self._delete_trial(tkey)
            self.suggestions.pop(key, None)
            self.services.pop(key, None)
            self.es_services.pop(key, None)
            del self.experiments[key]
            self.metrics.inc("katib_experiment_deleted_total", namespace=key[0])
            self._event(exp, "Normal", "Deleted", "Experiment deleted")
            p = self._journal_path(key)
            if os.path.exists(p):
                os.remove(p)

    def get_trial(self, name: str, namespace: Optional[str] = None) -> V1beta1Trial:
        with self._lock:
            t = self.trials.get(self._key(name, namespace))
            if t is None:
                raise KeyError('trials.kubeflow.org "%s" not found' % name)
            return t.deepcopy()

    def list_trials(self, experiment_name: Optional[str] = None, namespace: Optional[str] = None) -> List[V1beta1Trial]:
        with self._lock:
            ns = namespace or self.namespace
            out = []
            for (n, _), t in self.trials.items():
                if n != ns:
                    continue
                if experiment_name and (t.metadata.labels or {}).get(C.LABEL_EXPERIMENT_NAME) != experiment_name:
                    continue
                out.append(t.deepcopy())
            out.sort(key=lambda t: t.metadata.creation_timestamp)
            return out

    def get_suggestion(self, name: str, namespace: Optional[str] = None) -> V1beta1Suggestion:
        with self._lock:
            s = self.suggestions.get(self._key(name, namespace))
            if s is None:
                raise KeyError('suggestions.kubeflow.org "%s" not found' % name)
            return s.deepcopy()

    def list_suggestions(self, namespace: Optional[str] = None) -> List[V1beta1Suggestion]:
        with self._lock:
            ns = namespace or self.namespace
            return [s.deepcopy() for (n, _), s in sorted(self.suggestions.items()) if n == ns]

    def kill_trial(self, name: str, namespace: Optional[str] = None):
        """Kill a running trial: it ends in the Killed condition."""
        with self._lock:
            key = self._key(name, namespace)
            run = self.runs.get(key)
            if run is None or run.phase not in ("Running", "Launching", "Pending"):
                return False
            run.reason, run.message = C.TRIAL_KILLED_REASON, "Trial is killed by user"
            trial = self.trials[key]
            TC.mark_killed(trial, C.TRIAL_KILLED_REASON, "Trial is killed")
            trial.status.completion_time = now()
            self._stop_job(key)
            return True

    def get_observation_log(self, trial_name: str, metric_name: str = "", start_time: str = "", end_time: str = ""):
        return self.store.get(trial_name, metric_name, start_time, end_time)

    def report_observation_log(self, trial_name: str, logs):
        self.store.report(trial_name, logs)

    def delete_observation_log(self, trial_name: str):
        self.store.remove(trial_name)

    def set_trial_early_stopped(self, trial_name: str, namespace: Optional[str] = None):
        """EarlyStopping.SetTrialStatus equivalent (medianstop/service.py:184-238)."""
        with self._lock:
            t = self.trials.get(self._key(trial_name, namespace))
            if t is not None and not TC.is_early_stopped(t):
                TC.mark_early_stopped(t, C.TRIAL_EARLY_STOPPED_REASON, "Trial is early stopped")

    def add_configmap(self, namespace: str, name: str, data: Dict[str, str], labels=None):
        self.configmaps.put(namespace, name, data, labels)

    # ============================================================== event loop
    def step(self, timeout_ms: Optional[int] = None) -> bool:
        """One scheduler iteration. Returns True while any experiment is active."""
        if timeout_ms is None:
            timeout_ms = self.config.amd.poll_interval_ms
        events = self.runtime.poll(timeout_ms)
        # PrometheusMetric scrapes are blocking HTTP reads: take the due list under the lock,
        # scrape without it, record the results under it again
        with self._lock:
            due = self._due_scrapes()
        scraped = [(tkey, sc.scrape()) for tkey, sc in due]
        with self._lock:
            for tkey, logs in scraped:
                run = self.runs.get(tkey)
                if logs and run is not None and run.scraper is not None and not run.deleted:
                    self.store.report(tkey[1], logs)
            for ev in events:
                self._on_runtime_event(ev)
            for key in list(self.experiments):
                try:
                    self._reconcile_experiment(key)
                except Exception as e:  # ReconcileError: recorded, retried next iteration
                    log.exception("reconcile %s failed", key)
                    exp = self.experiments.get(key)
                    if exp is not None:
                        self._event(exp, "Warning", C.RECONCILE_ERROR_REASON, "Failed to reconcile: %s" % e)
            self._admit_trials()
            self._update_gauges()
            return any(not EC.is_completed(e) or EC.has_running_trials(e) for e in self.experiments.values())

    def run_until_complete(self, name: str, namespace: Optional[str] = None, timeout: float = 3600.0):
        key = self._key(name, namespace)
        deadline = time.time() + timeout
        while time.time() < deadline:
            self.step()
            e = self.experiments.get(key)
            if e is None:
                raise KeyError(name)
            if EC.is_completed(e) and not any(
                    self.runs.get(k) is not None and self.runs[k].phase in ("Running", "Launching")
                    for k, t in self.trials.items() if self._owner(t) == key):
                self._persist(key)
                return e.deepcopy()
        raise TimeoutError("experiment %s did not complete in %.0fs" % (name, timeout))

    def start(self):
        if self._thread is not None:
            return
        self._stop.clear()

        def loop():
            while not self._stop.is_set():
                self.step()

        self._thread = threading.Thread(target=loop, name="katib-amd-scheduler", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
            self._thread = None

    def shutdown(self):
        self.stop()
        self.runtime.shutdown()
        if self._zygote_thread is not None:
            self._zygote_thread.join(timeout=180)
        if self._zygote is not None:
            self._zygote.close()
            self._zygote = None
        if self._journal:
            self.store.close_journal()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.shutdown()

    # ============================================================== experiment controller
    def _owner(self, trial) -> Optional[Key]:
        exp = (trial.metadata.labels or {}).get(C.LABEL_EXPERIMENT_NAME)
        return (trial.metadata.namespace, exp) if exp else None

    def _exp_trials(self, key: Key) -> List[V1beta1Trial]:
        ts = [t for t in self.trials.values() if self._owner(t) == key]
        ts.sort(key=lambda t: (t.metadata.creation_timestamp, t.metadata.name))
        return ts

    def _reconcile_experiment(self, key: Key):
        """experiment_controller.go:156-247 Reconcile."""
        exp = self.experiments[key]
        fin = exp.metadata.finalizers or []
        if C.FINALIZER_UPDATE_PROMETHEUS_METRICS not in fin:
            exp.metadata.finalizers = fin + [C.FINALIZER_UPDATE_PROMETHEUS_METRICS]
            self.metrics.inc("katib_experiment_created_total", namespace=key[0])
            return
        before = json.dumps(exp.status.to_k8s(), sort_keys=True, default=str)
        if EC.is_completed(exp):
            if exp.spec.resume_policy in (C.RESUME_NEVER, C.RESUME_FROM_VOLUME):
                self._cleanup_suggestion(exp)
            action = SE.plan_restart(EC.is_completed_reason(exp, C.EXPERIMENT_MAX_TRIALS_REACHED_REASON),
                                     exp.spec.resume_policy, exp.spec.max_trial_count, exp.status.trials or 0,
                                     EC.has_running_trials(exp))
            if action == "restart":
                EC.mark_restarting(exp, C.EXPERIMENT_RESTARTING_REASON, "Experiment is restarted")
                if exp.spec.resume_policy == C.RESUME_FROM_VOLUME:
                    self._restart_suggestion(exp)
            elif action == "none":
                return
        if not EC.is_created(exp):
            if exp.status.start_time is None:
                exp.status.start_time = now()
            EC.mark_created(exp, C.EXPERIMENT_CREATED_REASON, "Experiment is created")
        else:
            self._reconcile_experiment_trials(key, exp)
        after = json.dumps(exp.status.to_k8s(), sort_keys=True, default=str)
        if before != after:
            self._persist(key)

    def _reconcile_experiment_trials(self, key, exp):
        """ReconcileExperiment (experiment_controller.go:250-271)."""
        trials = self._exp_trials(key)
        if trials:
            goal = self._update_trials_summary(exp, trials)
            if not EC.is_completed(exp):
                self._update_condition(exp, goal, False)
        if not EC.is_completed(exp):
            self._reconcile_trials(key, exp, trials)

    def _objective_value(self, trial) -> str:
        """getObjectiveMetricValue (status_util.go:151-183), native status engine."""
        return SE.objective_value(trial)

    def _update_trials_summary(self, exp, trials) -> bool:
        """updateTrialsSummary (status_util.go:57-148): bucketing, optimal trial and goal
        are decided by the native status engine (csrc/native/status_engine.cpp)."""
        st = exp.status
        obj = exp.spec.objective
        buckets, best_idx, goal_reached = SE.summarize(trials, obj.type, obj.goal)
        lists = SE.bucket_names(trials, buckets)
        st.trials = len(trials)
        st.killed_trial_list = lists["killed"] or None
        st.failed_trial_list = lists["failed"] or None
        st.succeeded_trial_list = lists["succeeded"] or None
        st.early_stopped_trial_list = lists["early"] or None
        st.running_trial_list = lists["running"] or None
        st.metrics_unavailable_trial_list = lists["mu"] or None
        st.pending_trial_list = lists["pending"] or None
        st.trials_killed = len(lists["killed"])
        st.trials_failed = len(lists["failed"])
        st.trials_succeeded = len(lists["succeeded"])
        st.trials_early_stopped = len(lists["early"])
        st.trials_running = len(lists["running"])
        st.trial_metrics_unavailable = len(lists["mu"])
        st.trials_pending = len(lists["pending"])
        if best_idx != -1:
            b = trials[best_idx]
            st.current_optimal_trial = V1beta1OptimalTrial(
                best_trial_name=b.metadata.name,
                parameter_assignments=[a.deepcopy() for a in b.spec.parameter_assignments or []],
                observation=V1beta1Observation(metrics=[m.deepcopy() for m in (b.status.observation.metrics or [])]))
        return goal_reached

    def _update_condition(self, exp, goal_reached: bool, suggestion_done: bool):
        """UpdateExperimentStatusCondition (status_util.go:187-235); the outcome comes from
        the native status engine."""
        st = exp.status
        ns = exp.metadata.namespace
        outcome = SE.decide_condition(st, goal_reached, suggestion_done, exp.spec.max_failed_trial_count,
                                      exp.spec.max_trial_count)
        if outcome == "running":
            EC.mark_running(exp, C.EXPERIMENT_RUNNING_REASON, "Experiment is running")
            return
        if outcome == "max_failed":
            EC.mark_failed(exp, C.EXPERIMENT_FAILED_REASON, "Experiment has failed because max failed count has reached")
            st.completion_time = now()
            self.metrics.inc("katib_experiment_failed_total", namespace=ns)
            return
        reason, msg = {
            "goal": (C.EXPERIMENT_GOAL_REACHED_REASON, "Experiment has succeeded because Objective goal has reached"),
            "max_trials": (C.EXPERIMENT_MAX_TRIALS_REACHED_REASON,
                           "Experiment has succeeded because max trial count has reached"),
            "suggestion_end": (C.EXPERIMENT_SUGGESTION_END_REACHED_REASON,
                               "Experiment has succeeded because suggestion service has reached the end"),
        }[outcome]
        EC.mark_succeeded(exp, reason, msg)
        st.completion_time = now()
        self.metrics.inc("katib_experiment_succeeded_total", namespace=ns)

    def _reconcile_trials(self, key, exp, trials):
        """ReconcileTrials (experiment_controller.go:274-330); the admission plan (deletions,
        additions, suggestion demand) comes from the native status engine."""
        es_no_obs = sum(1 for t in trials if not TC.is_observation_available(t) and TC.is_early_stopped(t))
        delete, add, requests = SE.plan_admission(exp.status, exp.spec.parallel_trial_count,
                                                  exp.spec.max_trial_count, len(trials), es_no_obs)
        if delete > 0:
            self._delete_newest_trials(key, exp, trials, delete)
        elif add > 0:
            self._create_trials(key, exp, trials, add, requests)

    def _delete_newest_trials(self, key, exp, trials, count):
        """deleteTrials (experiment_controller.go:362-442): newest first, then prune the suggestion."""
        ordered = sorted(trials, key=lambda t: t.metadata.creation_timestamp, reverse=True)
        deleted = set()
        for t in ordered[:count]:
            self._delete_trial((t.metadata.namespace, t.metadata.name))
            deleted.add(t.metadata.name)
        sug = self.suggestions.get(key)
        if sug is not None and sug.status is not None:
            keep = [a for a in sug.status.suggestions or [] if a.name not in deleted]
            sug.spec.requests = len(keep)
            sug.status.suggestions = keep
            sug.status.suggestion_count = len(keep)

    def _create_trials(self, key, exp, trials, add, requests):
        """createTrials + ReconcileSuggestions (experiment_controller.go:332-360, 445-493);
        ``requests`` = len(trials) + add - early-stopped trials without an observation."""
        names = {t.metadata.name for t in trials}
        sug = self._get_or_create_suggestion(key, exp, requests)
        if sug is None:
            return
        if SC.is_failed(sug):
            EC.mark_failed(exp, C.EXPERIMENT_FAILED_REASON, "Suggestion has failed")
            exp.status.completion_time = now()
            self.metrics.inc("katib_experiment_failed_total", namespace=key[0])
            return
        if sug.spec.requests != requests:
            sug.spec.requests = requests
        done = self._reconcile_suggestion(key, exp, sug, trials)
        assignments = []
        if len(sug.status.suggestions or []) > len(trials):
            assignments = [a for a in sug.status.suggestions if a.name not in names]
        for a in assignments:
            try:
                trial = self._trial_instance(exp, a)
            except Exception as e:
                self._event(exp, "Warning", C.RECONCILE_ERROR_REASON, "Get trial instance error: %s" % e)
                continue
            tkey = (trial.metadata.namespace, trial.metadata.name)
            if tkey in self.trials:
                continue
            self.trials[tkey] = trial
            self.metrics.inc("katib_trial_created_total", namespace=key[0])
            TC.mark_created(trial, C.TRIAL_CREATED_REASON, "Trial is created")
            self.tracer.instant("trial.created", trial=tkey[1], experiment=exp.metadata.name)
            self.runs[tkey] = TrialRun()
        if done and not assignments:
            st = exp.status
            active = (st.trials_pending or 0) + (st.trials_running or 0)
            if active == 0:
                self._update_condition(exp, False, True)

    def _trial_instance(self, exp, a: V1beta1TrialAssignment) -> V1beta1Trial:
        """getTrialInstance (experiment_controller_util.go:39-96)."""
        labels = {C.LABEL_EXPERIMENT_NAME: exp.metadata.name}
        labels.update(a.labels or {})
        md = V1ObjectMeta(name=a.name, namespace=exp.metadata.namespace, labels=labels,
                          creation_timestamp=now(), uid="%032x" % random.getrandbits(128),
                          owner_references=[{"apiVersion": C.API_VERSION, "kind": C.KIND_EXPERIMENT,
                                             "name": exp.metadata.name, "uid": exp.metadata.uid,
                                             "controller": True}])
        tt = exp.spec.trial_template
        spec = V1beta1TrialSpec(
            objective=exp.spec.objective.deepcopy(),
            parameter_assignments=[p.deepcopy() for p in a.parameter_assignments or []],
            run_spec=self.generator.run_spec(exp, a.name, exp.metadata.namespace, a.parameter_assignments or []),
            retain_run=bool(tt.retain) if tt is not None else False,
            metrics_collector=exp.spec.metrics_collector_spec.deepcopy() if exp.spec.metrics_collector_spec else None,
            primary_pod_labels=dict(tt.primary_pod_labels) if tt.primary_pod_labels else None,
            primary_container_name=tt.primary_container_name or None,
            labels=dict(a.labels) if a.labels else None)
        if exp.spec.early_stopping is not None:
            spec.early_stopping_rules = [r.deepcopy() for r in a.early_stopping_rules or []]
        if tt.success_condition and tt.failure_condition:
            spec.success_condition = tt.success_condition
            spec.failure_condition = tt.failure_condition
        return V1beta1Trial(api_version=C.API_VERSION, kind=C.KIND_TRIAL, metadata=md, spec=spec,
                            status=V1beta1TrialStatus())

    # ============================================================== suggestion controller
    def _get_or_create_suggestion(self, key, exp, requests) -> Optional[V1beta1Suggestion]:
        """experiment/suggestion/suggestion.go:53-103."""
        sug = self.suggestions.get(key)
        if sug is None:
            sug = V1beta1Suggestion(
                api_version=C.API_VERSION, kind=C.KIND_SUGGESTION,
                metadata=V1ObjectMeta(name=exp.metadata.name, namespace=exp.metadata.namespace,
                                      labels={C.LABEL_EXPERIMENT_NAME: exp.metadata.name},
                                      creation_timestamp=now()),
                spec=V1beta1SuggestionSpec(algorithm=exp.spec.algorithm.deepcopy(),
                                           early_stopping=exp.spec.early_stopping.deepcopy()
                                           if exp.spec.early_stopping else None,
                                           requests=requests, resume_policy=exp.spec.resume_policy),
                status=V1beta1SuggestionStatus(start_time=now(), suggestion_count=0, suggestions=[]))
            SC.mark_created(sug, C.SUGGESTION_CREATED_REASON, "Suggestion is created")
            self.suggestions[key] = sug
        return sug

    def _reconcile_suggestion(self, key, exp, sug, trials) -> bool:
        """suggestion_controller.go:176-282 + suggestionclient SyncAssignments (:83-198).
        Returns True when the algorithm reports it has nothing more to suggest."""
        if SC.is_succeeded(sug) or SC.is_failed(sug):
            return False
        svc = self.services.get(key)
        if svc is None:
            # "deployment": instantiate the in-process service (cold start = microseconds)
            try:
                svc = create_service(exp.spec.algorithm.algorithm_name, self.config.suggestions,
                                     data_root=os.path.join(self.state_dir, "pbt"),
                                     cache_dir=os.path.join(self.state_dir, "ctrl_cache"))
            except Exception as e:
                SC.mark_failed(sug, C.SUGGESTION_FAILED_REASON, str(e))
                return False
            self.services[key] = svc
            if exp.spec.early_stopping is not None:
                self.es_services[key] = create_early_stopping(
                    exp.spec.early_stopping.algorithm_name, self.config.early_stoppings,
                    log_source=self, set_trial_status=lambda n, ns=key[0]: self.set_trial_early_stopped(n, ns))
            SC.mark_deployment_ready(sug, C.CONDITION_TRUE, C.SUGGESTION_DEPLOYMENT_READY_REASON,
                                     "Deployment is ready")
        if not SC.is_running(sug):
            # first run: ValidateAlgorithmSettings / ValidateEarlyStoppingSettings
            err = self._validate_settings(exp, svc, key)
            if err:
                SC.mark_failed(sug, C.SUGGESTION_FAILED_REASON, err)
                self._event(sug, "Warning", C.SUGGESTION_FAILED_REASON, err)
                return False
            SC.mark_running(sug, C.CONDITION_TRUE, C.SUGGESTION_RUNNING_REASON, "Suggestion is running")
        need = (sug.spec.requests or 0) - (sug.status.suggestion_count or 0)
        if need <= 0:
            return False
        req = api.GetSuggestionsRequest(experiment=convert_experiment(exp, sug.status.algorithm_settings),
                                        trials=convert_trials(trials), current_request_number=need,
                                        total_request_number=sug.spec.requests)
        try:
            with self.tracer.span("suggestion.GetSuggestions", experiment=exp.metadata.name,
                                  algorithm=exp.spec.algorithm.algorithm_name, current_request_number=need):
                reply = svc.GetSuggestions(req)
        except AlgorithmError as e:
            SC.mark_failed(sug, C.SUGGESTION_FAILED_REASON, e.message)
            return False
        except Exception as e:
            # gRPC INTERNAL in the reference: reconcile error, retried on the next iteration
            self._event(sug, "Warning", C.RECONCILE_ERROR_REASON, "GetSuggestions failed: %s" % e)
            return False
        got = list(reply.parameter_assignments)
        if not got:
            # algorithm finished (grid exhausted, HyperBand outer loop done) - or, for services
            # that serve partial batches, simply nothing to hand out yet
            return svc.finished_on_empty()
        if len(got) != need:
            if not (getattr(svc, "partial_batches", False) and len(got) < need):
                self._event(sug, "Warning", C.RECONCILE_ERROR_REASON, "The response contains unexpected trials")
                return False
            sug.spec.requests = (sug.status.suggestion_count or 0) + len(got)
        rules = []
        es = self.es_services.get(key)
        if es is not None:
            es_reply = es.GetEarlyStoppingRules(api.GetEarlyStoppingRulesRequest(
                experiment=convert_experiment(exp, sug.status.algorithm_settings), trials=convert_trials(trials),
                db_manager_address=""))
            rules = [V1beta1EarlyStoppingRule(name=r.name, value=r.value, comparison=comparison_from_pb(r.comparison),
                                              start_step=int(r.start_step)) for r in es_reply.early_stopping_rules]
        for pa in got:
            name = pa.trial_name or "%s-%s" % (sug.metadata.name, "".join(random.choice(_RAND_ALPHABET)
                                                                           for _ in range(8)))
            ta = V1beta1TrialAssignment(
                name=name, parameter_assignments=[V1beta1ParameterAssignment(name=a.name, value=a.value)
                                                  for a in pa.assignments],
                early_stopping_rules=[r.deepcopy() for r in rules] or None,
                labels=dict(pa.labels) if len(pa.labels) else None)
            sug.status.suggestions.append(ta)
        sug.status.suggestion_count = len(sug.status.suggestions)
        if reply.HasField("algorithm"):
            cur = sug.status.algorithm_settings or []
            for s in reply.algorithm.algorithm_settings:
                for x in cur:
                    if x.name == s.name:
                        x.value = s.value
                        break
                else:
                    cur.append(V1beta1AlgorithmSetting(name=s.name, value=s.value))
            sug.status.algorithm_settings = cur
        return False

    def _validate_settings(self, exp, svc, key) -> str:
        class _Ctx:
            code = None
            details = ""

            def set_code(self, c):
                self.code = c

            def set_details(self, d):
                self.details = d

        ctx = _Ctx()
        try:
            svc.ValidateAlgorithmSettings(api.ValidateAlgorithmSettingsRequest(experiment=convert_experiment(exp)), ctx)
        except Exception as e:
            return "ValidateAlgorithmSettings failed: %s" % e
        if ctx.code is not None:
            return "ValidateAlgorithmSettings Error: rpc error: code = %s desc = %s" % (
                getattr(ctx.code, "name", ctx.code), ctx.details)
        es = self.es_services.get(key)
        if es is not None:
            ctx = _Ctx()
            es.ValidateEarlyStoppingSettings(api.ValidateEarlyStoppingSettingsRequest(
                early_stopping=convert_experiment(exp).spec.early_stopping), ctx)
            if ctx.code is not None:
                return "ValidateEarlyStoppingSettings Error: rpc error: code = %s desc = %s" % (
                    getattr(ctx.code, "name", ctx.code), ctx.details)
        return ""

    def _cleanup_suggestion(self, exp):
        """cleanupSuggestionResources (experiment_controller_util.go:140-178)."""
        key = (exp.metadata.namespace, exp.metadata.name)
        sug = self.suggestions.get(key)
        if sug is None or SC.is_completed(sug) or SC.is_restarting(sug):
            return
        if exp.spec.resume_policy == C.RESUME_NEVER:
            SC.mark_succeeded(sug, "Experiment is succeeded", "Suggestion is succeeded, can't be restarted")
        else:
            SC.mark_succeeded(sug, "Experiment is succeeded",
                              "Suggestion is succeeded, suggestion volume is not deleted, can be restarted")
        # suggestion controller: succeeded -> delete deployment (drop the in-process service)
        self.services.pop(key, None)
        self.es_services.pop(key, None)

    def _restart_suggestion(self, exp):
        key = (exp.metadata.namespace, exp.metadata.name)
        sug = self.suggestions.get(key)
        if sug is None or SC.is_restarting(sug):
            return
        from ..api.conditions import remove_condition

        remove_condition(sug, C.SUGGESTION_SUCCEEDED)
        SC.mark_running(sug, C.CONDITION_FALSE, C.SUGGESTION_RESTARTING_REASON, "Suggestion is not running")

    # ============================================================== trial controller
    def _delete_trial(self, tkey):
        run = self.runs.get(tkey)
        if run is not None and run.phase in ("Running", "Launching"):
            run.deleted = True
            self._stop_job(tkey)
            self._release(run)
        t = self.trials.pop(tkey, None)
        self.runs.pop(tkey, None)
        if t is not None:
            # finalizer clean-metrics-in-db
            self.store.remove(t.metadata.name)
            self.metrics.inc("katib_trial_deleted_total", namespace=tkey[0])

    def _stop_job(self, tkey):
        name = tkey[1]
        run = self.runs.get(tkey)
        self.runtime.kill_trial(name, False)
        if run is not None:
            for aux in run.aux:
                self.runtime.kill_trial(aux, False)

    def _admit_trials(self):
        """Launch pending trials onto free GPU slots / CPU slots (the 'pod scheduling')."""
        pending = [(k, r) for k, r in self.runs.items() if r.phase == "Pending" and k in self.trials]
        pending.sort(key=lambda kr: self.trials[kr[0]].metadata.creation_timestamp)
        for tkey, run in pending:
            trial = self.trials[tkey]
            if TC.is_completed(trial):
                run.phase = "Failed" if not run.phase else run.phase
                continue
            if run.plan is None:
                try:
                    run.plan = make_plan(trial.spec.run_spec, trial.spec.primary_container_name or "",
                                         trial.spec.primary_pod_labels, self.config.amd.multi_gpu_launch)
                except JobSpecError as e:
                    self._finish_trial(tkey, "Failed", "JobSpecInvalid", str(e))
                    continue
            gpus = run.plan.total_gpus
            # slots stack on one device only where each slot is its own process (rank plans /
            # one-GPU replicas); a process that asks for k GPUs gets k different devices. Plans
            # whose replicas all see every device of the trial (share_devices: rank plans,
            # training-operator jobs) pick their device per rank, so they never need distinct ones.
            distinct = not run.plan.share_devices and any(rep.gpus > 1 for rep in run.plan.replicas)
            if gpus > 0:
                healthy = self.n_devices - len(self.slots.quarantined())
                if distinct and gpus > healthy:
                    # acquire(gpus, distinct=True) could never succeed: fail instead of pending forever
                    self._finish_trial(tkey, "Failed", "Unschedulable",
                                       "0/1 nodes are available: insufficient amd.com/gpu (one process requested %d "
                                       "distinct GPUs, node has %d healthy)" % (gpus, healthy))
                    continue
                if gpus > self.slots.capacity():
                    self._finish_trial(tkey, "Failed", "Unschedulable",
                                       "0/1 nodes are available: insufficient amd.com/gpu (requested %d, node has %d)"
                                       % (gpus, self.slots.capacity()))
                    continue
                devs = self.slots.acquire(gpus, distinct)
                if not devs:
                    continue
                run.devices = list(devs)
            else:
                if self.cpu_slots_used >= self.config.amd.cpu_slots:
                    continue
                self.cpu_slots_used += 1
                run.cpu_slot = True
            try:
                self._launch(tkey, trial, run)
            except Exception as e:
                log.exception("launch failed")
                self._release(run)
                self._finish_trial(tkey, "Failed", "LaunchError", str(e))

    def _collector_cfg(self, trial, run) -> Dict:
        mc = trial.spec.metrics_collector
        kind = mc.collector.kind if mc is not None and mc.collector else C.COLLECTOR_STDOUT
        obj = trial.spec.objective
        names = [obj.objective_metric_name] + list(obj.additional_metric_names or [])
        cfg = {"kind": _KIND_CODES.get(kind, 3), "metric_names": names, "filters": [], "format": 0,
               "objective_type": 2 if obj.type == C.OBJECTIVE_MAXIMIZE else 1}
        src = mc.source if mc is not None else None
        if src is not None and src.filter is not None and src.filter.metrics_format:
            cfg["filters"] = list(src.filter.metrics_format)
        if src is not None and src.file_system_path is not None:
            fsp = src.file_system_path
            if fsp.format == C.FORMAT_JSON:
                cfg["format"] = 1
            if fsp.path:
                cfg["file_path"] = map_paths([fsp.path], run.path_map)[0]
        rules = []
        for r in trial.spec.early_stopping_rules or []:
            try:
                rules.append({"name": r.name, "value": float(r.value), "comparison": _CMP_CODES.get(r.comparison, 0),
                              "start_step": int(r.start_step or 0)})
            except (TypeError, ValueError):
                continue
        cfg["rules"] = rules
        return cfg

    def _launch(self, tkey, trial, run: TrialRun):
        """reconcileJob create (trial_controller.go:263-310) + the pod-injector's wrapping."""
        ns, name = tkey
        exp_name = (trial.metadata.labels or {}).get(C.LABEL_EXPERIMENT_NAME, "")
        run.trial_dir = os.path.join(self.state_dir, "trials", ns, name)
        os.makedirs(run.trial_dir, exist_ok=True)
        mc = trial.spec.metrics_collector
        paths = []
        if mc is not None and mc.source is not None and mc.source.file_system_path is not None:
            paths.append(mc.source.file_system_path.path or "")
        extra_map = {}
        exp = self.experiments.get(self._owner(trial)) if self._owner(trial) else None
        if exp is not None and exp.spec.algorithm.algorithm_name == "pbt":
            sdir = {s.name: s.value for s in exp.spec.algorithm.algorithm_settings or []}.get(
                C.SUGGESTION_VOLUME_MOUNT_KEY)
            svc = self.services.get(self._owner(trial))
            member_dir = svc.checkpoint_dir(name) if svc is not None and hasattr(svc, "checkpoint_dir") else ""
            if sdir and member_dir:
                extra_map[sdir.rstrip("/")] = member_dir
        run.path_map = path_mapping(run.trial_dir, paths) if self.config.amd.map_collector_paths else {}
        run.path_map.update(extra_map)
        for dst in run.path_map.values():
            d = dst if not os.path.splitext(dst)[1] else os.path.dirname(dst)
            os.makedirs(d, exist_ok=True)
        run.collector = self._collector_cfg(trial, run)
        prom_env = {}
        if run.collector.get("kind") == _KIND_CODES[C.COLLECTOR_PROMETHEUS]:
            from ..metricscollector.prometheus import Scraper
            from .jobs import free_port

            hg = mc.source.http_get if mc is not None and mc.source is not None else None
            mpath = (hg.path if hg is not None and hg.path else C.DEFAULT_PROMETHEUS_PATH)
            port = free_port()  # one port per trial: concurrent trials cannot share the spec's
            run.scraper = Scraper(port, mpath, run.collector["metric_names"])
            run.prom_final = os.path.join(run.trial_dir, "prometheus_final.prom")
            if os.path.exists(run.prom_final):
                os.remove(run.prom_final)  # a retry must not read the previous attempt's snapshot
            prom_env = {"KATIB_PROMETHEUS_PORT": str(port), "KATIB_PROMETHEUS_PATH": mpath,
                        "KATIB_PROMETHEUS_FINAL": run.prom_final}
        log_path = os.path.join(run.trial_dir, "metrics.log")
        base_env = {"KATIB_TRIAL_NAME": name, "KATIB_EXPERIMENT_NAME": exp_name, "KATIB_TRIAL_DIR": run.trial_dir,
                    "KATIB_NAMESPACE": ns, "PYTHONUNBUFFERED": "1",
                    "HIP_VISIBLE_DEVICES": ",".join(str(d) for d in sorted(set(run.devices))),
                    "KATIB_AMD_CHECKPOINT_DIR": extra_map and list(extra_map.values())[0] or "",
                    "KATIB_TRIAL_CHECKPOINT_DIR": extra_map and list(extra_map.values())[0] or "",
                    # trials may run the built-in workloads with `python -m katib_amd.workloads.X`
                    "PYTHONPATH": os.pathsep.join(p for p in (_PKG_ROOT, os.environ.get("PYTHONPATH", "")) if p)}
        base_env.update(prom_env)
        if run.cpu_slot and "OMP_NUM_THREADS" not in os.environ:
            # CPU trials share the host: cpu_slots concurrent trials each spinning a full
            # OpenMP pool oversubscribe it cpu_slots times over
            base_env["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // max(1, self.config.amd.cpu_slots)))
        # each replica gets its share of the trial's devices; rank plans and training-operator
        # jobs see all of them (a rank picks LOCAL_RANK % device_count, parallel/comm.py)
        dev_iter = iter(run.devices)
        plan = run.plan
        assign_ports(plan)  # fresh rendezvous ports for this attempt (the plan is cached across retries)
        all_devs = sorted(set(run.devices))
        run.attempt += 1
        run.phase = "Launching"
        run.started = time.time()
        trial.status.start_time = trial.status.start_time or now()
        self.tracer.begin(name, "trial", track=("gpu" + ",".join(str(d) for d in run.devices)) if run.devices
                          else "cpu", trial=name, experiment=exp_name, attempt=run.attempt)
        if self.fault_injector is not None and self.fault_injector("launch", tkey):
            raise RuntimeError("fault injected at launch")
        for rep in plan.replicas:
            devs = [next(dev_iter) for _ in range(rep.gpus)] if run.devices else []
            env = dict(base_env)
            if run.devices:
                vis = all_devs if plan.share_devices else sorted(set(devs))
                env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in vis)
            env.update({k: map_paths([v], run.path_map)[0] for k, v in rep.env.items()})
            if "PYTHONPATH" in rep.env:
                env["PYTHONPATH"] = os.pathsep.join((env["PYTHONPATH"], _PKG_ROOT))
            argv = map_paths(rep.argv, run.path_map)
            cwd = rep.cwd or run.trial_dir
            proc_name = name if rep.primary else "%s~%s-%d" % (name, rep.role, rep.index)
            cfg = run.collector if rep.primary else {"kind": 3, "metric_names": [], "rules": []}
            lp = log_path if rep.primary else os.path.join(run.trial_dir, "%s-%d.log" % (rep.role, rep.index))
            if not rep.primary:
                run.aux.append(proc_name)
            self._proc_to_trial[proc_name] = tkey
            if (rep.entrypoint or rep.function) and rep.gpus <= 1 and len(plan.replicas) == 1 \
                    and self.config.amd.warm_workers:
                payload = {"trial": name, "env": env, "cwd": cwd}
                if rep.function:
                    payload["function"] = rep.function
                else:
                    payload["entrypoint"] = rep.entrypoint
                    payload["args"] = argv
                self._dispatch_to_worker(tkey, proc_name, devs, payload, lp, cfg, plan.deadline)
                continue
            if rep.entrypoint or rep.function:
                argv = [sys.executable, "-m", "katib_amd.controller.runentry", json.dumps(
                    {"entrypoint": rep.entrypoint, "args": argv, "function": rep.function})]
            pid = self._zygote_spawn(proc_name, argv, env, cwd, lp, cfg, float(plan.deadline))
            run.launcher = "zygote" if pid > 0 else "exec"
            if pid < 0:
                pid = self.runtime.spawn(proc_name, argv, ["%s=%s" % kv for kv in env.items()], cwd, lp, cfg,
                                         float(plan.deadline))
            if pid < 0:
                raise RuntimeError("failed to start %s (see %s)" % (argv[0], lp))
        if run.phase == "Launching" and run.worker is None:
            self._mark_running(tkey)

    def start_zygote(self, wait: bool = True) -> bool:
        """Start the trial fork server now (a daemon does this at start-up; otherwise it starts with
        the first eligible trial and the trials launched before it is up are exec'd)."""
        if self._zygote is None and not self._zygote_failed and self._zygote_thread is None:
            self._zygote_start_thread()
        if wait and self._zygote_thread is not None:
            self._zygote_thread.join(timeout=180)
        return self._zygote is not None

    def _zygote_start_thread(self):
        """Start the fork server on a helper thread. It makes this process a child subreaper
        (trials and their orphaned descendants re-parent here), so the native runtime is told to
        reap zombie children it does not track, except the server itself (its Popen waits for it)."""
        from .zygote import Zygote

        def start():
            try:
                z = Zygote(self.state_dir)
                self.runtime.set_reap_orphans(True, [z.proc.pid])
                self._zygote = z
            except Exception as e:  # noqa: BLE001 - the exec path always works
                log.warning("fork server unavailable (%s): trials are exec'd", e)
                self._zygote_failed = True

        self._zygote_thread = threading.Thread(target=start, name="katib-zygote", daemon=True)
        self._zygote_thread.start()

    def _zygote_spawn(self, proc_name, argv, env, cwd, log_path, cfg, deadline) -> int:
        """Start a cold Python trial from the fork server (controller/zygote.py) and hand it to the
        native runtime (``TrialRuntime.adopt``); -1: not eligible or the server is unavailable,
        the caller then fork+execs as before. The trial sees the same environment as an exec'd
        one: this process's environment with the trial's entries on top."""
        from .zygote import Zygote

        if self._zygote_failed or not self.config.amd.zygote or os.environ.get("KATIB_AMD_ZYGOTE", "1") == "0" \
                or not Zygote.eligible(argv):
            return -1
        if self._zygote is None or not self._zygote.alive():
            # start the server in the background (import torch + torch.optim: ~3 s) and exec the
            # trials launched meanwhile instead of making them wait for it
            self._zygote = None
            if self._zygote_thread is None or not self._zygote_thread.is_alive():
                self._zygote_start_thread()
            return -1
        full = dict(os.environ)
        full.update(env)
        r, w = os.pipe()
        try:
            pid = self._zygote.spawn(argv, full, cwd, w)
        except Exception as e:  # noqa: BLE001
            log.warning("fork server spawn failed (%s): exec instead", e)
            os.close(r)
            os.close(w)
            return -1
        os.close(w)
        if not self.runtime.adopt(proc_name, pid, r, log_path, cfg, deadline):
            os.close(r)
            try:
                os.killpg(pid, 9)
                os.waitpid(pid, 0)
            except OSError:
                pass
            return -1
        return pid

    def _mark_running(self, tkey):
        run = self.runs[tkey]
        run.phase = "Running"
        trial = self.trials[tkey]
        status = job_status(run.plan.kind, "Running")
        if gjson.matches(status, trial.spec.failure_condition or ""):
            return
        if not TC.is_running(trial) and not TC.is_early_stopped(trial):
            TC.mark_running(trial, C.TRIAL_RUNNING_REASON, "Trial is running")
            self._event(trial, "Normal", C.JOB_RUNNING_REASON, "Job %s is running" % trial.metadata.name)

    # -- warm workers -------------------------------------------------------------------
    def _dispatch_to_worker(self, tkey, proc_name, devs, payload, log_path, cfg, deadline):
        dkey = ",".join(str(d) for d in devs)
        run = self.runs[tkey]
        for w in self.workers.values():
            if w.device_key == dkey and w.busy is None and w.pending is None and self.runtime.worker_alive(w.wid):
                if w.ready:
                    ok = self.runtime.assign(w.wid, proc_name, json.dumps(payload), log_path, cfg, float(deadline))
                    if ok:
                        w.busy = proc_name
                        run.worker = w.wid
                        self._mark_running(tkey)
                        return
                else:
                    w.pending = (tkey, proc_name, payload, log_path, cfg, deadline)
                    run.worker = w.wid
                    return
        py = self.config.amd.worker_python or sys.executable
        env = ["HIP_VISIBLE_DEVICES=%s" % dkey, "PYTHONUNBUFFERED=1"]
        wlog = os.path.join(self.state_dir, "workers", "worker-%s-%d.log" % (dkey or "cpu", len(self.workers)))
        os.makedirs(os.path.dirname(wlog), exist_ok=True)
        env.append("PYTHONPATH=%s%s" % (_PKG_ROOT, (":" + os.environ["PYTHONPATH"]) if os.environ.get("PYTHONPATH")
                                         else ""))
        wid = self.runtime.spawn_worker([py, "-m", "katib_amd.controller.worker"] + (["--warm"] if dkey else []),
                                        env, self.state_dir, wlog)
        if wid < 0:
            raise RuntimeError("failed to start warm worker")
        w = WorkerInfo(wid=wid, device_key=dkey, pending=(tkey, proc_name, payload, log_path, cfg, deadline))
        self.workers[wid] = w
        run.worker = wid

    def _worker_ready(self, wid):
        w = self.workers.get(wid)
        if w is None:
            return
        w.ready = True
        if w.pending is not None:
            tkey, proc_name, payload, log_path, cfg, deadline = w.pending
            w.pending = None
            if tkey not in self.runs or self.runs[tkey].deleted:
                return
            if self.runtime.assign(wid, proc_name, json.dumps(payload), log_path, cfg, float(deadline)):
                w.busy = proc_name
                self._mark_running(tkey)
            else:
                self._finish_trial(tkey, "Failed", "WorkerError", "could not assign trial to worker %d" % wid)

    # -- runtime events ---------------------------------------------------------------
    def _on_runtime_event(self, ev):
        t = ev["type"]
        if t == "worker_ready":
            self._worker_ready(ev["worker"])
            return
        if t == "worker_died":
            w = self.workers.pop(ev["worker"], None)
            if w is not None and w.pending is not None:
                tkey = w.pending[0]
                if tkey in self.runs:
                    self._finish_trial(tkey, "Failed", "WorkerDied",
                                       "warm worker exited with code %d" % ev["exit_code"])
            if ev["signal"] in (6, 11) and w is not None and w.device_key:
                for d in w.device_key.split(","):
                    self.slots.record_fault(int(d), self.config.amd.fault_quarantine_threshold)
            return
        if t != "exited":
            return
        proc = ev["trial"]
        tkey = self._proc_to_trial.pop(proc, None)
        if ev["worker"] >= 0 and ev["worker"] in self.workers:
            self.workers[ev["worker"]].busy = None
        if tkey is None or tkey not in self.runs:
            return
        run = self.runs[tkey]
        if proc in run.aux:
            if ev["exit_code"] != 0 and not run.deleted and run.phase == "Running":
                # a failed worker replica fails the whole distributed job
                self._stop_job(tkey)
            return
        # primary replica finished: stop the rest of the job
        for aux in run.aux:
            self.runtime.kill_trial(aux, False)
        if self.fault_injector is not None:
            act = self.fault_injector("exit", tkey)
            if act == "crash":
                ev = dict(ev, exit_code=1, early_stopped=False)
            elif act == "drop_metrics":
                self.store.remove(tkey[1])
            elif act == "gpu_fault":
                ev = dict(ev, exit_code=139, signal=11, early_stopped=False)
        if ev["signal"] in (6, 11) and run.devices:
            # a trial that died on SIGSEGV/SIGABRT on a GPU counts as a device fault
            for d in run.devices:
                self.slots.record_fault(int(d), self.config.amd.fault_quarantine_threshold)
        self._release(run)
        if run.deleted:
            return
        trial = self.trials.get(tkey)
        if trial is None:
            return
        if ev["early_stopped"]:
            run.early_stopped = True
            self.set_trial_early_stopped(tkey[1], tkey[0])
        code = ev["exit_code"]
        if run.collector.get("kind") == 2:
            self._collect_tfevent(trial, run)
        if run.scraper is not None and run.prom_final:
            logs = run.scraper.read_final(run.prom_final)  # the value published right before exit
            if logs:
                self.store.report(tkey[1], logs)
        outcome = SE.classify_exit(bool(ev["early_stopped"]), code, ev["worker"] >= 0, bool(run.early_stopped),
                                   bool(ev["deadline_exceeded"]), TC.is_killed(trial), run.attempt,
                                   run.plan.backoff_limit)
        if outcome == "succeeded":
            self._finish_trial(tkey, "Succeeded", "", "")
        elif outcome == "deadline_exceeded":
            self._finish_trial(tkey, "Failed", "DeadlineExceeded", "Job was active longer than specified deadline")
        elif outcome == "killed":
            run.phase = "Failed"
        elif outcome == "retry":
            run.phase = "Pending"  # retry (Job backoffLimit)
            self.store.remove(tkey[1])
        else:
            msg = ev["message"] or ""
            self._finish_trial(tkey, "Failed", "Error", "exit code %d%s" % (code, (": " + msg) if msg else ""))

    def _due_scrapes(self):
        """PrometheusMetric collector: running trials whose scrape interval is due."""
        now = time.time()
        out = []
        for tkey, run in self.runs.items():
            sc = run.scraper
            if sc is None or run.phase not in ("Launching", "Running") or not sc.due(now):
                continue
            sc.next_at = now + sc.interval  # not due again while this scrape is in flight
            out.append((tkey, sc))
        return out

    def _collect_tfevent(self, trial, run):
        from ..metricscollector.tfevent import collect

        fsp = trial.spec.metrics_collector.source.file_system_path
        d = map_paths([fsp.path], run.path_map)[0]
        obj = trial.spec.objective
        names = [obj.objective_metric_name] + list(obj.additional_metric_names or [])
        self.store.report(trial.metadata.name, collect(d, names))

    def _release(self, run: TrialRun):
        if run.devices:
            self.slots.release(run.devices)
            run.devices = []
        if run.cpu_slot:
            self.cpu_slots_used -= 1
            run.cpu_slot = False

    def _finish_trial(self, tkey, phase, reason, message):
        """reconcileTrial / UpdateTrialStatusCondition (trial_controller.go:209-261,
        trial_controller_util.go:42-122) on the synthesised job status."""
        run = self.runs[tkey]
        trial = self.trials[tkey]
        run.phase, run.reason, run.message = phase, reason, message
        run.finished = time.time()
        first = self._first_metric_time(tkey[1])
        if first is not None:
            self.tracer.instant("trial.first_metric", trial=tkey[1], at=first)
        self.tracer.end(tkey[1], phase=phase, reason=reason)
        kind = run.plan.kind if run.plan else C.JOB_KIND_JOB
        status = job_status(kind, phase, reason, message)
        st = gjson.deployed_job_status(status, trial.spec.success_condition or "",
                                       trial.spec.failure_condition or "", trial_running=True) or {}
        cond = st.get("condition")
        ns = tkey[0]
        if cond == "Succeeded":
            self._update_observation(trial)
        # the condition change is decided by the native trial state machine
        action = SE.trial_transition(cond, trial, cond == "Succeeded" and TC.is_observation_available(trial))
        if action == "mark_failed":
            TC.mark_failed(trial, "%s. Job reason: %s" % (C.TRIAL_FAILED_REASON, reason) if reason
                           else C.TRIAL_FAILED_REASON,
                           "Trial has failed. Job message: %s" % message if message else "Trial has failed")
            self._event(trial, "Normal", C.JOB_FAILED_REASON, "Job %s has failed. %s %s"
                        % (trial.metadata.name, message, reason))
            self.metrics.inc("katib_trial_failed_total", namespace=ns)
        elif action == "mark_succeeded":
            TC.mark_succeeded(trial, C.CONDITION_TRUE, C.TRIAL_SUCCEEDED_REASON, "Trial has succeeded")
            self._event(trial, "Normal", C.JOB_SUCCEEDED_REASON, "Job %s has succeeded" % trial.metadata.name)
            self.metrics.inc("katib_trial_succeeded_total", namespace=ns)
        elif action == "mark_metrics_unavailable":
            TC.mark_metrics_unavailable(trial, C.TRIAL_METRICS_UNAVAILABLE_REASON, "Metrics are not available")
            self._event(trial, "Warning", C.JOB_METRICS_UNAVAILABLE_REASON,
                        "Metrics are not available for Job %s" % trial.metadata.name)
            self.metrics.inc("katib_trial_metrics_unavailable_total", namespace=ns)
        if action != "none":
            trial.status.completion_time = now()
            self._completed += 1
        if not trial.spec.retain_run:
            # the Job is deleted once the trial completed (trial_controller.go:297-306)
            self._event(trial, "Normal", C.JOB_DELETED_REASON, "Job %s has been deleted" % trial.metadata.name)

    def _first_metric_time(self, trial_name: str) -> Optional[float]:
        try:
            logs = self.store.get(trial_name, "", "", "")
        except Exception:
            return None
        ts = []
        for lg in logs:
            r = self.N.parse_rfc3339(str(lg[0])) if isinstance(lg, (tuple, list)) and lg else None
            if r is not None:
                ts.append(r[0] + r[1] * 1e-9)
        return min(ts) if ts else None

    def _update_observation(self, trial):
        """UpdateTrialStatusObservation + getMetrics (trial_controller_util.go:124-217); the
        min/max/latest reduction runs natively over the store."""
        strategies = trial.spec.objective.metric_strategies or []
        names = [s.name for s in strategies]
        if not names or self.store.size(trial.metadata.name) == 0:
            return
        red = self.store.reduce(trial.metadata.name, names)
        trial.status.observation = V1beta1Observation(
            metrics=[V1beta1Metric(name=n, min=mn, max=mx, latest=lt) for n, mn, mx, lt in red])

    # ============================================================== misc
    def _event(self, obj, typ, reason, message):
        self.events.append({"time": time.time(), "kind": obj.kind, "name": obj.metadata.name,
                            "namespace": obj.metadata.namespace, "type": typ, "reason": reason, "message": message})
        if len(self.events) > 10000:
            del self.events[:5000]

    def _update_gauges(self):
        per_ns: Dict[Tuple[str, str], int] = {}
        for (ns, _), e in self.experiments.items():
            st = "Succeeded" if EC.is_succeeded(e) else "Failed" if EC.is_failed(e) else \
                "Running" if EC.is_running(e) else "Created"
            per_ns[(ns, st)] = per_ns.get((ns, st), 0) + 1
        for (ns, st), n in per_ns.items():
            self.metrics.set("katib_experiments_current", n, namespace=ns, status=st)
        hours = max((time.time() - self._t0) / 3600.0, 1e-9)
        self.metrics.set("katib_amd_trials_per_hour", self._completed / hours)
        cap = self.slots.capacity()
        self.metrics.set("katib_amd_gpu_slots_total", cap)
        self.metrics.set("katib_amd_gpu_slots_busy", cap - self.slots.free_slots())

    def _journal_path(self, key):
        return os.path.join(self.state_dir, "experiments", key[0], key[1] + ".json")

    def _persist(self, key):
        if not self._journal:
            return
        exp = self.experiments.get(key)
        if exp is None:
            return
        doc = {"experiment": exp.to_k8s(),
               "trials": [t.to_k8s() for t in self._exp_trials(key)],
               "suggestion": self.suggestions[key].to_k8s() if key in self.suggestions else None}
        p = self._journal_path(key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp"
        with open(tmp, "w") as f:
            json.dump(doc, f, default=str)
        os.replace(tmp, p)

    def restore(self) -> List[str]:
        """Reload journaled experiments (resume after a scheduler restart). Trials that were
        running when the previous scheduler died are marked Failed (their processes died
        with it: PR_SET_PDEATHSIG)."""
        restored = []
        root = os.path.join(self.state_dir, "experiments")
        if not os.path.isdir(root):
            return restored
        with self._lock:
            for ns in os.listdir(root):
                for fn in os.listdir(os.path.join(root, ns)):
                    if not fn.endswith(".json"):
                        continue
                    with open(os.path.join(root, ns, fn)) as f:
                        doc = json.load(f)
                    exp = V1beta1Experiment.from_k8s(doc["experiment"])
                    key = (exp.metadata.namespace, exp.metadata.name)
                    if key in self.experiments:
                        continue
                    self.experiments[key] = exp
                    for td in doc.get("trials") or []:
                        t = V1beta1Trial.from_k8s(td)
                        tkey = (t.metadata.namespace, t.metadata.name)
                        self.trials[tkey] = t
                        run = TrialRun()
                        if TC.is_completed(t):
                            run.phase = "Succeeded"
                        elif TC.is_running(t):
                            TC.mark_failed(t, C.TRIAL_FAILED_REASON, "Trial was running when the scheduler stopped")
                            t.status.completion_time = now()
                            run.phase = "Failed"
                        self.runs[tkey] = run
                    if doc.get("suggestion"):
                        self.suggestions[key] = V1beta1Suggestion.from_k8s(doc["suggestion"])
                    restored.append(exp.metadata.name)
        return restored

    def _install_default_templates(self):
        """The ``trial-templates`` ConfigMap of the reference install
        (manifests/v1beta1/components/controller/trial-templates.yaml), pointing at
        first-party MI355X workloads."""
        lbl = {C.LABEL_TRIAL_TEMPLATE_CONFIGMAP_NAME: C.LABEL_TRIAL_TEMPLATE_CONFIGMAP_VALUE}
        tpl = {
            "defaultTrialTemplate.yaml": json.dumps({
                "apiVersion": "batch/v1", "kind": "Job",
                "spec": {"template": {"spec": {"containers": [{
                    "name": "training-container",
                    "command": [sys.executable, "-m", "katib_amd.workloads.mnist_mlp",
                                "--lr=${trialParameters.learningRate}", "--momentum=${trialParameters.momentum}"],
                }], "restartPolicy": "Never"}}}}),
        }
        self.configmaps.put("kubeflow", "trial-templates", tpl, lbl)
