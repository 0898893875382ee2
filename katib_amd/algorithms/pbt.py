"""Population Based Training suggestion service (reference ``pkg/suggestion/v1beta1/pbt/service.py:39-409``).

Required settings ``suggestion_trial_dir``, ``n_population`` (>= 5) and
``truncation_threshold`` (in [0, 1]); optional ``resample_probability``.
The objective is scaled so that the queue always maximises. Trials are named
``<experiment>-<uuid4>`` and labelled
``pbt.suggestion.katib.kubeflow.org/{generation,parent}``.

Checkpoint hand-off: each member owns ``<data_root>/<experiment>/<uid>``; a new
member's directory is seeded from its parent's. On a MI355X node the trial
workers additionally keep the latest member checkpoint resident in HBM and the
exploit copy goes GPU->GPU over xGMI (see :mod:`katib_amd.parallel.checkpoint`);
the directory copy is the durable fallback (``FromVolume`` resume).

Divergence (documented): the reference exploits the winner's
*hyperparameters* but records ``parent`` = the truncated trial itself
(service.py:383-390), so the loser's own checkpoint is copied. Classic PBT copies
the winner's weights; that is our default (``exploit_checkpoint: winner``); set
``exploit_checkpoint: self`` for bit-for-bit reference behaviour.
"""

from __future__ import annotations

import os
import shutil
import uuid

import numpy as np

from ..rpc import api_pb2 as api
from .internal import (CATEGORICAL, DISCRETE, DOUBLE, INTEGER, SuggestionService, abort, convert_parameter,
                       make_reply_assignments)

REQUIRED_SETTINGS = ["suggestion_trial_dir", "n_population", "truncation_threshold"]
LABEL_GENERATION = "pbt.suggestion.katib.kubeflow.org/generation"
LABEL_PARENT = "pbt.suggestion.katib.kubeflow.org/parent"
DEFAULT_DATA_PATH = os.environ.get("KATIB_AMD_PBT_DATA", "/tmp/katib-amd/pbt")


class ParamSampler:
    def __init__(self, p, rng):
        self.p = p
        self.rng = rng
        if p.type in (INTEGER, DOUBLE):
            step = p.step if p.step else (1 if p.type == INTEGER else None)
            if step is None:
                # DOUBLE without step: the reference np.arange would fail; use 100 bins
                step = (p.max - p.min) / 100.0 if p.max > p.min else 1.0
            self.sample_list = np.arange(p.min, p.max + step / 2, step).astype(int if p.type == INTEGER else float)
        else:
            self.sample_list = list(p.list)

    @property
    def name(self):
        return self.p.name

    def sample(self):
        v = self.sample_list[self.rng.randint(0, len(self.sample_list))]
        return v.item() if hasattr(v, "item") else v

    def perturb(self, value):
        p = self.p
        if p.type == INTEGER:
            nv = int(int(value) * self.rng.choice([0.8, 1.2]))
            return max(float(p.min), min(float(p.max), nv))
        if p.type == DOUBLE:
            nv = float(value) * self.rng.choice([0.8, 1.2])
            return max(float(p.min), min(float(p.max), nv))
        idx = self.sample_list.index(value) + int(self.rng.choice([-1, 1]))
        if idx >= len(self.sample_list):
            return self.sample_list[0]
        return self.sample_list[idx]


class PbtJob:
    def __init__(self, uid, params, generation, parent=None):
        self.uid = uid
        self.params = {k: str(v) for k, v in params}
        self.generation = generation
        self.parent = parent
        self.metric_value = None

    def get(self):
        labels = {LABEL_GENERATION: self.generation}
        if self.parent is not None:
            labels[LABEL_PARENT] = self.parent
        return list(self.params.items()), labels, self.uid


class PbtJobQueue:
    def __init__(self, experiment_name, data_root, population_size, truncation_threshold, resample_probability,
                 search_space, metric_name, metric_scaler, rng, exploit_checkpoint="winner"):
        self.experiment_name = experiment_name
        self.suggestion_dir = os.path.join(data_root, experiment_name)
        self.population_size = population_size
        self.truncation_threshold = truncation_threshold
        self.resample_probability = resample_probability
        self.search_space = search_space
        self.metric_name = metric_name
        self.metric_scaler = metric_scaler
        self.rng = rng
        self.exploit_checkpoint = exploit_checkpoint
        self.pending, self.running, self.completed = [], {}, {}
        self.sample_pool = {"previous": [], "current": []}
        self._seed(population_size)

    def __len__(self):
        return len(self.pending)

    def _objective(self, trial):
        for m in trial.status.observation.metrics:
            if m.name == self.metric_name:
                try:
                    return self.metric_scaler * float(m.value)
                except ValueError:
                    return None
        return None

    def _seed(self, count):
        for _ in range(count):
            self.append([(p.name, p.sample()) for p in self.search_space], 0)

    def append(self, assignments, generation, parent=None):
        job = PbtJob("{}-{}".format(self.experiment_name, uuid.UUID(bytes=self.rng.bytes(16), version=4)),
                     assignments, generation, parent)
        self.pending.append(job)
        new_dir = os.path.join(self.suggestion_dir, job.uid)
        if os.path.isdir(new_dir):
            shutil.rmtree(new_dir)
        if parent is None:
            os.makedirs(new_dir, exist_ok=True)
        else:
            src = os.path.join(self.suggestion_dir, parent)
            if os.path.isdir(src):
                shutil.copytree(src, new_dir)
            else:
                os.makedirs(new_dir, exist_ok=True)
        return job.uid

    def get(self):
        if not self.pending:
            raise RuntimeError("Pending queue is empty!")
        job = self.pending.pop(0)
        self.running[job.uid] = job
        return job.get()

    def update(self, trial):
        uid = trial.name
        if trial.status.condition in (api.TrialStatus.CREATED, api.TrialStatus.RUNNING):
            return
        if uid in self.completed or uid not in self.running:
            return
        job = self.running.pop(uid)
        job.metric_value = self._objective(trial)
        self.completed[uid] = job
        if trial.status.condition in (api.TrialStatus.KILLED, api.TrialStatus.FAILED) or job.metric_value is None:
            self.append([(a.name, a.value) for a in trial.spec.parameter_assignments.assignments],
                        job.generation, job.parent)
            return
        self.sample_pool["current"].append(uid)

    def _segment(self, pool, count):
        jobs = [self.completed[u] for u in self.sample_pool[pool]]
        values = [j.metric_value for j in jobs]
        lo, hi = np.quantile(values, (self.truncation_threshold, 1 - self.truncation_threshold))
        exploit, explore, upper = [], [], []
        for j in jobs:
            if j.metric_value < lo:
                exploit.append(j.uid)
            else:
                explore.append(j.uid)
                if j.metric_value >= hi:
                    upper.append(j.uid)
        self.rng.shuffle(exploit)
        self.rng.shuffle(explore)
        exploit = list(exploit[: int(count * self.truncation_threshold)])
        explore = list(explore[: count - len(exploit)])
        return exploit, explore, upper

    def generate(self, min_count):
        if len(self.sample_pool["current"]) <= self.population_size:
            if not self.sample_pool["previous"]:
                self._seed(min_count)
                return
            exploit, explore, upper = self._segment("previous", min_count)
        else:
            exploit, explore, upper = self._segment("current", self.population_size)
            self.sample_pool["previous"] = self.sample_pool["current"]
            self.sample_pool["current"] = []
        if exploit and upper:
            winners = self.rng.choice(upper, len(exploit))
            for n, uid in enumerate(exploit):
                job = self.completed[uid]
                winner = self.completed[winners[n]]
                parent = winner.uid if self.exploit_checkpoint == "winner" else job.uid
                self.append(list(winner.params.items()), job.generation + 1, parent)
        for uid in explore:
            job = self.completed[uid]
            out = []
            for ps in self.search_space:
                if self.resample_probability is None:
                    nv = ps.perturb(job.params[ps.name] if ps.p.type in (CATEGORICAL, DISCRETE)
                                    else job.params[ps.name])
                elif self.rng.random_sample() < self.resample_probability:
                    nv = ps.sample()
                else:
                    nv = job.params[ps.name]
                out.append((ps.name, nv))
            self.append(out, job.generation + 1, job.uid)


class PbtService(SuggestionService):
    algorithm_names = ("pbt",)

    def __init__(self, data_root: str = None, seed=None):
        self.data_root = data_root or DEFAULT_DATA_PATH
        self.job_queue = None
        self.rng = np.random.RandomState(seed)

    def ValidateAlgorithmSettings(self, request, context=None):
        s = {e.name: e.value for e in request.experiment.spec.algorithm.algorithm_settings}

        def bad(msg):
            abort(context, "INVALID_ARGUMENT", msg)
            return api.ValidateAlgorithmSettingsReply()

        missing = [k for k in REQUIRED_SETTINGS if k not in s]
        if missing:
            return bad("Required params missing: {}".format(", ".join(missing)))
        if int(s["n_population"]) < 5:
            return bad("Param(n_population) should be >= 5")
        if not 0 <= float(s["truncation_threshold"]) <= 1:
            return bad("Param(truncation_threshold) should be between 0 and 1, inclusive")
        if "resample_probability" in s and not 0 <= float(s["resample_probability"]) <= 1:
            return bad("Param(resample_probability) should be null to perturb at 0.8 or 1.2, or be between 0 and 1,"
                       " inclusive, to resample")
        if s.get("exploit_checkpoint", "winner") not in ("winner", "self"):
            return bad("Param(exploit_checkpoint) should be winner or self")
        return api.ValidateAlgorithmSettingsReply()

    def GetSuggestions(self, request, context=None):
        exp = request.experiment
        if self.job_queue is None:
            s = {e.name: e.value for e in exp.spec.algorithm.algorithm_settings}
            if "random_state" in s:
                self.rng = np.random.RandomState(int(s["random_state"]))
            space = [ParamSampler(convert_parameter(p), self.rng) for p in exp.spec.parameter_specs.parameters]
            scale = 1 if exp.spec.objective.type == api.MAXIMIZE else -1
            self.job_queue = PbtJobQueue(
                exp.name, s.get("data_root", self.data_root), int(s["n_population"]),
                float(s["truncation_threshold"]),
                None if "resample_probability" not in s else float(s["resample_probability"]),
                space, exp.spec.objective.objective_metric_name, scale, self.rng,
                s.get("exploit_checkpoint", "winner"))
        for t in request.trials:
            self.job_queue.update(t)
        n = request.current_request_number
        if len(self.job_queue) < n:
            self.job_queue.generate(n)
        jobs = [self.job_queue.get() for _ in range(n)]
        return api.GetSuggestionsReply(parameter_assignments=make_reply_assignments(
            [j[0] for j in jobs], trial_names=[j[2] for j in jobs], labels=[j[1] for j in jobs]))

    def checkpoint_dir(self, trial_name: str) -> str:
        return os.path.join(self.job_queue.suggestion_dir, trial_name) if self.job_queue is not None else ""
