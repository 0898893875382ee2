"""Trial "jobs" on a single MI355X node.

A trial's ``runSpec`` (the rendered trial template) is turned into a
:class:`LaunchPlan` - one or more local processes - instead of a Kubernetes
object. Supported kinds:

* ``batch/v1 Job`` - the primary container's ``command``/``args``/``env``/
  ``workingDir``; ``resources.limits`` ``amd.com/gpu`` (or ``nvidia.com/gpu``)
  selects the GPU count; ``activeDeadlineSeconds`` and an explicit
  ``backoffLimit`` are honoured.
* Kubeflow training jobs (``PyTorchJob``, ``TFJob``, ``XGBoostJob``, ``MXJob``,
  ``MPIJob``): one process per replica, wired with ``MASTER_ADDR=127.0.0.1``,
  ``MASTER_PORT``, ``WORLD_SIZE``, ``RANK``, ``LOCAL_RANK`` (torch.distributed over
  RCCL) or ``TF_CONFIG``; metrics come from the primary replica selected by
  ``primaryPodLabels`` (master/chief/launcher), mirroring the reference's
  primary-pod semantics (``inject_webhook.go:143-148``).
* ``LocalProcess`` (native kind, ``apiVersion: katib-amd.io/v1``): ``command`` for
  a subprocess or ``entrypoint: module:function`` to run in a warm GPU worker.

A ``Job`` / ``LocalProcess`` trial that asks for N > 1 GPUs runs as N *rank* processes
(one process per GPU, the MI355X way to drive several GPUs) with the torchrun env
(``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR``,
``MASTER_PORT``); rank 0 is the primary whose output the metrics collector parses, the
way the reference collects from the primary pod only. This replaces the reference's
one-process-over-all-GPUs trials (the ENAS child's ``MirroredStrategy``,
``examples/v1beta1/trial-images/enas-cnn-cifar10/RunTrial.py:54-63``). A program that
drives every GPU itself opts out with the container env ``KATIB_AMD_LAUNCH=single`` (or
``amd.multi_gpu_launch: single`` in the KatibConfig). Every rank - and every replica of a
training-operator job - sees the trial's whole device list and picks
``LOCAL_RANK % device_count`` (``parallel/comm.py``).
* ``Function``: SDK ``tune()`` objective source executed in a warm worker.

The job status handed to the GJSON success/failure conditions is synthesised in
the shape of the corresponding Kubernetes status (``status.conditions[]``).
"""

from __future__ import annotations

import collections
import json
import os
import socket
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..api import constants as C

GPU_RESOURCE_KEYS = ("amd.com/gpu", "nvidia.com/gpu", "gpu")

_REPLICA_KEYS = {
    "PyTorchJob": ("pytorchReplicaSpecs", ["Master", "Worker"]),
    "TFJob": ("tfReplicaSpecs", ["Chief", "Master", "Worker", "PS", "Evaluator"]),
    "XGBoostJob": ("xgbReplicaSpecs", ["Master", "Worker"]),
    "MXJob": ("mxReplicaSpecs", ["Scheduler", "Server", "Worker", "Tuner", "TunerServer", "TunerTracker"]),
    "MPIJob": ("mpiReplicaSpecs", ["Launcher", "Worker"]),
}
_PRIMARY_ROLE = {"PyTorchJob": "Master", "TFJob": "Chief", "XGBoostJob": "Master", "MXJob": "Scheduler",
                 "MPIJob": "Launcher"}


@dataclass
class ReplicaPlan:
    role: str
    index: int
    argv: List[str]
    env: Dict[str, str]
    cwd: Optional[str]
    gpus: int
    primary: bool
    entrypoint: Optional[str] = None  # "module:function" for warm-worker execution
    function: Optional[Dict] = None  # {"source":..., "entry":..., "params": {...}}


@dataclass
class LaunchPlan:
    kind: str
    replicas: List[ReplicaPlan] = field(default_factory=list)
    deadline: float = 0.0
    backoff_limit: int = 0
    share_devices: bool = False  # every replica sees all the trial's devices (rank plans, training jobs)
    ports_managed: bool = False  # rendezvous ports in the replicas' env are ours: fresh ones per attempt

    @property
    def primary(self) -> ReplicaPlan:
        for r in self.replicas:
            if r.primary:
                return r
        return self.replicas[0]

    @property
    def total_gpus(self) -> int:
        return sum(r.gpus for r in self.replicas)


class JobSpecError(ValueError):
    pass


def _gpus(container: Dict) -> int:
    res = container.get("resources") or {}
    for section in ("limits", "requests"):
        sec = res.get(section) or {}
        for k in GPU_RESOURCE_KEYS:
            if k in sec:
                try:
                    return int(sec[k])
                except (TypeError, ValueError):
                    return 1
    return 0


def _env(container: Dict) -> Dict[str, str]:
    out = {}
    for e in container.get("env") or []:
        if "value" in e and e.get("name"):
            out[e["name"]] = str(e["value"])
    return out


def _container(pod_spec: Dict, primary_name: str) -> Dict:
    cs = pod_spec.get("containers") or []
    if not cs:
        raise JobSpecError("pod template has no containers")
    for c in cs:
        if c.get("name") == primary_name:
            return c
    return cs[0]


def _argv(c: Dict) -> List[str]:
    cmd = list(c.get("command") or []) + list(c.get("args") or [])
    if not cmd:
        raise JobSpecError("container %r has no command: image ENTRYPOINT lookup is not available on a "
                           "node-local scheduler; set command/args explicitly" % c.get("name"))
    return [str(a) for a in cmd]


_RECENT_PORTS: "collections.deque" = collections.deque(maxlen=512)
_PORT_LOCK = threading.Lock()


def free_port() -> int:
    """An ephemeral TCP port for a trial's rendezvous / Prometheus endpoint. The port is free
    when probed but only bound later by the trial, so two launches racing for the same number
    are possible in principle; within this scheduler a port handed out recently (the last 512)
    is never handed out again, which removes the race between concurrent trials. A clash with
    an unrelated process binding the port in between surfaces as the trial's bind error (its
    retry gets a new port)."""
    with _PORT_LOCK:
        for _ in range(64):
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            if port not in _RECENT_PORTS:
                break
        _RECENT_PORTS.append(port)
        return port


LAUNCH_MODES = ("ranks", "single")


def rank_env(rank: int, world: int, port: int) -> Dict[str, str]:
    """torchrun-style env of one rank of a single-node job."""
    return {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world), "RANK": str(rank),
            "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "NODE_RANK": "0"}


def _ranked(plan: LaunchPlan, base: ReplicaPlan, mode: str) -> LaunchPlan:
    """Expand a single-process replica that asks for N > 1 GPUs into N rank processes."""
    mode = base.env.get("KATIB_AMD_LAUNCH", mode)
    if mode not in LAUNCH_MODES:
        raise JobSpecError("KATIB_AMD_LAUNCH must be one of %s, got %r" % ("/".join(LAUNCH_MODES), mode))
    if base.gpus <= 1 or mode == "single":
        plan.replicas.append(base)
        return plan
    port = free_port()
    plan.share_devices = True
    plan.ports_managed = True
    # split the CPU threads between the ranks (torchrun does the same): N ranks each spinning
    # a full OpenMP pool on a CPU-side collective oversubscribe the host by N x
    threads = max(1, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1) // base.gpus)
    for r in range(base.gpus):
        env = {"OMP_NUM_THREADS": str(threads)}
        env.update(base.env)
        env.update(rank_env(r, base.gpus, port))
        plan.replicas.append(ReplicaPlan("primary" if r == 0 else "rank", r, list(base.argv), env, base.cwd, 1,
                                         r == 0, entrypoint=base.entrypoint, function=base.function))
    return plan


def assign_ports(plan: LaunchPlan) -> None:
    """Fresh rendezvous ports for one launch attempt of a plan whose ports are ours
    (``ports_managed``): ``MASTER_PORT`` (rank plans, PyTorchJob, XGBoostJob), ``DMLC_PS_ROOT_PORT``
    (MXJob) and every task address of a TFJob's ``TF_CONFIG`` cluster, all from free_port's ledger.
    A retry after a backoff or a wait for GPU slots never reuses a port a previous attempt's rank
    may still hold."""
    if not plan.ports_managed or not plan.replicas:
        return
    master = free_port()
    cluster = None
    for rep in plan.replicas:
        if "TF_CONFIG" in rep.env and cluster is None:
            old = json.loads(rep.env["TF_CONFIG"])["cluster"]
            cluster = {role: ["127.0.0.1:%d" % free_port() for _ in addrs] for role, addrs in old.items()}
    for rep in plan.replicas:
        if "MASTER_PORT" in rep.env:
            rep.env["MASTER_PORT"] = str(master)
        if "DMLC_PS_ROOT_PORT" in rep.env:
            rep.env["DMLC_PS_ROOT_PORT"] = str(master)
        if "TF_CONFIG" in rep.env:
            cfg = json.loads(rep.env["TF_CONFIG"])
            cfg["cluster"] = cluster
            rep.env["TF_CONFIG"] = json.dumps(cfg)


def make_plan(run_spec: Dict, primary_container: str, primary_pod_labels: Optional[Dict[str, str]] = None,
              multi_gpu_launch: str = "ranks") -> LaunchPlan:
    kind = run_spec.get("kind", "")
    spec = run_spec.get("spec") or {}
    if kind == C.JOB_KIND_JOB:
        pod = (spec.get("template") or {}).get("spec") or {}
        c = _container(pod, primary_container)
        plan = LaunchPlan(kind=kind, deadline=float(spec.get("activeDeadlineSeconds") or 0),
                          backoff_limit=int(spec["backoffLimit"]) if "backoffLimit" in spec else 0)
        return _ranked(plan, ReplicaPlan("primary", 0, _argv(c), _env(c), c.get("workingDir"), _gpus(c), True),
                       multi_gpu_launch)
    if kind == C.JOB_KIND_LOCAL:
        plan = LaunchPlan(kind=kind, deadline=float(spec.get("activeDeadlineSeconds") or 0),
                          backoff_limit=int(spec.get("backoffLimit") or 0))
        env = {e["name"]: str(e["value"]) for e in spec.get("env") or [] if "value" in e}
        args = [str(a) for a in spec.get("args") or []]
        gpus = int(spec.get("gpus") or 0)
        if spec.get("entrypoint"):
            base = ReplicaPlan("primary", 0, args, env, spec.get("workingDir"), gpus, True,
                               entrypoint=spec["entrypoint"])
        else:
            cmd = [str(a) for a in spec.get("command") or []] + args
            if not cmd:
                raise JobSpecError("LocalProcess needs spec.command or spec.entrypoint")
            base = ReplicaPlan("primary", 0, cmd, env, spec.get("workingDir"), gpus, True)
        return _ranked(plan, base, multi_gpu_launch)
    if kind == "Function":
        plan = LaunchPlan(kind=kind, deadline=float(spec.get("activeDeadlineSeconds") or 0))
        env = {e["name"]: str(e["value"]) for e in spec.get("env") or [] if "value" in e}
        plan.replicas.append(ReplicaPlan("primary", 0, [], env, spec.get("workingDir"), int(spec.get("gpus") or 0),
                                         True, function={"source": spec.get("source", ""),
                                                         "entry": spec.get("entry", ""),
                                                         "params": spec.get("params", {}),
                                                         "packages": spec.get("packages", [])}))
        return plan
    if kind in _REPLICA_KEYS:
        key, roles = _REPLICA_KEYS[kind]
        rspecs = spec.get(key) or {}
        if not rspecs:
            raise JobSpecError("%s has no %s" % (kind, key))
        plan = LaunchPlan(kind=kind, deadline=float((spec.get("runPolicy") or {}).get("activeDeadlineSeconds")
                                                    or spec.get("activeDeadlineSeconds") or 0), share_devices=True)
        primary_role = _PRIMARY_ROLE[kind]
        if kind == "TFJob" and "Chief" not in rspecs and "Master" in rspecs:
            primary_role = "Master"
        ordered = [r for r in roles if r in rspecs] + [r for r in rspecs if r not in roles]
        if primary_role not in rspecs:
            primary_role = ordered[0]
        world = sum(int(rspecs[r].get("replicas", 1)) for r in ordered
                    if not (kind == "MPIJob" and r == "Launcher"))
        plan.ports_managed = True
        port = free_port()
        rank = 0
        cluster = {}
        for role in ordered:  # every task address through free_port's ledger (never port arithmetic)
            n = int(rspecs[role].get("replicas", 1))
            cluster[role.lower()] = ["127.0.0.1:%d" % free_port() for _ in range(n)]
        for role in ordered:
            rs = rspecs[role]
            pod = ((rs.get("template") or {}).get("spec")) or {}
            c = _container(pod, primary_container)
            n = int(rs.get("replicas", 1))
            for i in range(n):
                env = {"OMP_NUM_THREADS": str(max(1, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
                                                  // max(1, world)))}
                env.update(_env(c))
                if kind in ("PyTorchJob", "XGBoostJob"):
                    # all replicas run on this node: LOCAL_RANK = RANK, and every replica sees the
                    # trial's devices (share_devices), so rank r drives device r % device_count
                    env.update(rank_env(rank, world, port))
                    env["PET_NNODES"] = str(world)
                elif kind == "TFJob":
                    env["TF_CONFIG"] = json.dumps({"cluster": cluster, "task": {"type": role.lower(), "index": i}})
                elif kind == "MXJob":
                    env.update({"DMLC_ROLE": role.lower(), "DMLC_PS_ROOT_URI": "127.0.0.1",
                                "DMLC_PS_ROOT_PORT": str(port)})
                is_primary = role == primary_role and i == 0
                if kind == "MPIJob" and role == "Worker":
                    continue  # mpirun in the launcher spawns the workers itself
                plan.replicas.append(ReplicaPlan(role.lower(), i, _argv(c), env, c.get("workingDir"), _gpus(c),
                                                 is_primary))
                rank += 1
        return plan
    raise JobSpecError("unsupported trial kind %r (supported: Job, %s, LocalProcess, Function)"
                       % (kind, ", ".join(_REPLICA_KEYS)))


def job_status(kind: str, phase: str, reason: str = "", message: str = "") -> Dict:
    """phase: Created | Running | Succeeded | Failed."""
    conds = []
    if kind in _REPLICA_KEYS:
        conds.append({"type": "Created", "status": "True"})
        if phase in ("Running", "Succeeded", "Failed"):
            conds.append({"type": "Running", "status": "True" if phase == "Running" else "False"})
        if phase == "Succeeded":
            conds.append({"type": "Succeeded", "status": "True", "reason": reason, "message": message})
        if phase == "Failed":
            conds.append({"type": "Failed", "status": "True", "reason": reason, "message": message})
        return {"status": {"conditions": conds}}
    st = {"active": 1 if phase == "Running" else 0, "succeeded": 1 if phase == "Succeeded" else 0,
          "failed": 1 if phase == "Failed" else 0}
    if phase == "Succeeded":
        conds.append({"type": "Complete", "status": "True", "reason": reason, "message": message})
    elif phase == "Failed":
        conds.append({"type": "Failed", "status": "True", "reason": reason, "message": message})
    st["conditions"] = conds
    return {"status": st}


def map_paths(values: List[str], mapping: Dict[str, str]) -> List[str]:
    out = []
    for v in values:
        for src, dst in mapping.items():
            if src and src in v:
                v = v.replace(src, dst)
        out.append(v)
    return out


def path_mapping(trial_dir: str, paths: List[str]) -> Dict[str, str]:
    """Absolute collector paths (``/var/log/katib/...``) are remapped under the
    trial directory so concurrent trials never share a metrics file."""
    mapping = {}
    for p in paths:
        if p and os.path.isabs(p):
            d = p.rstrip("/")
            mapping[d] = os.path.join(trial_dir, "fs") + d
    # longest first so nested paths map correctly
    return dict(sorted(mapping.items(), key=lambda kv: -len(kv[0])))
