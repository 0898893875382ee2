#!/usr/bin/env python3
"""Trials/hour benchmark (36.3 completed trials/hour, random search on an
MNIST MLP, parallelTrialCount=3, K8s CPU jobs).

Runs BASELINE config 2 end to end through the in-process scheduler: a TPE
Experiment over (lr, batch size, hidden width) of the MNIST MLP workload with
``--parallel`` trials spread over the node's GPUs (``--slots-per-gpu`` warm workers
per GPU), and reports completed trials per hour of wall clock from experiment
creation to completion. One process drives all GPUs (no torchrun).

    python bench_trials.py --trials 48 --parallel 8 [--epochs 3] [--num-train 60000]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

B1_TRIALS_PER_HOUR = 36.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=48)
    ap.add_argument("--parallel", type=int, default=8)
    ap.add_argument("--gpus", type=int, default=0, help="0 = all visible")
    ap.add_argument("--slots-per-gpu", type=int, default=0, help="0 = ceil(parallel / gpus)")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--num-train", type=int, default=60000)
    ap.add_argument("--algorithm", default="tpe")
    ap.add_argument("--state-dir", default="")
    ap.add_argument("--experiment", default="",
                    help="run this Experiment YAML as is (trials / parallel / epochs from the file unless given); "
                         "e.g. examples/hp-tuning/b1-random-mnist-mlp.yaml (the reference's B1 shape)")
    ap.add_argument("--warm-daemon", type=int, default=1,
                    help="--experiment: start the scheduler's trial fork server before the clock starts, as the "
                         "long-running daemon (python -m katib_amd serve) has it up from start-up; its start-up time "
                         "is reported as fork_server_start_s. 0: it starts with the first trial (inside the wall)")
    args = ap.parse_args()
    if args.experiment:
        return run_file(args)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from katib_amd.api.conditions import ExperimentConditions as EC
    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.controller.config import detect_gpus
    from katib_amd.controller.manager import Manager

    n_gpus = args.gpus or detect_gpus()
    slots = args.slots_per_gpu or (max(1, -(-args.parallel // n_gpus)) if n_gpus else 1)
    state = args.state_dir or tempfile.mkdtemp(prefix="katib-amd-bench-")
    m = Manager(state_dir=state, num_devices=n_gpus, journal=False)
    m.config.amd.slots_per_device = slots
    m.slots = m.N.SlotPool(m.n_devices, slots)
    e = load_experiment(os.path.join(os.path.dirname(os.path.abspath(__file__)), "examples", "hp-tuning",
                                     "tpe-mnist-mlp.yaml"))
    e.spec.max_trial_count = args.trials
    e.spec.parallel_trial_count = min(args.parallel, args.trials)
    e.spec.max_failed_trial_count = min(e.spec.max_failed_trial_count or 0, args.trials)
    e.spec.objective.goal = None
    e.spec.algorithm.algorithm_name = args.algorithm
    if args.algorithm != "tpe":
        e.spec.algorithm.algorithm_settings = []
    spec = e.spec.trial_template.trial_spec["spec"]
    spec["gpus"] = 1 if n_gpus else 0
    spec["args"] = [a for a in spec["args"] if not a.startswith("--epochs")] + [
        "--epochs=%d" % args.epochs, "--num-train=%d" % args.num_train]
    t0 = time.time()
    m.create_experiment(e)
    done = m.run_until_complete(e.metadata.name, timeout=3 * 3600)
    wall = time.time() - t0
    completed = (done.status.trials_succeeded or 0) + (done.status.trials_failed or 0) + \
        (done.status.trials_early_stopped or 0) + (done.status.trials_killed or 0)
    best = done.status.current_optimal_trial
    best_acc = None
    if best is not None and best.observation is not None:
        for mt in best.observation.metrics or []:
            if mt.name == "Validation-accuracy":
                best_acc = float(mt.max)
    m.shutdown()
    tph = completed / wall * 3600.0
    print(json.dumps({
        "metric": "completed_trials_per_hour", "value": round(tph, 1), "unit": "trials/h", "n_gpus": n_gpus,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": round(tph / B1_TRIALS_PER_HOUR, 2),
        "dtype": "bf16", "data": "synthetic (MNIST-shaped teacher task, device-resident)",
        "wall_s": round(wall, 2), "trials_completed": completed, "trials_succeeded": done.status.trials_succeeded,
        "succeeded": EC.is_succeeded(done), "best_validation_accuracy": best_acc,
        "config": {"experiment": "tpe-mnist-mlp", "algorithm": args.algorithm, "parallel": args.parallel,
                   "max_trials": args.trials, "epochs": args.epochs, "num_train": args.num_train,
                   "slots_per_gpu": slots}}))


def run_file(args):
    """B1-shaped run: the Experiment file as written (cold batch/v1 Job trials, its own algorithm,
    parallelism and budget), trials/hour of wall clock from creation to completion."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from katib_amd.api.conditions import ExperimentConditions as EC
    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.controller.config import detect_gpus
    from katib_amd.controller.manager import Manager

    os.environ.setdefault("KATIB_AMD_TRIAL_PHASES", "1")  # trials print their phase marks (trial_phases)
    e = load_experiment(args.experiment)
    n_gpus = args.gpus or detect_gpus()
    par = e.spec.parallel_trial_count or 3
    slots = args.slots_per_gpu or (max(1, -(-par // n_gpus)) if n_gpus else 1)
    state = args.state_dir or tempfile.mkdtemp(prefix="katib-amd-bench-")
    m = Manager(state_dir=state, num_devices=n_gpus, journal=False)
    m.config.amd.slots_per_device = slots
    m.slots = m.N.SlotPool(m.n_devices, slots)
    if not n_gpus:  # CPU-only node: trials without GPUs
        c = e.spec.trial_template.trial_spec["spec"]["template"]["spec"]["containers"][0]
        c.pop("resources", None)
    zs = None
    if args.warm_daemon and m.config.amd.zygote and os.environ.get("KATIB_AMD_ZYGOTE", "1") != "0":
        tz = time.time()
        m.start_zygote(wait=True)  # the daemon's warm state; not part of the experiment's wall clock
        zs = round(time.time() - tz, 2)
    t0 = time.time()
    m.create_experiment(e)
    done = m.run_until_complete(e.metadata.name, timeout=3 * 3600)
    wall = time.time() - t0
    st = done.status
    completed = sum(int(x or 0) for x in (st.trials_succeeded, st.trials_failed, st.trials_early_stopped,
                                           st.trials_killed))
    best = st.current_optimal_trial
    best_acc = None
    if best is not None and best.observation is not None:
        for mt in best.observation.metrics or []:
            if mt.name == e.spec.objective.objective_metric_name:
                best_acc = float(mt.max)
    per_trial = []
    phases = trial_phases(m, e.metadata.name)
    for t in m.list_trials(e.metadata.name):
        a, b = t.status.start_time, t.status.completion_time
        if a and b:
            if isinstance(a, str):
                from datetime import datetime

                a, b = (datetime.strptime(v, "%Y-%m-%dT%H:%M:%SZ") for v in (a, b))
            per_trial.append((b - a).total_seconds())
    m.shutdown()
    tph = completed / wall * 3600.0
    print(json.dumps({
        "metric": "completed_trials_per_hour", "value": round(tph, 1), "unit": "trials/h", "n_gpus": n_gpus,
        "higher_is_better": True, "vs_baseline": round(tph / B1_TRIALS_PER_HOUR, 2),
        "wall_s": round(wall, 2), "trials_completed": completed, "trials_succeeded": st.trials_succeeded,
        "succeeded": EC.is_succeeded(done), "best_objective": best_acc,
        "median_trial_s": sorted(per_trial)[len(per_trial) // 2] if per_trial else None,
        "median_trial_wall_s": phases.get("total"),
        "trial_phases_s": phases.get("phases"),
        "launcher": phases.get("launcher"),
        "fork_server_start_s": zs, "daemon": "warm (fork server up before create)" if zs is not None else "cold",
        "config": {"experiment": e.metadata.name, "algorithm": e.spec.algorithm.algorithm_name,
                   "parallel": par, "max_trials": e.spec.max_trial_count, "slots_per_gpu": slots,
                   "trial_kind": e.spec.trial_template.trial_spec.get("kind")}}))


PHASES = ["module", "torch", "hip_init", "data", "model", "captured", "first_metric", "trained"]


def trial_phases(m, exp_name):
    """Median cold-trial phase durations (s): launch (scheduler) -> the trial module starts
    importing -> torch imported -> HIP up -> data on device -> model built -> graph captured ->
    first epoch metric -> training done -> reaped (scheduler saw the exit). Trials print
    ``katib-phase`` lines when KATIB_AMD_TRIAL_PHASES=1 (workloads/common.py ``phase``)."""
    import statistics

    rows = []
    launchers = set()
    for (ns, name), run in list(m.runs.items()):
        if not run.trial_dir or not run.started or not run.finished:
            continue
        launchers.add(getattr(run, "launcher", "exec"))
        marks = {}
        try:
            with open(os.path.join(run.trial_dir, "metrics.log")) as f:
                for ln in f:
                    if ln.startswith("katib-phase "):
                        _, k, v = ln.split()
                        marks[k] = float(v)
        except OSError:
            continue
        if not all(k in marks for k in PHASES):
            continue
        seq = [("launch", run.started)] + [(k, marks[k]) for k in PHASES] + [("reaped", run.finished)]
        rows.append({b[0]: b[1] - a[1] for a, b in zip(seq, seq[1:])} | {"total": run.finished - run.started})
    if not rows:
        return {}
    keys = [k for k, _ in zip(PHASES + ["reaped"], range(99))]
    return {"n": len(rows), "total": round(statistics.median(r["total"] for r in rows), 3),
            "launcher": ",".join(sorted(launchers)),
            "phases": {k: round(statistics.median(r[k] for r in rows), 3) for k in keys}}


if __name__ == "__main__":
    sys.exit(main())
