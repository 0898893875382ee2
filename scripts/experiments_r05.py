#!/usr/bin/env python3
"""Experiment-level numbers of the BASELINE configs on one MI355X, each run
through the in-process scheduler from create to completion (all trial slots on GPU 0):

* ``darts-b5``: examples/nas/darts-cifar10.yaml - the reference's B5 number (282 s) is exactly this
  span, Experiment create -> Succeeded (``examples/v1beta1/sdk/nas-with-darts.ipynb:487,727-740``);
* ``hyperband-resnet18``: examples/early-stopping/hyperband-medianstop-resnet18.yaml with the goal
  removed so it runs to maxTrialCount (trials completed / early-stopped, trials per hour);
* ``pbt-gpt2``: examples/pbt/pbt-gpt2-small.yaml cut to ``--pbt-trials`` (two generations of 8):
  per-generation wall clock and the exploit hand-off (checkpoint source, load seconds, bytes) parsed
  from the members' logs.

One JSON line per experiment; ``--only NAME`` runs one.
"""
import argparse
import json
import os
import re
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _metrics_lines(run):
    try:
        with open(os.path.join(run.trial_dir, "metrics.log")) as f:
            return f.read().splitlines()
    except OSError:
        return []


def run_experiment(name, path, slots, mutate=None, timeout=900):
    from katib_amd.api.conditions import ExperimentConditions as EC
    from katib_amd.api.yaml_io import load_experiment
    from katib_amd.controller.config import detect_gpus
    from katib_amd.controller.manager import Manager

    e = load_experiment(os.path.join(ROOT, path))
    if mutate:
        mutate(e)
    n = detect_gpus()
    m = Manager(state_dir=tempfile.mkdtemp(prefix="katib-exp-"), num_devices=n, journal=False)
    m.config.amd.slots_per_device = slots
    m.slots = m.N.SlotPool(m.n_devices, slots)
    t0 = time.time()
    m.create_experiment(e)
    done = m.run_until_complete(e.metadata.name, timeout=timeout)
    wall = time.time() - t0
    trials = m.list_trials(e.metadata.name)
    st = done.status
    out = {"experiment": name, "file": path, "n_gpus": n, "slots_per_gpu": slots, "wall_s": round(wall, 2),
           "condition": done.status.conditions[-1].type if done.status.conditions else None,
           "reason": done.status.conditions[-1].reason if done.status.conditions else None,
           "trials": len(trials), "succeeded": st.trials_succeeded or 0, "failed": st.trials_failed or 0,
           "early_stopped": st.trials_early_stopped or 0, "killed": st.trials_killed or 0,
           "succeeded_ok": EC.is_succeeded(done)}
    completed = out["succeeded"] + out["failed"] + out["early_stopped"] + out["killed"]
    out["completed_trials_per_hour"] = round(completed / wall * 3600.0, 1)
    best = st.current_optimal_trial
    if best is not None and best.observation is not None:
        out["best"] = {mt.name: mt.latest for mt in best.observation.metrics or []}
    runs = {k[1]: r for k, r in m.runs.items()}
    durs = [r.finished - r.started for r in runs.values() if r.started and r.finished]
    if durs:
        out["median_trial_s"] = round(statistics.median(durs), 3)
    if name == "pbt-gpt2":
        gens = {}
        for t in trials:
            g = (t.metadata.labels or {}).get("pbt.suggestion.katib.kubeflow.org/generation")
            r = runs.get(t.metadata.name)
            if g is None or r is None or not r.started or not r.finished:
                continue
            a, b = gens.get(g, (r.started, r.finished))
            gens[g] = (min(a, r.started), max(b, r.finished))
        out["generation_wall_s"] = {g: round(b - a, 2) for g, (a, b) in sorted(gens.items(), key=lambda kv: int(kv[0]))}
        hand = []
        for r in runs.values():
            for ln in _metrics_lines(r):
                if "checkpoint_source=" in ln:
                    kv = dict(re.findall(r"([\w-]+)=(\S+)", ln))
                    hand.append(kv)
        p2p = [h for h in hand if h.get("checkpoint_source") == "p2p"]
        out["exploit_handoffs"] = {
            "loads": len(hand), "p2p": len(p2p), "file": sum(1 for h in hand if h.get("checkpoint_source") == "file"),
            "median_load_s": round(statistics.median(float(h["checkpoint_load_seconds"]) for h in hand), 4) if hand else None,
            "median_p2p_load_s": round(statistics.median(float(h["checkpoint_load_seconds"]) for h in p2p), 4) if p2p else None,
            "bytes": int(float(hand[0]["checkpoint_bytes"])) if hand and "checkpoint_bytes" in hand[0] else None}
        if out["exploit_handoffs"]["bytes"] and out["exploit_handoffs"]["median_p2p_load_s"]:
            out["exploit_handoffs"]["p2p_GB_per_s"] = round(
                out["exploit_handoffs"]["bytes"] / out["exploit_handoffs"]["median_p2p_load_s"] / 1e9, 2)
    m.shutdown()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--pbt-trials", type=int, default=16)
    ap.add_argument("--hb-trials", type=int, default=32)
    a = ap.parse_args()

    def hb(e):
        e.spec.objective.goal = None  # run to maxTrialCount
        e.spec.max_trial_count = a.hb_trials

    def pbt(e):
        e.spec.max_trial_count = a.pbt_trials

    plan = [("darts-b5", "examples/nas/darts-cifar10.yaml", None),
            ("hyperband-resnet18", "examples/early-stopping/hyperband-medianstop-resnet18.yaml", hb),
            ("pbt-gpt2", "examples/pbt/pbt-gpt2-small.yaml", pbt)]
    for name, path, mut in plan:
        if a.only and name != a.only:
            continue
        print(json.dumps(run_experiment(name, path, a.slots, mut)), flush=True)


if __name__ == "__main__":
    main()
