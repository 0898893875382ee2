"""Toy PBT trial (reference ``examples/v1beta1/trial-images/simple-pbt/pbt_test.py:31-127``).

A scalar "accuracy" climbs at a rate set by how close ``--lr`` is to a triangle-wave
optimum that moves with the training step; the state ``{step, accuracy}`` lives in
``training.json`` in the checkpoint directory and every trial resumes from it (the
PBT suggestion service seeds the directory from the parent). Prints
``Validation-accuracy=<a>`` per step. Runs at least ``--min-seconds`` like the
reference so concurrent members overlap.
"""

from __future__ import annotations

import argparse
import json
import os
import time


def optimal_lr(step: int, period: int = 40, lo: float = 0.0001, hi: float = 0.02) -> float:
    phase = (step % period) / period
    tri = 2 * phase if phase < 0.5 else 2 * (1 - phase)
    return lo + (hi - lo) * tri


def main(argv=None):
    p = argparse.ArgumentParser(description="simple PBT toy trial")
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--epochs", type=int, default=20)
    p.add_argument("--checkpoint", default=os.environ.get("KATIB_TRIAL_CHECKPOINT_DIR", "."))
    p.add_argument("--min-seconds", type=float, default=0.0)
    args = p.parse_args(argv if argv is not None else [])
    t0 = time.time()
    os.makedirs(args.checkpoint, exist_ok=True)
    path = os.path.join(args.checkpoint, "training.json")
    st = {"step": 0, "accuracy": 0.0}
    if os.path.exists(path):
        with open(path) as f:
            st = json.load(f)
    for _ in range(args.epochs):
        dist = abs(args.lr - optimal_lr(st["step"])) / 0.02
        st["accuracy"] += (1.0 - st["accuracy"]) * max(0.0, 0.05 * (1.0 - dist))
        st["step"] += 1
        print("Validation-accuracy=%.6f" % st["accuracy"], flush=True)
    with open(path, "w") as f:
        json.dump(st, f)
    rest = args.min_seconds - (time.time() - t0)
    if rest > 0:
        time.sleep(rest)
    return st["accuracy"]


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
