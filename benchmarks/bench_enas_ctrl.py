#!/usr/bin/env python3
"""ENAS controller cost of one GetSuggestions call (reference nas/enas/service.py:238-398):
``controller_train_steps`` REINFORCE steps + sampling ``n`` arcs, for the enas-gpu.yaml
search space (8 layers, 106 operations, hidden 64).

Backends: ``torch`` (host PyTorch, the reference's CPU placement) and ``hip`` (one
persistent-workgroup launch for all train steps + one launch for the arcs). Prints one
JSON line per backend.

    python benchmarks/bench_enas_ctrl.py [--layers 8] [--ops 106] [--steps 50] [--arcs 8] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--ops", type=int, default=106)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--arcs", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--backends", default="torch,hip")
    args = ap.parse_args()
    import torch

    from katib_amd.models.enas_controller import EnasController, EnasControllerHip

    for backend in args.backends.split(","):
        if backend == "hip" and not torch.cuda.is_available():
            continue
        cls = EnasControllerHip if backend == "hip" else EnasController
        c = cls(num_layers=args.layers, num_operations=args.ops, hidden_size=args.hidden, seed=0)
        c.train(0.5, 2)
        c.sample_arcs(args.arcs)
        if backend == "hip":
            torch.cuda.synchronize()
        times = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            c.train(0.5, args.steps)
            arcs = c.sample_arcs(args.arcs)
            if backend == "hip":
                torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        assert len(arcs) == args.arcs
        best = min(times)
        phases = None
        if backend == "hip":  # in-kernel phase split (wall_clock64 at 100 MHz) of one train call
            pc = torch.zeros(5, dtype=torch.int64, device=c.device)
            c._K.enas_train(c.flat, c.m, c.v, c.g, c._tape_for(1),
                            torch.empty(args.steps, c.arc_len, dtype=torch.int32, device=c.device),
                            torch.empty(args.steps, 8, device=c.device), c.base_t, c.num_layers, c.num_operations,
                            c.H, c.cfg, 0.5, args.steps, c.adam_t, c.rng_seed, c.rng_offset, None, pc)
            torch.cuda.synchronize()
            names = ["sample_fwd", "bptt", "weight_grads_mfma", "adam", "stage_w"]
            phases = {n: round(float(v) / 100.0 / args.steps, 2) for n, v in zip(names, pc.cpu().tolist())}
        print(json.dumps({"bench": "enas_controller_get_suggestions", "backend": backend, "layers": args.layers,
                          "ops": args.ops, "hidden": args.hidden, "train_steps": args.steps, "arcs": args.arcs,
                          "ms_per_call": round(best * 1e3, 3), "ms_per_train_step": round(best * 1e3 / args.steps, 4),
                          "n_params": sum(p.numel() for p in c.parameters()),
                          "us_per_step_by_phase": phases}), flush=True)


if __name__ == "__main__":
    main()
