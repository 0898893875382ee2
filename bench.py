#!/usr/bin/env python3
"""Headline benchmark: DARTS CIFAR-10 search wall-clock (BASELINE.md B5 / BASELINE.json config 4).

Runs the flagship workload - one full DARTS search step (second-order architect:
5 forward + 5 backward passes, Adam on alphas, clipped SGD on weights) - on N
GPUs of one node, one process per GPU (torchrun env; one-shot xGMI / RCCL
all-reduce of the flat gradient buffers inside the captured step). Times exactly
``--steps`` steps after ``--warmup`` untimed steps, bracketed by barrier +
synchronize, MAX over ranks, then projects the reference's end-to-end search:
``epochs x (steps/epoch x step time + validation pass)`` with the B5 config (C=4,
L=2, N=3, stem x1, 6 primitives + none, 25k/25k split, 2 epochs) unless
``--config default`` (darts-gpu.yaml: C=16, L=3, N=4, stem x3).

Scaling: ``--scaling strong`` (default) keeps B5's global batch of 128 at every N,
each rank taking 128/N rows, so every N runs the same search (196 steps per epoch);
``--scaling weak`` keeps 128 rows per GPU (global batch 128 N: a different search,
labelled as such).

The same JSON line also carries
* ``trials_per_hour``: BASELINE config 2 end to end through the scheduler (TPE over the
  MNIST MLP, ``--trial-slots`` trials per GPU at a time over all N GPUs, warm workers), run by rank 0
  in a child process *before* any rank touches the GPU (``bench_trials.py``);
* ``torch_eager_ms_per_step``: the same search step on the PyTorch op backend launched
  eagerly (MIOpen / hipBLASLt / PyTorch kernels, no HIP graph), a same-node comparator.

Lower is better; vs_baseline = value / 282 s (B5, 1x NVIDIA GPU, end to end).
Data: synthetic CIFAR-10-shaped tensors resident in HBM, random-init weights.

``--dtype bf16`` (secondary config, BASELINE.json config 4's precision): the DARTS edge kernels
of the ``_hipkern_zbf16`` build store the per-op intermediates (depthwise outputs, pre-BN op
outputs) as bf16; node states, gradients, BN statistics, weights and all arithmetic stay fp32.
The headline (default) is fp32 like the reference.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

B5_SECONDS = 282.0
PRIMS = ["separable_convolution_3x3", "dilated_convolution_3x3", "dilated_convolution_5x5", "avg_pooling_3x3",
         "max_pooling_3x3", "skip_connection"]
CONFIGS = {
    "b5": dict(init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1, epochs=2),
    "default": dict(init_channels=16, num_layers=3, num_nodes=4, stem_multiplier=3, epochs=3),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="b5", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=128, help="global batch (strong) / per-GPU batch (weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--trials", type=int, default=12, help="trials per GPU of the trials/hour experiment (0: skip)")
    ap.add_argument("--trial-slots", type=int, default=1,
                    help="concurrent trials per GPU in the trials/hour experiment (warm workers per GPU)")
    ap.add_argument("--comparator-steps", type=int, default=5,
                    help="steps of each same-GPU comparator (torch ops eager / torch ops in a HIP graph / the "
                         "nn.Module trainer eager; 0: skip)")
    ap.add_argument("--b1", type=int, default=1,
                    help="also run the B1-shaped experiment (examples/hp-tuning/b1-random-mnist-mlp.yaml: random "
                         "search, 12 cold batch/v1 Job trials, 3 in parallel) -> b1_trials_per_hour")
    ap.add_argument("--experiment", type=int, default=1,
                    help="also run examples/nas/darts-cifar10.yaml through the scheduler, Experiment create -> "
                         "Succeeded (the span the reference's 282 s measures) -> b5_experiment_wall_s")
    ap.add_argument("--capture", type=int, default=1)
    ap.add_argument("--ops", default=os.environ.get("KATIB_AMD_DARTS_OPS", "hip"))
    ap.add_argument("--valid-batches", type=int, default=10)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: per-op intermediates stored as bf16 (the _hipkern_zbf16 build)")
    ap.add_argument("--full-search", type=int, default=-1,
                    help="also run the whole search (epochs x (steps/epoch train steps + validation)) and report "
                         "its measured wall clock next to the projection (-1: on for the b5 config)")
    ap.add_argument("--floor", type=int, default=1,
                    help="N>1: rank 0 also times a dp1 step at the per-rank batch (per_rank_floor_ms)")
    ap.add_argument("--hessian", default="concurrent", choices=["stacked", "concurrent", "sequential"],
                    help="finite-difference Hessian passes: two concurrent graph branches (default), stacked into "
                         "shared launches (profiles/darts_hessian_stacked_ab_r06.log), or one after the other")
    ap.add_argument("--per-rank-bn", type=int, default=1,
                    help="N>1 with SyncBN: also time the step with per-rank BatchNorm (DDP semantics) -> "
                         "per_rank_bn_ms_per_step")
    ap.add_argument("--sync-bn", type=int, default=-1,
                    help="BatchNorm statistics over the global batch (all ranks) instead of per rank; "
                         "-1: on for strong scaling (keeps B5's BN over 128 images at every N)")
    args = ap.parse_args()
    if args.sync_bn < 0:
        args.sync_bn = 1 if args.scaling == "strong" else 0

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N`: become N ranks, one per GPU, before anything touches the GPU
        return self_launch(args.gpus)
    ws_env = int(os.environ.get("WORLD_SIZE", "1"))
    if ws_env != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d; refusing to time a different world size"
              % (ws_env, args.gpus), file=sys.stderr)
        return 2

    if args.dtype == "bf16" and not os.environ.get("KATIB_AMD_HIPKERN"):
        # the variant extension replaces the fp32 one module-wide: rerun in a child that loads it
        # (before this process touches the GPU; the child inherits the torchrun env)
        from katib_amd import _build

        env = dict(os.environ, KATIB_AMD_HIPKERN=_build.zbf16_target())
        return subprocess.call([sys.executable] + sys.argv, env=env)

    # trials/hour (BASELINE config 2) first, from rank 0, before this process touches the GPU:
    # the scheduler's warm workers then own every GPU while the experiment runs
    tph = b1 = b5x = None
    if args.trials > 0 and int(os.environ.get("RANK", "0")) == 0:
        tph = trials_per_hour(args.gpus, args.trials, args.trial_slots)
    if args.b1 and int(os.environ.get("RANK", "0")) == 0:
        b1 = b1_trials_per_hour(args.gpus)
    if args.experiment and int(os.environ.get("RANK", "0")) == 0 and args.config == "b5":
        b5x = b5_experiment()

    import torch

    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops
    from katib_amd.parallel.comm import Comm
    from katib_amd.workloads.data import cifar10

    comm = Comm.from_env()
    dev = comm.device
    if dev.type == "cuda" and args.ops == "hip":
        try:
            dops.set_backend("hip")
            from katib_amd.ops import hip_darts  # noqa: F401  (fails loudly if the extension is missing)
            if args.dtype == "bf16" and hip_darts.ZDT != torch.bfloat16:
                raise RuntimeError("--dtype bf16 needs the _hipkern_zbf16 build (KATIB_AMD_HIPKERN)")
        except Exception as e:
            if comm.rank == 0:
                print("hip ops unavailable (%s); using torch ops" % e, file=sys.stderr)
            dops.set_backend("torch")
            args.ops = "torch"
    if dev.type != "cuda":
        args.ops = "torch"
    cfg = CONFIGS[args.config]
    layout = DartsLayout(PRIMS, init_channels=cfg["init_channels"], num_layers=cfg["num_layers"],
                         num_nodes=cfg["num_nodes"], stem_multiplier=cfg["stem_multiplier"])
    sync_bn = bool(args.sync_bn) and comm.distributed
    search = DartsSearch(layout, dev, comm, capture=bool(args.capture) and dev.type == "cuda", sync_bn=sync_bn,
                         hessian=args.hessian)
    n_train = 50000
    ds = cifar10(dev, n=n_train)
    train, valid = ds.subset(0, n_train // 2), ds.subset(n_train // 2, n_train)
    if args.scaling == "strong":
        bs = max(1, args.batch // comm.world_size)  # global batch stays args.batch
    else:
        bs = args.batch
    tb = train.batches(bs, seed=0, shard=comm.rank, num_shards=comm.world_size, drop_last=True)
    vb = valid.batches(bs, seed=1, shard=comm.rank, num_shards=comm.world_size, drop_last=True)
    batches = []
    for i, (t, v) in enumerate(zip(tb, vb)):
        batches.append((t, v))
        if len(batches) >= 16:
            break

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for i in range(args.warmup):
        (tx, ty), (vx, vy) = batches[i % len(batches)]
        search.step(tx, ty, vx, vy)
    sync()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        (tx, ty), (vx, vy) = batches[i % len(batches)]
        search.step(tx, ty, vx, vy)
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    ms_step = comm.allreduce_max(dt * 1000.0 / args.steps)
    loss = float(search.loss_out)

    # validation pass cost (no_grad forward, BN in eval mode) -- part of every search epoch; the
    # validation batches go EVAL_GROUP at a time through one captured forward (the same losses and
    # correct counts: eval-mode BN is per sample), timed per original batch
    from katib_amd.models.darts_search import EVAL_GROUP, eval_groups

    nv = min(len(batches), -(-max(args.valid_batches, 1) // EVAL_GROUP) * EVAL_GROUP)  # whole groups
    vbatches = [v for _, v in batches][:nv]
    vgroups = list(eval_groups(vbatches))
    for vx, vy in (vgroups[0], vgroups[-1]):  # every group shape captured before timing
        search.evaluate(vx, vy)
    sync()
    t1 = time.perf_counter()
    for vx, vy in vgroups:
        search.evaluate(vx, vy)
    sync()
    ms_valid = comm.allreduce_max((time.perf_counter() - t1) * 1000.0 / max(len(vbatches), 1))

    steps_per_epoch = math.ceil((n_train // 2) / (bs * comm.world_size))
    epoch_s = steps_per_epoch * ms_step / 1000.0 + steps_per_epoch * ms_valid / 1000.0
    wall = cfg["epochs"] * epoch_s

    # cross-check of the projection: the whole search, end to end (train steps + per-epoch validation)
    full_s = None
    if args.full_search > 0 or (args.full_search < 0 and args.config == "b5"):
        sync()
        comm.barrier()
        sync()
        t2 = time.perf_counter()
        for _ in range(cfg["epochs"]):
            for i in range(steps_per_epoch):
                (tx, ty), (vx, vy) = batches[i % len(batches)]
                search.step(tx, ty, vx, vy)
            for vx, vy in eval_groups(vbatches[i % len(vbatches)] for i in range(steps_per_epoch)):
                search.evaluate(vx, vy)
        sync()
        comm.barrier()
        sync()
        full_s = comm.allreduce_max(time.perf_counter() - t2)

    # the reference's own data-parallel semantic (DDP with per-rank BatchNorm,
    # examples/v1beta1/trial-images/pytorch-mnist/mnist.py:190-191) next to the SyncBN headline: the
    # same search step with each rank normalising over its own 128/N images (4 rendezvous per step:
    # the gradient buckets only), timed the same way on every rank
    per_rank_bn_ms = ms_step if (comm.distributed and not sync_bn) else None
    if comm.distributed and sync_bn and args.per_rank_bn:
        prb = DartsSearch(layout, dev, comm, capture=bool(args.capture) and dev.type == "cuda", sync_bn=False,
                          hessian=args.hessian)
        for i in range(args.warmup):
            (tx, ty), (vx, vy) = batches[i % len(batches)]
            prb.step(tx, ty, vx, vy)
        sync()
        comm.barrier()
        sync()
        t5 = time.perf_counter()
        for i in range(args.steps):
            (tx, ty), (vx, vy) = batches[i % len(batches)]
            prb.step(tx, ty, vx, vy)
        sync()
        comm.barrier()
        sync()
        per_rank_bn_ms = comm.allreduce_max((time.perf_counter() - t5) * 1000.0 / args.steps)
        del prb
    distinct = comm.distinct_devices() if comm.distributed else 1

    # per-rank floor: what one rank's step costs on its own at the per-rank batch (dp1, rank 0's
    # GPU, the other ranks parked at the barrier) - the best an N-rank step could do without the
    # all-reduces and BN synchronisation
    floor_ms = None
    if comm.distributed and args.floor and dev.type == "cuda":
        if comm.rank == 0:
            solo = DartsSearch(layout, dev, Comm(device=dev), capture=bool(args.capture), hessian=args.hessian)
            for i in range(max(args.warmup, 2)):
                (tx, ty), (vx, vy) = batches[i % len(batches)]
                solo.step(tx, ty, vx, vy)
            sync()
            t4 = time.perf_counter()
            for i in range(args.steps):
                (tx, ty), (vx, vy) = batches[i % len(batches)]
                solo.step(tx, ty, vx, vy)
            sync()
            floor_ms = (time.perf_counter() - t4) * 1000.0 / args.steps
            del solo
        comm.barrier()

    # same-GPU comparators (rank 0 of a 1-rank run): the same search step on the PyTorch op backend
    # launched eagerly (MIOpen / hipBLASLt / PyTorch kernels), the same PyTorch ops captured in a HIP
    # graph (isolates kernel quality from launch overhead), and the reference-shaped nn.Module
    # trainer (models/darts_module.py) run eagerly
    comp = {"torch_eager": None, "torch_graph": None, "module_eager": None}
    if args.comparator_steps > 0 and dev.type == "cuda" and args.dtype == "fp32" and not comm.distributed:
        def timed(obj, warm):
            for i in range(warm):
                (tx, ty), (vx, vy) = batches[i % len(batches)]
                obj.step(tx, ty, vx, vy)
            sync()
            t3 = time.perf_counter()
            for i in range(args.comparator_steps):
                (tx, ty), (vx, vy) = batches[i % len(batches)]
                obj.step(tx, ty, vx, vy)
            sync()
            return (time.perf_counter() - t3) * 1000.0 / args.comparator_steps

        dops.set_backend("torch")
        try:
            comp["torch_eager"] = timed(DartsSearch(layout, dev, Comm(device=dev), capture=False), 2)
        except Exception as e:  # noqa: BLE001 - a comparator must not sink the headline
            print("torch-eager comparator failed: %s" % e, file=sys.stderr)
        try:
            comp["torch_graph"] = timed(DartsSearch(layout, dev, Comm(device=dev), capture=True), 3)
        except Exception as e:  # noqa: BLE001
            print("torch-graph comparator failed: %s" % e, file=sys.stderr)
        dops.set_backend(args.ops)
        try:
            from katib_amd.models.darts_module import ModuleSearch

            comp["module_eager"] = timed(ModuleSearch(PRIMS, cfg["init_channels"], cfg["num_layers"],
                                                      cfg["num_nodes"], cfg["stem_multiplier"], dev), 2)
        except Exception as e:  # noqa: BLE001
            print("module comparator failed: %s" % e, file=sys.stderr)
    torch_ms = comp["torch_eager"]
    allreduce = (("xgmi-oneshot" if comm.xgmi is not None else ("rccl" if comm.backend == "nccl" else comm.backend))
                 if comm.distributed else None)
    if comm.rank == 0:
        out = {
            "metric": "darts_cifar10_search_wall_clock_s",
            "value": round(wall, 3),
            "unit": "s",
            "n_gpus": args.gpus,
            "ranks_seen": comm.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": False,
            "scaling": args.scaling,
            "vs_baseline": round(wall / B5_SECONDS, 5) if args.config == "b5" else None,
            "dtype": args.dtype,
            "precision": ("fp32" if args.dtype == "fp32" else
                          "bf16 per-op intermediates (d, z); fp32 node states, gradients, BN statistics, weights, math"),
            "data": "synthetic (CIFAR-10-shaped, device-resident); random-init weights",
            "config": {"model": "darts-cnn-cifar10 supernet (%s: C=%d, L=%d, N=%d, stem x%d, 6 primitives + none)"
                                % (args.config, cfg["init_channels"], cfg["num_layers"], cfg["num_nodes"],
                                   cfg["stem_multiplier"]),
                       "global_batch": bs * comm.world_size, "per_gpu_batch": bs, "seq_len": None,
                       "parallelism": "dp%d" % comm.world_size, "epochs": cfg["epochs"],
                       "steps_per_epoch": steps_per_epoch, "ops": args.ops, "hip_graph": bool(search.capture),
                       "allreduce": allreduce, "sync_bn": sync_bn,
                       "second_order": True, "hessian": search.hessian},
            "allreduce": allreduce,
            # one-shot xGMI all-reduce self-test verdict (None at one rank), the SyncBN fold path
            # (xgmi-oneshot / rccl-graph / host), and the cross-rank rendezvous one step issues
            # (gradient buckets + SyncBN folds) and whether they sit inside the captured graph
            "xgmi_self_test": comm.xgmi_status if comm.distributed else None,
            "syncbn_path": search._hsync.path if getattr(search, "_hsync", None) is not None else None,
            "rendezvous_per_step": search.rendezvous_per_step if comm.distributed else 0,
            "rendezvous_serial_per_step": search.rendezvous_serial_per_step if comm.distributed else 0,
            "rendezvous_in_graph": search.rendezvous_in_graph if comm.distributed else None,
            "hessian_stack": search.stack_stats,
            "batchnorm": ("global batch (sync-bn)" if sync_bn else
                          ("per rank" if comm.distributed else "global batch")),
            "per_rank_floor_ms": round(floor_ms, 4) if floor_ms is not None else None,
            # DDP semantics (per-rank BN, the reference's DP); with it the projected search wall clock
            "per_rank_bn_ms_per_step": round(per_rank_bn_ms, 4) if per_rank_bn_ms is not None else None,
            "per_rank_bn_search_wall_s": (round(cfg["epochs"] * steps_per_epoch * (per_rank_bn_ms + ms_valid) / 1000.0, 3)
                                          if per_rank_bn_ms is not None else None),
            # physical GPUs behind the ranks: < n_gpus means a shared-GPU rehearsal (IPC copies on one
            # device, no xGMI link crossed)
            "distinct_devices": distinct,
            "ms_valid_batch": round(ms_valid, 4),
            "measured_search_wall_s": round(full_s, 3) if full_s is not None else None,
            "train_images_per_s": round(bs * comm.world_size * 1000.0 / ms_step, 1),
            "final_loss": round(loss, 4),
            "baseline_b5_s": B5_SECONDS,
            "torch_eager_ms_per_step": round(torch_ms, 3) if torch_ms is not None else None,
            "speedup_vs_torch_eager": round(torch_ms / ms_step, 2) if torch_ms else None,
            "torch_graph_ms_per_step": round(comp["torch_graph"], 3) if comp["torch_graph"] else None,
            "speedup_vs_torch_graph": round(comp["torch_graph"] / ms_step, 2) if comp["torch_graph"] else None,
            "module_eager_ms_per_step": round(comp["module_eager"], 3) if comp["module_eager"] else None,
            "speedup_vs_module_eager": round(comp["module_eager"] / ms_step, 2) if comp["module_eager"] else None,
            "trials_per_hour": tph,
            "b1_trials_per_hour": b1,
            # the reference's B5 span end to end on 1 GPU: the DARTS Experiment through the scheduler
            "b5_experiment_wall_s": b5x.get("wall_s") if b5x else None,
            "b5_experiment": b5x,
        }
        print(json.dumps(out), flush=True)
    comm.destroy()


def self_launch(n: int) -> int:
    """Run this same command as ``n`` ranks under ``torch.distributed.run`` (a CHILD process:
    this one never touches the GPU, so nothing is exec'd after GPU init) and relay rank 0's JSON
    line. The driver's form (torchrun around bench.py) skips this: WORLD_SIZE is then set."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from katib_amd.controller.jobs import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    for ln in r.stdout.splitlines():
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if r.returncode != 0 or len(lines) != 1:
        print("bench.py: %d-rank run failed (rc %d, %d JSON lines)" % (n, r.returncode, len(lines)), file=sys.stderr)
        return r.returncode or 1
    print(lines[0], flush=True)
    return 0


def b5_experiment():
    """examples/nas/darts-cifar10.yaml (the B5 config) through the in-process scheduler, Experiment
    create -> Succeeded, in a child process before this one touches the GPU (scripts/experiments_r05.py)."""
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, os.path.join(here, "scripts", "experiments_r05.py"), "--only", "darts-b5", "--slots", "1"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not line:
            print("B5 experiment failed: %s" % (r.stderr[-2000:],), file=sys.stderr)
            return None
        res = json.loads(line[-1])
    except (subprocess.TimeoutExpired, ValueError) as e:
        print("B5 experiment failed: %s" % e, file=sys.stderr)
        return None
    return {"wall_s": res["wall_s"], "condition": res["condition"], "baseline_b5_s": B5_SECONDS,
            "vs_b5": round(res["wall_s"] / B5_SECONDS, 4), "trial_s": res.get("median_trial_s"),
            "span": "Experiment create -> Succeeded (reference nas-with-darts.ipynb:487,727-740)"}


def b1_trials_per_hour(gpus: int):
    """The reference's B1 experiment shape (docs/workflow-design.md:39-108): random search, 12 trials,
    3 in parallel, lr / num-layers / optimizer of an MNIST MLP at batch 64, each trial a cold
    batch/v1 Job process (examples/hp-tuning/b1-random-mnist-mlp.yaml), on ``gpus`` GPUs."""
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, os.path.join(here, "bench_trials.py"), "--experiment",
           os.path.join(here, "examples", "hp-tuning", "b1-random-mnist-mlp.yaml"), "--gpus", str(gpus)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not line:
            print("B1 experiment failed: %s" % (r.stderr[-2000:],), file=sys.stderr)
            return None
        res = json.loads(line[-1])
    except (subprocess.TimeoutExpired, ValueError) as e:
        print("B1 experiment failed: %s" % e, file=sys.stderr)
        return None
    return {"value": res["value"], "unit": "trials/h", "vs_b1": res["vs_baseline"], "wall_s": res["wall_s"],
            "trials_completed": res["trials_completed"], "median_trial_s": res["median_trial_s"],
            "launcher": res.get("launcher"), "trial_phases_s": res.get("trial_phases_s"),
            "fork_server_start_s": res.get("fork_server_start_s"), "daemon": res.get("daemon"),
            "best_validation_accuracy": res["best_objective"], "n_gpus": gpus,
            "config": "B1 shape: random, 12 trials, parallel 3, cold batch/v1 Job processes (forked from the "
                      "trial fork server unless KATIB_AMD_ZYGOTE=0), MLP lr / "
                      "num-layers / optimizer, batch 64, 3 epochs", "b1_trials_per_hour": 36.3}


def trials_per_hour(gpus: int, per_gpu: int, slots: int = 1):
    """BASELINE config 2 (TPE over the MNIST MLP, examples/hp-tuning/tpe-mnist-mlp.yaml) end to
    end through the in-process scheduler: parallelTrialCount = one trial per GPU,
    ``per_gpu`` trials per GPU, 3 epochs of 60k rows each. Completed trials per hour of wall
    clock from experiment creation to completion (includes warm-worker start). B1, the
    reference's 36.3 trials/h, is a 12-trial random search at parallelTrialCount=3 on a K8s
    CPU cluster (docs/workflow-design.md:41-164): same kind of experiment, not the same
    trial program (the reference's MXNet MLP image is not in the reference tree)."""
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, os.path.join(here, "bench_trials.py"), "--trials", str(per_gpu * gpus), "--parallel",
           str(gpus * slots), "--gpus", str(gpus), "--slots-per-gpu", str(slots), "--epochs", "3"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not line:
            print("trials/hour experiment failed: %s" % (r.stderr[-2000:],), file=sys.stderr)
            return None
        res = json.loads(line[-1])
    except (subprocess.TimeoutExpired, ValueError) as e:
        print("trials/hour experiment failed: %s" % e, file=sys.stderr)
        return None
    return {"value": res["value"], "unit": "trials/h", "n_gpus": gpus, "vs_b1": res["vs_baseline"],
            "wall_s": res["wall_s"], "trials_completed": res["trials_completed"],
            "trials_succeeded": res["trials_succeeded"], "best_validation_accuracy": res["best_validation_accuracy"],
            "config": "tpe-mnist-mlp: %d trials, parallel %d (%d per GPU), 3 epochs x 60k, warm workers"
                      % (res["trials_completed"], gpus * slots, slots), "b1_trials_per_hour": 36.3}


if __name__ == "__main__":
    sys.exit(main())
