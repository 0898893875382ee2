"""DARTS CIFAR-10 search trial (drop-in for the reference ``darts-cnn-cifar10`` trial image,
``examples/v1beta1/trial-images/darts-cnn-cifar10/run_trial.py``).

Same CLI (``--algorithm-settings``, ``--search-space``, ``--num-layers`` as emitted by
the darts suggestion service), same 50/50 train/valid split, cosine LR schedule,
per-epoch validation and the final ``Best-Genotype=Genotype(...)`` line collected
with the ``([\\w-]+)=(Genotype.*)`` filter. MI355X additions: data-parallel search
across the trial's GPUs (``WORLD_SIZE`` ranks, RCCL), HIP-graph capture of the
search step, the HIP op backend, and synthetic device-resident CIFAR-10.

Data parallelism keeps the reference's algorithm: ``batch_size`` is the *global* batch
(the reference's single-GPU batch) and each of the W ranks takes ``batch_size / W`` rows of
it, so a 1-GPU and an 8-GPU search take the same number of steps per epoch over the same
data. BN batch statistics are per rank (DDP semantics, no SyncBN); the running statistics
used by validation are averaged over the ranks before every validation pass, and the
validation accuracy is the global one, ``sum(correct) / sum(n)`` over all ranks' shards
(the reference averages over the whole valid split, ``run_trial.py:225-255``).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time


def parse_args(argv):
    p = argparse.ArgumentParser(description="DARTS search trial (katib-amd)")
    p.add_argument("--algorithm-settings", type=str, default="")
    p.add_argument("--search-space", type=str, default="")
    p.add_argument("--num-layers", type=str, default="")
    p.add_argument("--num-train", type=int, default=50000, help="train set size before the 50/50 split")
    p.add_argument("--capture", type=int, default=1)
    p.add_argument("--ops", type=str, default=os.environ.get("KATIB_AMD_DARTS_OPS", "hip"))
    p.add_argument("--max-steps", type=int, default=0, help="stop each epoch after N steps (0 = full epoch)")
    return p.parse_args(argv)


def _strip(s: str) -> str:
    s = s.strip()
    if len(s) >= 2 and s[0] == s[-1] == '"':
        s = s[1:-1]
    return s


def validate(search, comm, batches, max_batches: int = 0):
    """Validation pass over this rank's shard -> global (mean loss, top-1) over all ranks.

    BN running statistics are first averaged over the ranks (``sync_bn_stats``); the loss
    and correct counts accumulate on the device (no host sync per batch) and one all-reduce
    of [sum loss*n, sum correct, n] gives ``sum(correct) / sum(n)`` over the whole split."""
    import torch

    from ..models.darts_search import eval_groups

    search.sync_bn_stats()
    acc = torch.zeros(3, dtype=torch.float64, device=search.device)

    def capped():
        for i, b in enumerate(batches):
            if max_batches and i >= max_batches:
                return
            yield b

    # consecutive batches merged per captured forward (models/darts_search.py EVAL_GROUP)
    for vx, vy in eval_groups(capped()):
        loss, top1, _ = search.evaluate(vx, vy)
        acc[:2] += torch.stack([loss, top1]).double() * vy.numel()
        acc[2] += vy.numel()
    comm.allreduce_sum_(acc)
    tot_loss, correct, n = acc.tolist()
    return tot_loss / max(n, 1.0), correct / max(n, 1.0)


def main(argv=None):
    import torch

    from ..models.darts import DartsLayout
    from ..models.darts_search import DartsSearch
    from ..ops import darts as dops
    from ..parallel.comm import Comm
    from .data import cifar10

    args = parse_args(sys.argv[1:] if argv is None else argv)
    settings = json.loads(_strip(args.algorithm_settings).replace("'", '"')) if args.algorithm_settings else {}
    from ..algorithms.nas import DARTS_DEFAULT_SETTINGS

    st = dict(DARTS_DEFAULT_SETTINGS)
    st.update({k: v for k, v in settings.items() if v is not None})
    prims = json.loads(_strip(args.search_space).replace("'", '"')) if args.search_space else [
        "separable_convolution_3x3", "dilated_convolution_3x3", "dilated_convolution_5x5", "avg_pooling_3x3",
        "max_pooling_3x3", "skip_connection"]
    num_layers = int(_strip(args.num_layers)) if args.num_layers else 8
    comm = Comm.from_env()
    dev = comm.device
    if dev.type == "cuda" and args.ops == "hip":
        dops.set_backend("hip")
    torch.manual_seed(2)
    layout = DartsLayout(prims, init_channels=int(st["init_channels"]), num_layers=num_layers,
                         num_nodes=int(st["num_nodes"]), stem_multiplier=int(st["stem_multiplier"]))
    search = DartsSearch(layout, dev, comm, settings=st, capture=bool(args.capture) and dev.type == "cuda")
    ds = cifar10(dev, n=args.num_train)
    split = args.num_train // 2
    train, valid = ds.subset(0, split), ds.subset(split, args.num_train)
    gbs = int(st["batch_size"])  # global batch
    bs = max(1, gbs // comm.world_size)  # per-rank share
    if comm.rank == 0 and bs * comm.world_size != gbs:
        print(">>> batch_size %d is not divisible by %d ranks: global batch %d" % (gbs, comm.world_size,
                                                                                   bs * comm.world_size))
    epochs = int(st["num_epochs"])
    lr_max, lr_min = float(st["w_lr"]), float(st["w_lr_min"])
    print_step = int(st["print_step"])
    if comm.rank == 0:
        print(">>> Algorithm settings", json.dumps(st))
        print(">>> Primitives", layout.prims, "weights", layout.n_weights, "alphas", layout.n_alphas)
    best_top1, best_geno = -1.0, None
    t0 = time.time()
    for epoch in range(epochs):
        lr = lr_min + (lr_max - lr_min) * (1 + math.cos(math.pi * epoch / epochs)) / 2
        search.set_lr(lr)
        tb = train.batches(bs, seed=epoch, shard=comm.rank, num_shards=comm.world_size, drop_last=True)
        vb = valid.batches(bs, seed=1000 + epoch, shard=comm.rank, num_shards=comm.world_size, drop_last=True)
        nsteps = train.steps_per_epoch(bs, comm.world_size)
        for step, ((tx, ty), (vx, vy)) in enumerate(zip(tb, vb)):
            if args.max_steps and step >= args.max_steps:
                break
            search.step(tx, ty, vx, vy)
            if comm.rank == 0 and (step % print_step == 0):
                loss, top1, top5 = search.train_metrics(ty)
                print("Train: [%2d/%d] Step %03d/%03d Loss %.3f Prec@(1,5) (%.1f%%, %.1f%%)"
                      % (epoch + 1, epochs, step, nsteps - 1, loss, 100 * top1, 100 * top5), flush=True)
        # validation (no_grad forward over the valid split): loss / correct counts accumulate on
        # the device (no host sync per batch), then one all-reduce gives the global accuracy
        vbatches = valid.batches(bs, seed=5000 + epoch, shard=comm.rank, num_shards=comm.world_size,
                                 drop_last=True)
        _, top1 = validate(search, comm, vbatches, args.max_steps)
        geno = search.genotype()
        if comm.rank == 0:
            print("Valid: [%2d/%d] Final Prec@1 %.4f%%" % (epoch + 1, epochs, 100 * top1))
            print("Model genotype = %s" % (geno,))
            print("epoch-time=%.3f" % (time.time() - t0), flush=True)
        if top1 > best_top1:
            best_top1, best_geno = top1, geno
    if comm.rank == 0:
        print("Final best Prec@1 = %.4f%%" % (100 * best_top1))
        print("Best-Genotype=%s" % str(best_geno).replace(" ", ""), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
