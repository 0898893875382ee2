"""PyTorch (Fashion)MNIST CNN trial with optional data parallelism (reference
``examples/v1beta1/trial-images/pytorch-mnist/mnist.py:32-205``).

Same network (Conv 1->20 5x5, pool, Conv 20->50 5x5, pool, FC 800->500, FC 500->10,
log-softmax / NLL, SGD with momentum), same CLI (``--lr``, ``--momentum``,
``--batch-size``, ``--epochs``, ``--log-interval``, ``--backend``, ``--log-path``,
``--logger {standard,hypertune}``), same metric lines (``{metricName}={value}``
or hypertune JSON into ``--log-path``). As a ``PyTorchJob`` trial every replica is a
rank (``WORLD_SIZE``/``RANK``/``MASTER_ADDR`` set by the scheduler) and gradients are
averaged with one flat all-reduce per step over ``--backend`` (``nccl`` = RCCL over
xGMI on MI355X, or ``gloo``); only rank 0 prints metrics (the primary replica).
``--tb-dir`` additionally writes TensorBoard event files for the TFEvent collector.
Data: a synthetic 28x28 teacher task resident on the device.
"""

from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel.comm import Comm


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(4 * 4 * 50, 500)
        self.fc2 = nn.Linear(500, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.conv1(x)), 2, 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2, 2)
        x = F.relu(self.fc1(x.view(-1, 4 * 4 * 50)))
        return F.log_softmax(self.fc2(x), dim=1)


def parse_args(argv):
    p = argparse.ArgumentParser(description="PyTorch MNIST trial (katib-amd)")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--test-batch-size", type=int, default=1000)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--log-interval", type=int, default=10)
    p.add_argument("--log-path", type=str, default="")
    p.add_argument("--logger", type=str, choices=["standard", "hypertune"], default="standard")
    p.add_argument("--backend", type=str, default="nccl" if torch.cuda.is_available() else "gloo")
    p.add_argument("--num-train", type=int, default=60000)
    p.add_argument("--num-test", type=int, default=10000)
    p.add_argument("--tb-dir", type=str, default="")
    return p.parse_args(argv)


def _data(n, seed, dev):
    g = torch.Generator().manual_seed(seed)
    protos = torch.randn(10, 1, 7, 7, generator=g)
    y = torch.randint(0, 10, (n,), generator=g)
    x = F.interpolate(protos[y], size=(28, 28), mode="bilinear", align_corners=False) + \
        0.8 * torch.randn(n, 1, 28, 28, generator=g)
    return x.to(dev), y.to(dev)


def main(argv=None):
    args = parse_args(argv if argv is not None else [])
    # DDP (mnist.py:130-133,164-166,189-192): one rank per GPU, rank r on device LOCAL_RANK %
    # device_count; ranks sharing a GPU fall back to gloo + the one-shot IPC all-reduce (Comm)
    comm = Comm.from_env("cpu" if args.no_cuda or not torch.cuda.is_available() else "cuda",
                         backend=args.backend if args.backend != "mpi" else None)
    ws, rank, dev = comm.world_size, comm.rank, comm.device
    torch.manual_seed(args.seed)
    dist = comm if comm.distributed else None
    if dist is not None and dev.type == "cuda":
        comm.enable_xgmi()
    x, y = _data(args.num_train + args.num_test, 55, dev)
    tx, ty, vx, vy = x[:args.num_train], y[:args.num_train], x[args.num_train:], y[args.num_train:]
    model = Net().to(dev)
    params = list(model.parameters())
    if dist is not None:
        flat = torch.nn.utils.parameters_to_vector(params).detach()
        comm.broadcast_(flat, 0)
        torch.nn.utils.vector_to_parameters(flat, params)
    opt = torch.optim.SGD(params, lr=args.lr, momentum=args.momentum)
    writer = None
    if args.tb_dir and rank == 0:
        from ..metricscollector.tfevent import EventWriter

        writer = EventWriter(os.path.join(args.tb_dir, "test"))
    log_file = None
    if args.log_path and args.logger == "standard" and rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(args.log_path)), exist_ok=True)
        log_file = open(args.log_path, "a")

    def log(msg):  # logging.info to --log-path when set, else stdout (mnist.py:150-156)
        if rank != 0:
            return
        if log_file is not None:
            log_file.write(msg + "\n")
            log_file.flush()
        else:
            print(msg, flush=True)

    shard = args.num_train // ws
    gen = torch.Generator(device=dev).manual_seed(args.seed + rank)
    step = 0
    for epoch in range(1, args.epochs + 1):
        model.train()
        perm = torch.randperm(shard, device=dev, generator=gen) + rank * shard
        nb = shard // args.batch_size
        for b in range(nb):
            idx = perm[b * args.batch_size:(b + 1) * args.batch_size]
            loss = F.nll_loss(model(tx[idx]), ty[idx])
            opt.zero_grad()
            loss.backward()
            if dist is not None:
                g = torch.cat([p.grad.reshape(-1) for p in params])
                comm.allreduce_mean_(g)
                torch.nn.utils.vector_to_parameters(g, [p.grad for p in params])
            opt.step()
            step += 1
            if b % args.log_interval == 0:
                log("Train Epoch: {} [{}/{} ({:.0f}%)]\tloss={:.4f}".format(
                    epoch, b * args.batch_size * ws, args.num_train, 100.0 * b / max(nb, 1), float(loss)))
        model.eval()
        with torch.no_grad():
            out = torch.cat([model(vx[i:i + args.test_batch_size]) for i in range(0, args.num_test,
                                                                                    args.test_batch_size)])
            test_loss = float(F.nll_loss(out, vy, reduction="sum")) / args.num_test
            acc = float((out.argmax(1) == vy).float().mean())
        if rank == 0:
            if args.logger == "hypertune" and args.log_path:
                os.makedirs(os.path.dirname(os.path.abspath(args.log_path)), exist_ok=True)
                with open(args.log_path, "a") as f:
                    f.write(json.dumps({"metric": "accuracy", "accuracy": str(acc), "timestamp": time.time()}) +
                            "\n")
                    f.write(json.dumps({"metric": "loss", "loss": str(test_loss), "timestamp": time.time()}) + "\n")
            else:
                log("{{metricName: accuracy, metricValue: {:.4f}}};{{metricName: loss, metricValue: {:.4f}}}"
                    .format(acc, test_loss))
            if writer is not None:
                writer.add_scalar("accuracy", acc, epoch)
                writer.add_scalar("loss", test_loss, epoch)
    if writer is not None:
        writer.close()
    if log_file is not None:
        log_file.close()
    if dist is not None:
        comm.barrier()
        comm.destroy()
    return acc


if __name__ == "__main__":
    import sys

    main(sys.argv[1:])
