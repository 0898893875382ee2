"""Rank process for tests/test_gpu_syncbn.py: the HIP DARTS step data-parallel over W ranks that
share the box's GPU (gloo control plane, one-shot IPC all-reduces and the fused SyncBN fold
inside the captured graph), each rank on 1/W of the global batch; afterwards rank 0 runs the
single-process step on the whole batch. With SyncBN both are the same search."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from katib_amd.models.darts import DartsLayout  # noqa: E402
from katib_amd.models.darts_search import DartsSearch  # noqa: E402
from katib_amd.ops import darts as dops  # noqa: E402
from katib_amd.parallel.comm import Comm  # noqa: E402


def main():
    comm = Comm.from_env("cuda")
    dev = comm.device
    dops.set_backend("hip")
    sync = os.environ.get("SYNC_BN", "1") == "1"
    steps = int(os.environ.get("STEPS", "30"))
    layout = DartsLayout(["separable_convolution_3x3", "dilated_convolution_3x3", "dilated_convolution_5x5",
                          "avg_pooling_3x3", "max_pooling_3x3", "skip_connection"], init_channels=4, num_layers=2,
                         num_nodes=3, stem_multiplier=1)
    B, W, r = 64, comm.world_size, comm.rank
    g = torch.Generator().manual_seed(11)
    # a learnable task (class-dependent channel means) and a larger alpha lr, as in the 30-step trajectory
    # test: the architecture then moves by gradient signal, so its genotype is decided by the search and
    # not by rounding noise (pure-noise batches left the alphas at ~7e-3 from init, where a near-tie
    # between two edges could flip on summation order alone)
    proto = torch.randn(10, 3, 1, 1, generator=g)
    data = []
    for _ in range(steps):
        ty, vy = torch.randint(0, 10, (B,), generator=g), torch.randint(0, 10, (B,), generator=g)
        tx = proto[ty] + 0.5 * torch.randn(B, 3, 32, 32, generator=g)
        vx = proto[vy] + 0.5 * torch.randn(B, 3, 32, 32, generator=g)
        data.append([t.to(dev) for t in (tx, ty, vx, vy)])
    settings = {"alpha_lr": 3e-2}
    dp = DartsSearch(layout, dev, comm, seed=3, capture=True, sync_bn=sync, settings=settings)
    sl = slice(r * B // W, (r + 1) * B // W)
    W1 = None
    verbose = os.environ.get("SYNCBN_VERBOSE") == "1"
    for i, (tx, ty, vx, vy) in enumerate(data):
        dp.step(tx[sl], ty[sl], vx[sl], vy[sl])
        if i == 0:
            W1 = dp.W.cpu()
        if verbose:
            torch.cuda.synchronize()
            print("rank %d step %d" % (r, i), file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if comm.xgmi is not None:
        comm.xgmi.check()
    res = {"W": dp.W.cpu(), "A": dp.A.cpu(), "bn": dp.bn.mean.cpu(), "geno": str(dp.genotype()),
           "loss": float(dp.loss_out), "capture": dp.capture, "allreduce": "xgmi" if comm.xgmi else comm.backend}
    comm.barrier()
    if r == 0:
        single = DartsSearch(layout, dev, Comm(device=dev), seed=3, capture=True, settings=settings)
        A0 = single.A.clone()
        dW1 = None
        for i, (tx, ty, vx, vy) in enumerate(data):
            single.step(tx, ty, vx, vy)
            if i == 0:
                dW1 = float((W1 - single.W.cpu()).abs().max())
        torch.cuda.synchronize()
        # run-to-run noise of the single-process search itself (float atomics: summation order
        # varies between runs; Adam turns near-zero alpha gradients' rounding into O(lr) steps)
        again = DartsSearch(layout, dev, Comm(device=dev), seed=3, capture=True, settings=settings)
        for tx, ty, vx, vy in data:
            again.step(tx, ty, vx, vy)
        torch.cuda.synchronize()
        out = {"geno_ss_equal": str(again.genotype()) == str(single.genotype()),
               "dA_ss": float((again.A - single.A).abs().max()), "dW_ss": float((again.W - single.W).abs().max()),
               "dW1": dW1, "dW": float((res["W"] - single.W.cpu()).abs().max()), "W_scale": float(single.W.abs().max()),
               "dA": float((res["A"] - single.A.cpu()).abs().max()),
               "A_disp": float((single.A - A0).abs().max()), "dBN": float((res["bn"] - single.bn.mean.cpu()).abs().max()),
               "geno_equal": res["geno"] == str(single.genotype()), "loss_dp": res["loss"],
               "loss_single": float(single.loss_out), "capture": res["capture"], "allreduce": res["allreduce"]}
        print("SYNCBN_RESULT " + json.dumps(out), flush=True)
    comm.barrier()
    comm.destroy()


if __name__ == "__main__":
    main()
