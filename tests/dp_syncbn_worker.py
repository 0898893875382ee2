"""torchrun worker for tests/test_parallel.py::test_darts_dp_syncbn_matches_single_process:
W ranks each take 1/W of a global batch with SyncBN; rank 0 also runs the single-process step
on the whole batch. gloo on CPU (the HIP kernels' fused SyncBN runs on MI355X)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from katib_amd.models.darts import DartsLayout  # noqa: E402
from katib_amd.models.darts_search import DartsSearch  # noqa: E402
from katib_amd.parallel.comm import Comm  # noqa: E402


def main():
    torch.set_num_threads(1)
    torch.manual_seed(0)
    comm = Comm.from_env("cpu")
    sync = os.environ.get("SYNC_BN", "1") == "1"
    layout = DartsLayout(["separable_convolution_3x3", "dilated_convolution_3x3", "avg_pooling_3x3",
                          "max_pooling_3x3", "skip_connection"], init_channels=4, num_layers=2, num_nodes=2,
                         stem_multiplier=1)
    dp = DartsSearch(layout, "cpu", comm, seed=5, sync_bn=sync)
    single = DartsSearch(layout, "cpu", Comm(), seed=5) if comm.rank == 0 else None
    g = torch.Generator().manual_seed(7)  # the same global batches on every rank
    B, W, r = 8, comm.world_size, comm.rank
    steps = int(os.environ.get("STEPS", "3"))
    for _ in range(steps):
        tx, vx = torch.randn(B, 3, 16, 16, generator=g), torch.randn(B, 3, 16, 16, generator=g)
        ty, vy = torch.randint(0, 10, (B,), generator=g), torch.randint(0, 10, (B,), generator=g)
        sl = slice(r * B // W, (r + 1) * B // W)
        dp.step(tx[sl], ty[sl], vx[sl], vy[sl])
        if single is not None:
            single.step(tx, ty, vx, vy)
    if comm.rank == 0:
        A0 = DartsSearch(layout, "cpu", Comm(), seed=5).A
        disp = float((single.A - A0).abs().max())
        print(json.dumps({"dW": float((dp.W - single.W).abs().max()), "W_scale": float(single.W.abs().max()),
                          "dA": float((dp.A - single.A).abs().max()), "A_disp": disp,
                          "dBN": float((dp.bn.mean - single.bn.mean).abs().max()),
                          "geno_equal": str(dp.genotype()) == str(single.genotype())}), flush=True)
    comm.barrier()
    comm.destroy()


if __name__ == "__main__":
    main()
