"""torchrun worker for tests/test_parallel.py (gloo on CPU; the same code runs over RCCL)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from katib_amd.models.darts import DartsLayout  # noqa: E402
from katib_amd.models.darts_search import DartsSearch  # noqa: E402
from katib_amd.parallel.comm import Comm  # noqa: E402


def main():
    torch.set_num_threads(1)
    comm = Comm.from_env("cpu")
    layout = DartsLayout(["separable_convolution_3x3", "max_pooling_3x3", "skip_connection"], init_channels=4,
                         num_layers=2, num_nodes=2, stem_multiplier=1)
    s = DartsSearch(layout, "cpu", comm, seed=5)
    g = torch.Generator().manual_seed(100 + comm.rank)  # each rank its own shard
    for _ in range(2):
        tx, vx = torch.randn(4, 3, 16, 16, generator=g), torch.randn(4, 3, 16, 16, generator=g)
        ty, vy = torch.randint(0, 10, (4,), generator=g), torch.randint(0, 10, (4,), generator=g)
        loss = float(s.step(tx, ty, vx, vy))
    ws = [torch.zeros_like(s.W) for _ in range(comm.world_size)]
    dist.all_gather(ws, s.W)
    al = [torch.zeros_like(s.A) for _ in range(comm.world_size)]
    dist.all_gather(al, s.A)
    mx = comm.allreduce_max(float(comm.rank))
    if comm.rank == 0:
        print(json.dumps({"dW": max(float((w - ws[0]).abs().max()) for w in ws),
                          "dA": max(float((a - al[0]).abs().max()) for a in al),
                          "loss": loss, "max_rank": mx}), flush=True)
    comm.barrier()
    comm.destroy()


if __name__ == "__main__":
    main()
