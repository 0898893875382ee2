"""torchrun worker for tests/test_parallel.py::test_darts_dp_global_validation (gloo, CPU):
the DARTS trial's validation pass over 2 rank shards gives the same global accuracy as one
process validating the whole split."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from katib_amd.models.darts import DartsLayout  # noqa: E402
from katib_amd.models.darts_search import DartsSearch  # noqa: E402
from katib_amd.parallel.comm import Comm  # noqa: E402
from katib_amd.workloads.darts_cifar10 import validate  # noqa: E402
from katib_amd.workloads.data import DeviceDataset  # noqa: E402


def main():
    torch.set_num_threads(1)
    comm = Comm.from_env("cpu")
    layout = DartsLayout(["separable_convolution_3x3", "max_pooling_3x3", "skip_connection"], init_channels=4,
                         num_layers=2, num_nodes=2, stem_multiplier=1)
    s = DartsSearch(layout, "cpu", comm, seed=5)
    # a few training steps on different shards so the BN running stats differ per rank
    g = torch.Generator().manual_seed(100 + comm.rank)
    for _ in range(2):
        tx, vx = torch.randn(4, 3, 16, 16, generator=g), torch.randn(4, 3, 16, 16, generator=g)
        ty, vy = torch.randint(0, 10, (4,), generator=g), torch.randint(0, 10, (4,), generator=g)
        s.step(tx, ty, vx, vy)
    ds = DeviceDataset(96, (3, 16, 16), 10, "cpu", seed=3)
    valid = ds.subset(32, 96)
    gbs = 16
    loss, top1 = validate(s, comm, valid.batches(gbs // comm.world_size, seed=7, shard=comm.rank,
                                                 num_shards=comm.world_size, drop_last=True))
    # the same split through ONE process (after the stats sync every rank holds the same model)
    single = Comm(device=torch.device("cpu"))
    s.comm = single
    loss1, top1_1 = validate(s, single, valid.batches(gbs, seed=7, drop_last=True))
    if comm.rank == 0:
        print(json.dumps({"top1": top1, "top1_single": top1_1, "loss": loss, "loss_single": loss1}), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
