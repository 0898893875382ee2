"""Child process of tests/test_gpu_rccl_capture.py: a one-rank RCCL (`nccl`) process group on the
box's GPU. Checks that Comm.probe_rccl_capture() accepts graph capture, that a grouped
all-reduce (allreduce_sum_many_) and a mean all-reduce replay correctly from a captured HIP
graph, and that a subgroup communicator is usable inside a capture too."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from katib_amd.parallel.comm import Comm  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
c = Comm(0, 1, 0, "nccl", dev)
assert c.probe_rccl_capture(), "RCCL capture probe failed"
side = c.subgroup()
assert side.probe_rccl_capture()
a = torch.zeros(37, dtype=torch.float64, device=dev)
b = torch.zeros(5, dtype=torch.float64, device=dev)
m = torch.zeros(1000, device=dev)
c.world_size = side.world_size = 2  # make the Comm methods issue their collectives (1 real rank)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    a.add_(1.0)
    c.allreduce_sum_many_([a, b])
    side.allreduce_sum_(b)
    m.add_(2.0)
    dist.all_reduce(m, op=dist.ReduceOp.AVG)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
assert torch.equal(a, torch.full_like(a, 3.0)), a
assert torch.equal(m, torch.full_like(m, 6.0)), m
assert c.calls >= 1 and side.calls >= 1
dist.destroy_process_group()
print("RCCL_CAPTURE_OK", flush=True)
