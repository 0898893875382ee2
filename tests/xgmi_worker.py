"""Rank process for tests/test_gpu_xgmi.py: the one-shot xGMI all-reduce between
processes. On a one-GPU box every rank maps device 0 (cross-process HIP IPC, the
same code path as peers over xGMI; the 8 XCD L2s of one MI355X are not coherent
with each other either, so the release/acquire protocol is exercised)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from katib_amd.parallel.xgmi import XgmiAllReduce  # noqa: E402


def rank_data(seed, r, n):
    return torch.randn(n, generator=torch.Generator().manual_seed(seed * 131 + r))


def ref_sum(seed, world, n, scale=1.0):
    acc = rank_data(seed, 0, n)
    for r in range(1, world):
        acc = acc + rank_data(seed, r, n)  # rank order, like the kernel
    return acc * scale if scale != 1.0 else acc


def darts_dp(ar, rank, world, dev):
    """Data-parallel DARTS search step with the all-reduces inside the captured graph:
    replicas must stay bit-identical and match the eager (uncaptured) DP run."""
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops
    from katib_amd.parallel.comm import Comm

    dops.set_backend("hip")
    layout = DartsLayout(["separable_convolution_3x3", "dilated_convolution_3x3", "avg_pooling_3x3",
                          "max_pooling_3x3", "skip_connection"], init_channels=4, num_layers=2, num_nodes=3,
                         stem_multiplier=1)
    Ws = {}
    for capture in (False, True):
        comm = Comm(rank, world, rank, "gloo", dev)
        comm.xgmi = ar
        s = DartsSearch(layout, dev, comm, seed=5, capture=capture)
        gen = torch.Generator().manual_seed(100 + rank)  # each rank its own shard
        for _ in range(3):
            tx, vx = torch.randn(16, 3, 32, 32, generator=gen), torch.randn(16, 3, 32, 32, generator=gen)
            ty, vy = torch.randint(0, 10, (16,), generator=gen), torch.randint(0, 10, (16,), generator=gen)
            s.step(tx.to(dev), ty.to(dev), vx.to(dev), vy.to(dev))
        torch.cuda.synchronize()
        if capture:
            assert len(s.graphs) == 1, "the whole DP step should be one graph"
        W = s.W.cpu()
        allw = [torch.zeros_like(W) for _ in range(world)]
        dist.all_gather(allw, W)
        assert all(torch.equal(w, allw[0]) for w in allw), "replicas diverged (capture=%s)" % capture
        Ws[capture] = W
    d = float((Ws[True] - Ws[False]).abs().max())
    assert d < 1e-4, "captured DP step differs from eager: %g" % d
    assert ar.error() == 0


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", rank % ndev if os.environ.get("XGMI_SPREAD") == "1" else 0)
    torch.cuda.set_device(dev)
    ar = XgmiAllReduce(rank, world, dev, capacity=1 << 20, blocks=64, timeout_s=5.0)
    assert ar.ok, "self test failed"
    seed = 0
    for n in [1, 3, 4, 17, 1000, 65536 + 7, 1 << 20]:
        for average in (False, True):
            seed += 1
            x = rank_data(seed, rank, n).to(dev)
            ar.allreduce_(x, average=average)
            ref = ref_sum(seed, world, n, (1.0 / world) if average else 1.0)
            got = x.cpu()
            assert torch.equal(got, ref), (n, average, (got - ref).abs().max().item())
        # unaligned (scalar) path, out-of-place
        seed += 1
        buf = torch.zeros(n + 1, device=dev)
        buf[1:].copy_(rank_data(seed, rank, n).to(dev))
        out = torch.empty(n, device=dev)
        ar.allreduce(buf[1:], out)
        assert torch.equal(out.cpu(), ref_sum(seed, world, n)), ("unaligned", n)
    # graph capture: the epoch lives on the device, so replays keep working
    static = torch.zeros(4099, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.allreduce_(static)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ar.allreduce_(static)
    for k in range(5):
        seed += 1
        static.copy_(rank_data(seed, rank, 4099).to(dev))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(static.cpu(), ref_sum(seed, world, 4099)), ("graph replay", k)
    assert ar.error() == 0
    # latency (same-device IPC here: not an xGMI number, reported for reference)
    res = {}
    for n in (9406, 444922):
        t = torch.ones(n, device=dev)
        for _ in range(20):
            ar.allreduce_(t)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(200):
            ar.allreduce_(t)
        torch.cuda.synchronize()
        res[n] = (time.perf_counter() - t0) / 200 * 1e6
    assert ar.error() == 0
    if os.environ.get("XGMI_DARTS") == "1":
        darts_dp(ar, rank, world, dev)
    print("XGMI_OK rank=%d world=%d us_per_call=%s" % (rank, world, {k: round(v, 1) for k, v in res.items()}),
          flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
