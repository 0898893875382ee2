"""bench.py's driver contract, rehearsed on the CPU: one rank per process under
torch.distributed.run (gloo, world size 2), global batch 128 split over the ranks (strong
scaling keeps the B5 config at every N), ONE JSON line from rank 0 with the keys the driver
reads. The same code path runs over RCCL / the one-shot xGMI all-reduce on MI355X."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


BENCH_ARGS = ["--steps", "2", "--warmup", "1", "--trials", "0", "--b1", "0", "--experiment", "0", "--comparator-steps", "0", "--full-search", "0",
              "--valid-batches", "2"]


def _run(nproc, *extra, torchrun=True, gpus=None, rc=0):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(gpus or nproc)] + BENCH_ARGS + list(extra)
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + bench
    else:  # the plain `python bench.py --gpus N` form: bench.py launches its N ranks itself
        cmd = [sys.executable] + bench
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    if rc != 0:
        assert out.returncode != 0, out.stdout[-2000:]
        return out
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


def test_bench_two_ranks_strong_scaling():
    r = _run(2)
    assert KEYS <= set(r)
    assert r["metric"] == "darts_cifar10_search_wall_clock_s" and r["higher_is_better"] is False
    assert r["n_gpus"] == 2 and r["ranks_seen"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["scaling"] == "strong" and r["allreduce"] == "gloo" and r["batchnorm"] == "global batch (sync-bn)"
    c = r["config"]
    assert c["global_batch"] == 128 and c["per_gpu_batch"] == 64 and c["parallelism"] == "dp2"
    assert c["steps_per_epoch"] == 196 and c["second_order"] is True and c["allreduce"] == "gloo"
    # the projected search: epochs x steps/epoch x (step + validation batch)
    want = c["epochs"] * c["steps_per_epoch"] * (r["ms_per_step"] + r["ms_valid_batch"]) / 1000.0
    assert abs(r["value"] - want) <= 0.01 * want
    assert abs(r["vs_baseline"] - r["value"] / r["baseline_b5_s"]) < 1e-3
    assert r["final_loss"] == r["final_loss"]  # finite
    # DDP semantics (per-rank BN) timed next to the SyncBN headline, and the
    # physical devices behind the ranks (both ranks on this one host's CPU: 1)
    assert r["per_rank_bn_ms_per_step"] > 0 and r["per_rank_bn_search_wall_s"] > 0
    assert r["distinct_devices"] == 1
    # CPU: torch ops, sequential Hessian passes -> every rendezvous is on the critical path
    assert r["rendezvous_serial_per_step"] == r["rendezvous_per_step"] > 4


def test_bench_two_ranks_weak_scaling_label():
    r = _run(2, "--scaling", "weak")
    assert r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 256 and r["config"]["per_gpu_batch"] == 128
    assert r["config"]["steps_per_epoch"] == 98


def test_bench_self_launches_n_ranks():
    """plain `python bench.py --gpus 2` (no torchrun around it) runs 2 ranks and
    relays rank 0's single JSON line; n_gpus == ranks_seen == 2."""
    r = _run(2, torchrun=False)
    assert r["n_gpus"] == 2 and r["ranks_seen"] == 2 and r["config"]["parallelism"] == "dp2"
    assert r["config"]["per_gpu_batch"] == 64 and r["allreduce"] == "gloo"


def test_bench_refuses_world_size_mismatch():
    """Under torchrun, --gpus must equal WORLD_SIZE: a 2-rank launch told --gpus 4 exits non-zero
    instead of timing (and labelling) a different world size."""
    out = _run(2, torchrun=True, gpus=4, rc=1)
    assert "WORLD_SIZE=2 but --gpus 4" in out.stderr


def test_bench_per_rank_bn_label():
    r = _run(2, "--sync-bn", "0")
    assert r["batchnorm"] == "per rank" and r["config"]["sync_bn"] is False
    assert r["per_rank_bn_ms_per_step"] == r["ms_per_step"]


def test_bench_eight_ranks_syncbn_rehearsal():
    """the driver's N=8 case, rehearsed on the CPU - plain `python bench.py
    --gpus 8` (self-launched, gloo), strong scaling at per-rank batch 16 with SyncBN, one JSON
    line carrying the rendezvous keys. On MI355X the same code runs over RCCL / the one-shot
    xGMI kernel; here every rendezvous is a host-side gloo call (not in a graph)."""
    r = _run(8, torchrun=False)
    assert r["n_gpus"] == 8 and r["ranks_seen"] == 8 and r["config"]["parallelism"] == "dp8"
    assert r["config"]["per_gpu_batch"] == 16 and r["config"]["global_batch"] == 128
    assert r["batchnorm"] == "global batch (sync-bn)" and r["allreduce"] == "gloo"
    assert r["xgmi_self_test"] is None or r["xgmi_self_test"] != "passed"  # CPU: no one-shot path
    # 4 gradient buckets per step + the torch-op SyncBN all-reduces of every BN layer's statistics
    assert r["rendezvous_per_step"] > 4 and r["rendezvous_in_graph"] is False
    assert r["final_loss"] == r["final_loss"]
