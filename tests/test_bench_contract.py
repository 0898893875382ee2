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


def _run(nproc, *extra):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--trials", "0", "--comparator-steps", "0",
           "--full-search", "0", "--valid-batches", "2", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # rank 0 only
    return json.loads(lines[0])


def test_bench_two_ranks_strong_scaling():
    r = _run(2)
    assert KEYS <= set(r)
    assert r["metric"] == "darts_cifar10_search_wall_clock_s" and r["higher_is_better"] is False
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1 and r["scaling"] == "strong"
    c = r["config"]
    assert c["global_batch"] == 128 and c["per_gpu_batch"] == 64 and c["parallelism"] == "dp2"
    assert c["steps_per_epoch"] == 196 and c["second_order"] is True and c["allreduce"] == "gloo"
    # the projected search: epochs x steps/epoch x (step + validation batch)
    want = c["epochs"] * c["steps_per_epoch"] * (r["ms_per_step"] + r["ms_valid_batch"]) / 1000.0
    assert abs(r["value"] - want) <= 0.01 * want
    assert abs(r["vs_baseline"] - r["value"] / r["baseline_b5_s"]) < 1e-3
    assert r["final_loss"] == r["final_loss"]  # finite


def test_bench_two_ranks_weak_scaling_label():
    r = _run(2, "--scaling", "weak")
    assert r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 256 and r["config"]["per_gpu_batch"] == 128
    assert r["config"]["steps_per_epoch"] == 98
