"""Data-parallel DARTS search over torch.distributed (gloo on CPU, world size 2).

The same code path runs over RCCL (backend "nccl") on MI355X: flat-buffer all-reduces
of the four gradient vectors per step (darts_search.py). Checks: ranks stay
bit-identical in W/A after steps on different shards, and a 2-rank step on shards
equals the average-gradient semantics (weights move, loss finite).
"""
import json
import os
import socket
import subprocess
import sys

import torch

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_darts_dp_gloo_world2():
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dp_worker.py")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), worker],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["dW"] == 0.0 and res["dA"] == 0.0  # replicas stay identical
    assert res["loss"] == res["loss"] and res["max_rank"] == 1.0


def test_comm_single_process_noop():
    from katib_amd.parallel.comm import Comm

    c = Comm()
    t = torch.ones(3)
    assert c.allreduce_mean_(t) is t and float(t.sum()) == 3.0
    assert c.allreduce_max(2.5) == 2.5
    assert not c.distributed


def test_darts_dp_global_validation():
    """Validation accuracy of a 2-rank DARTS trial is sum(correct)/sum(n) over both shards,
    equal to a single process validating the same split."""
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dp_valid_worker.py")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), worker],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert abs(res["top1"] - res["top1_single"]) < 1e-9, res
    assert abs(res["loss"] - res["loss_single"]) < 1e-5 * max(1.0, abs(res["loss_single"])), res


def test_p2p_handle_file_is_json_roundtrip():
    """The P2P checkpoint handle file is data-only JSON (no pickle from a trial-writable
    directory): the nested skeleton - int-keyed optimizer state, tuples - round-trips."""
    import json as _json

    from katib_amd.parallel import p2p_ckpt as P

    st = {"model": {"w": torch.zeros(3)},
          "optim": {"state": {0: {"step": torch.tensor(5.0)}},
                    "param_groups": [{"lr": 0.1, "betas": (0.9, 0.99), "params": [0]}]}, "step": 42}
    ts = []
    sk = _json.loads(_json.dumps(P._flatten(st, ts)))
    out = P._unflatten(sk, ts)
    assert out["optim"]["state"][0]["step"] is ts[1]
    assert out["optim"]["param_groups"][0]["betas"] == (0.9, 0.99) and out["step"] == 42
    import pytest

    with pytest.raises(KeyError):  # classes / dtypes only through the whitelists
        P._decode_handle([[3], [1], 0, "os.system", "torch.float32", 0, "00", 12, 0, False, None, 0, None, False])


def _run_syncbn(sync: bool, nproc: int = 2):
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", SYNC_BN="1" if sync else "0")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dp_syncbn_worker.py")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % nproc,
                          "--master-addr", "127.0.0.1", "--master-port", str(port), worker],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])


def test_darts_dp_syncbn_matches_single_process():
    """with SyncBN a 2-rank strong-scaling step (half the batch per rank) IS the
    single-process step on the whole batch - weights, alphas and BN running statistics agree to
    float rounding; per-rank BN (the old behaviour) visibly diverges."""
    res = _run_syncbn(True)
    assert res["dW"] <= 1e-5 * max(1.0, res["W_scale"]), res
    assert res["dA"] <= 0.01 * res["A_disp"], res
    assert res["dBN"] <= 1e-5, res
    assert res["geno_equal"], res
    per_rank = _run_syncbn(False)
    assert per_rank["dA"] > 10 * max(res["dA"], 1e-12), (per_rank, res)


def test_syncbn_rejects_fold_modes_without_cross_rank_sum(monkeypatch):
    """under SyncBN ``_bn`` divides by count * world, which is only right when the fold
    launch summed the BN reductions over the ranks. FOLD=0 and self-folding producers skip that
    fold, so SyncBN and sync_scope refuse them instead of normalising with local sums / world."""
    import pytest

    from katib_amd.ops import hip_darts as h

    class FakeComm:
        world_size, xgmi = 2, None

        def allreduce_sum_(self, t):
            pass

        def probe_rccl_capture(self):
            return False

    sync = h.SyncBN(FakeComm())  # default modes: accepted
    monkeypatch.setattr(h, "FOLD", False)
    with pytest.raises(RuntimeError, match="hip_darts.FOLD"):
        h.SyncBN(FakeComm())
    with pytest.raises(RuntimeError, match="hip_darts.FOLD"):
        with h.sync_scope(sync):
            pass
    monkeypatch.setattr(h, "FOLD", True)
    monkeypatch.setattr(h, "SELFFOLD", True)
    with pytest.raises(RuntimeError, match="SELFFOLD"):
        with h.sync_scope(sync):
            pass
    monkeypatch.setattr(h, "SELFFOLD", False)
    with h.sync_scope(sync):
        with pytest.raises(RuntimeError, match="SyncBN"):
            h.set_selffold(True)
    with h.sync_scope(None):  # per-rank BN: any fold mode
        pass
