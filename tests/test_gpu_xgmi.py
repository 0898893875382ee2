"""One-shot xGMI all-reduce (HIP IPC + flag barrier kernel) between rank processes:
bit-exact sums in rank order, mean, unaligned/scalar path, capacity-sized messages,
HIP-graph capture and replay. Ranks share the box's GPU(s) via cross-process IPC."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allreduce_ranks(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "xgmi_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", XGMI_DARTS="1" if world == 2 else "0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0, out[-3000:]
    assert out.count("XGMI_OK") == world
