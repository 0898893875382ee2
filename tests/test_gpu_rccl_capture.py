"""RCCL collectives inside a captured HIP graph: the fallback of the DARTS DP
step when the one-shot xGMI self-test fails keeps the step captured instead of running it
eagerly. One GPU allows only a one-rank RCCL communicator (RCCL refuses two ranks on one
device), which exercises the capture plumbing - ProcessGroupNCCL under torch.cuda.graph, grouped
all-reduces, a second communicator - but not cross-GPU traffic."""
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


def test_rccl_allreduce_captured_in_graph():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_capture_worker.py")], capture_output=True,
                       text=True, timeout=180, env=env)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0 and "RCCL_CAPTURE_OK" in out, out[-3000:]
