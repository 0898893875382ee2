"""GPU-resident checkpoint hand-off between two processes (PBT exploit path)."""
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_p2p_checkpoint_between_processes(tmp_path):
    d = str(tmp_path / "member")
    w = os.path.join(HERE, "p2p_worker.py")
    prod = subprocess.Popen([sys.executable, w, "producer", d], stdout=subprocess.PIPE, text=True)
    try:
        line = prod.stdout.readline()
        assert "published" in line
        cons = subprocess.run([sys.executable, w, "consumer", d], capture_output=True, text=True, timeout=120)
        assert cons.returncode == 0, cons.stdout + cons.stderr
    finally:
        open(os.path.join(d, "done"), "a").close()
        prod.wait(timeout=60)


def test_p2p_fetch_missing_producer(tmp_path):
    import json

    from katib_amd.parallel import p2p_ckpt

    d = tmp_path / "m"
    d.mkdir()
    with open(d / p2p_ckpt.HANDLE_FILE, "w") as f:
        json.dump({"pid": 2 ** 22 + 12345, "host": "nohost", "handles": {}, "layout": [], "skeleton": {}}, f)
    assert p2p_ckpt.fetch(str(d)) is None
    (d / p2p_ckpt.HANDLE_FILE).write_bytes(b"\x80\x04not json")  # e.g. a pickle planted by trial code
    assert p2p_ckpt.fetch(str(d)) is None
