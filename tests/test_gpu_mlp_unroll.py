"""MNIST-MLP trial (BASELINE configs 1-2, B1): U SGD steps per captured graph replay, batch indices
read on the device from the epoch permutation, must train exactly like one replay per step (same
batches in the same order) - the per-epoch metrics agree."""
import io
import re
from contextlib import redirect_stdout

import pytest

pytestmark = pytest.mark.gpu


def _run(unroll, optimizer):
    from katib_amd.workloads import mnist_mlp

    buf = io.StringIO()
    args = ["--num-train", "2000", "--num-valid", "500", "--batch-size", "64", "--epochs", "2", "--num-layers", "2",
            "--optimizer", optimizer, "--lr", "0.05", "--unroll", str(unroll)]
    with redirect_stdout(buf):
        acc = mnist_mlp.main(args)
    losses = [float(m) for m in re.findall(r"\bloss=([0-9.eE+-]+)", buf.getvalue())]
    return acc, losses


@pytest.mark.parametrize("optimizer", ["sgd", "adam"])
def test_unrolled_replays_match_per_step_replays(optimizer):
    acc1, l1 = _run(1, optimizer)
    acc16, l16 = _run(16, optimizer)  # 31 steps per epoch: one 16-step chunk + 15 single-step replays
    assert len(l1) == len(l16) == 2
    for a, b in zip(l1, l16):
        assert abs(a - b) <= 2e-3 * max(1.0, abs(a)), (l1, l16)
    assert abs(acc1 - acc16) <= 0.01, (acc1, acc16)
