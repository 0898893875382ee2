"""HIP-graph hygiene on every captured workload: before EVERY replay the
graph's private memory pool - and, for DARTS, the step-scoped fp64 arena of the BN reductions
(``ops/hip_darts.py`` _Arena, zeroed inside the graph) - is filled with NaN
(``utils/graphcheck.py``), with eager work interleaved between replays. A graph that reads a
temporary before writing it (the round-2 ENAS failure: PyTorch cross-workgroup reductions reading
their staging memory) turns non-finite at once; a clean graph computes the same numbers as an
unpoisoned run. The gradient replica rows are persistent zero-invariant state, not temporaries:
the DARTS test checks instead that rows 1.. are zero after every step."""
import math
import re

import pytest
import torch

pytestmark = pytest.mark.gpu


def _poison_all(graphs, extra=()):
    from katib_amd.utils.graphcheck import POISON_WORD, poison_graph_pool

    n = 0
    for g in graphs:
        n += poison_graph_pool(g)
    for t in extra:
        t.view(torch.int32).fill_(POISON_WORD)
    torch.cuda.synchronize()
    return n


def _darts(seed=3):
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops

    dops.set_backend("hip")
    layout = DartsLayout(["separable_convolution_3x3", "dilated_convolution_3x3", "dilated_convolution_5x5",
                          "avg_pooling_3x3", "max_pooling_3x3", "skip_connection"], init_channels=4, num_layers=2,
                         num_nodes=3, stem_multiplier=1)
    return DartsSearch(layout, torch.device("cuda", 0), seed=seed, capture=True)


def test_darts_train_and_eval_graphs_with_poisoned_pools():
    from katib_amd.ops import hip_darts as hd

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    data = [(torch.randn(64, 3, 32, 32, device=dev, generator=g), torch.randint(0, 10, (64,), device=dev, generator=g),
             torch.randn(64, 3, 32, 32, device=dev, generator=g), torch.randint(0, 10, (64,), device=dev, generator=g))
            for _ in range(20)]
    clean, dirty = _darts(), _darts()
    ref_losses, ref_evals = [], []
    for tx, ty, vx, vy in data:
        ref_losses.append(float(clean.step(tx, ty, vx, vy)))
        ref_evals.append(float(clean.evaluate(vx, vy)[0]))
    losses, evals = [], []
    poisoned = 0
    for i, (tx, ty, vx, vy) in enumerate(data):
        if dirty.graphs is not None:
            arena = [hd._ARENA.buf] if hd._ARENA.buf is not None else []
            poisoned += _poison_all([gr for gr, _ in dirty.graphs], arena)
        losses.append(float(dirty.step(tx, ty, vx, vy)))
        assert float(dirty.gW_rep[1:].abs().max()) == 0.0 and float(dirty.gWv_rep[1:].abs().max()) == 0.0
        _ = torch.randn(1 << 20, device=dev).sum()  # eager work between replays (allocator churn)
        if dirty._eval_graphs:
            poisoned += _poison_all([e[0] for e in dirty._eval_graphs.values()])
        evals.append(float(dirty.evaluate(vx, vy)[0]))
    assert poisoned > 0
    assert all(math.isfinite(v) for v in losses + evals), (losses, evals)
    for a, b in zip(losses + evals, ref_losses + ref_evals):  # float-atomic summation order only
        assert abs(a - b) <= 2e-3 * max(1.0, abs(b)), (losses, ref_losses, evals, ref_evals)


def _poisoned_captured_step(monkeypatch):
    from katib_amd.utils.graphcheck import poison_graph_pool
    from katib_amd.workloads import common

    orig = common.CapturedStep.__call__
    count = {"n": 0}

    def poisoned(self):
        if self.graph is not None:
            poison_graph_pool(self.graph)
            count["n"] += 1
        return orig(self)
    monkeypatch.setattr(common.CapturedStep, "__call__", poisoned)
    return count


def test_mlp_captured_step_with_poisoned_pool(monkeypatch, capsys):
    from katib_amd.workloads import mnist_mlp

    count = _poisoned_captured_step(monkeypatch)
    acc = mnist_mlp.main(["--epochs", "2", "--num-train", "8192", "--num-valid", "2048", "--batch-size", "256"])
    out = capsys.readouterr().out
    losses = [float(m) for m in re.findall(r"loss=([^\s]+)", out)]
    assert count["n"] >= 20 and len(losses) == 2 and all(math.isfinite(v) for v in losses), out
    assert acc > 0.3


def test_gpt2_captured_step_with_poisoned_pool(monkeypatch, tmp_path):
    from katib_amd.workloads import gpt2_pbt
    from katib_amd.workloads.gpt2_pbt import GPTConfig

    count = _poisoned_captured_step(monkeypatch)
    gpt2_pbt.PRESETS["hygiene"] = GPTConfig(vocab=1000, ctx=128, n_layer=2, n_head=4, d=256)
    v = gpt2_pbt.main(["--model", "hygiene", "--batch-size", "8", "--lr", "3e-3", "--num-tokens", "200000",
                       "--p2p", "0", "--steps", "25", "--checkpoint-dir", str(tmp_path / "ck"), "--impl", "flat"])
    assert count["n"] >= 20
    assert math.isfinite(v) and v < math.log(1000) - 0.3, v
