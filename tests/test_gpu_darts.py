"""HIP DARTS kernels vs the PyTorch fp32 oracle (same functional network, torch backend).

Checks one MixedOp edge (forward, d input, d softmax-weights, d every weight, running
BN statistics) for normal and reduction edges at several widths, the preprocess
layers, eval mode, and a full second-order search step (eager and HIP-graph).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ALL = ["max_pooling_3x3", "avg_pooling_3x3", "skip_connection", "separable_convolution_3x3",
       "separable_convolution_5x5", "dilated_convolution_3x3", "dilated_convolution_5x5"]


def _setup(C, prims=ALL, L=2, N=2):
    from katib_amd.models.darts import BNState, DartsLayout

    layout = DartsLayout(prims, init_channels=C, num_layers=L, num_nodes=N, stem_multiplier=1)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    W = torch.zeros(layout.n_weights)
    layout.init_weights(W, g)
    return layout, W.to(dev), dev, BNState


def _run_edge(backend, layout, W, dev, BNState, edge, x, w, R, training=True):
    from katib_amd.models.darts import DartsNetwork
    from katib_amd.ops import darts as dops

    dops.set_backend(backend)
    try:
        net = DartsNetwork(layout)
        Wl = W.clone()
        gW = torch.zeros_like(Wl)
        P = layout.views(Wl)
        G = layout.views(gW)
        for k, v in P.items():
            v.requires_grad_(True)
            v.grad = G[k]
        bn = BNState(layout, dev)
        bn.mean.normal_(generator=torch.Generator(device=dev).manual_seed(3))
        bn.var.uniform_(0.5, 2.0, generator=torch.Generator(device=dev).manual_seed(4))
        xl = x.clone().requires_grad_(True)
        wl = w.clone().requires_grad_(True)
        out = net.mixed_op(xl, edge, P, wl, bn, training)
        loss = (out * R).sum()
        loss.backward(inputs=[xl, wl] + list(P.values()))
        torch.cuda.synchronize()
        return out.detach(), xl.grad, wl.grad, gW, bn.mean.clone(), bn.var.clone()
    finally:
        dops.set_backend("torch")


def _close(a, b, name, rtol=2e-4, atol=2e-4):
    scale = b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * scale, "%s: max err %.3e (scale %.3e)" % (name, err, scale)


@pytest.mark.parametrize("C,cell_idx,edge_idx", [(4, 0, 0), (4, 1, 0), (4, 1, 4), (16, 0, 1), (16, 1, 1),
                                                 (32, 0, 0), (8, 1, 4), (8, 1, 2)])
def test_mixed_edge_matches_torch(C, cell_idx, edge_idx):
    layout, W, dev, BNState = _setup(C)
    cell = layout.cells[cell_idx]
    edge = cell["edges"][edge_idx]
    Cc = cell["C"]
    H = 16 if (cell["reduction"] and edge["stride"] == 1) else 32
    gen = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(8, Cc, H, H, device=dev, generator=gen)
    w = torch.softmax(torch.randn(len(layout.prims), device=dev, generator=gen), 0)
    Ho = (x.shape[2] - 1) // edge["stride"] + 1
    R = torch.randn(8, Cc, Ho, Ho, device=dev, generator=gen)
    ref = _run_edge("torch", layout, W, dev, BNState, edge, x, w, R)
    got = _run_edge("hip", layout, W, dev, BNState, edge, x, w, R)
    for name, a, b in zip(["out", "dx", "dw_softmax", "dW", "running_mean", "running_var"], got, ref):
        _close(a, b, name, rtol=1e-3, atol=1e-4)


def test_mixed_edge_eval_mode():
    layout, W, dev, BNState = _setup(16)
    edge = layout.cells[0]["edges"][0]
    gen = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(4, 16, 32, 32, device=dev, generator=gen)
    w = torch.softmax(torch.randn(len(layout.prims), device=dev, generator=gen), 0)
    R = torch.randn(4, 16, 32, 32, device=dev, generator=gen)
    ref = _run_edge("torch", layout, W, dev, BNState, edge, x, w, R, training=False)
    got = _run_edge("hip", layout, W, dev, BNState, edge, x, w, R, training=False)
    for name, a, b in zip(["out", "dx", "dw_softmax", "dW"], got[:4], ref[:4]):
        _close(a, b, name, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("reduce", [False, True])
def test_preprocess_matches_torch(reduce):
    from katib_amd.models.darts import DartsNetwork
    from katib_amd.ops import darts as dops

    layout, W, dev, BNState = _setup(16)
    ci = 1 if not reduce else None
    # cells.1 follows no reduction; with L=2 cell 1 is the reduction cell, so build L=3 for reduce_prev
    if reduce:
        layout, W, dev, BNState = _setup(16, L=3)
        ci = 2
    cell = layout.cells[ci]
    name = "cells.%d.pre0" % ci
    Cin = cell["cpp"]
    H = 32 if reduce else 16
    gen = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(8, Cin, H, H, device=dev, generator=gen)
    results = []
    for backend in ("torch", "hip"):
        dops.set_backend(backend)
        net = DartsNetwork(layout)
        Wl = W.clone()
        gW = torch.zeros_like(Wl)
        P, G = layout.views(Wl), layout.views(gW)
        for k, v in P.items():
            v.requires_grad_(True)
            v.grad = G[k]
        bn = BNState(layout, dev)
        xl = x.clone().requires_grad_(True)
        out = net.preprocess(xl, name, cell["reduction_prev"], P, bn, True)
        R = torch.randn(out.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
        (out * R).sum().backward(inputs=[xl] + list(P.values()))
        results.append((out.detach(), xl.grad, gW, bn.mean.clone(), bn.var.clone()))
    dops.set_backend("torch")
    for name_, a, b in zip(["out", "dx", "dW", "rm", "rv"], results[1], results[0]):
        _close(a, b, name_, rtol=1e-3, atol=1e-4)


def test_wide_preprocess_128_to_64_matches_torch():
    """darts-gpu.yaml's last reduction cell: StdConv 128 -> 64 at 16x16 (pw_fwd_wave / pw_bwd_wave
    <128, 64> instantiations)."""
    from katib_amd.models.darts import DartsNetwork
    from katib_amd.ops import darts as dops

    layout, W, dev, BNState = _setup(16, L=3, N=4)
    cell = layout.cells[2]
    assert cell["cp"] == 128 and cell["C"] == 64
    gen = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(16, 128, 16, 16, device=dev, generator=gen)
    results = []
    for backend in ("torch", "hip"):
        dops.set_backend(backend)
        net = DartsNetwork(layout)
        Wl = W.clone()
        gW = torch.zeros_like(Wl)
        P, G = layout.views(Wl), layout.views(gW)
        for k, v in P.items():
            v.requires_grad_(True)
            v.grad = G[k]
        bn = BNState(layout, dev)
        xl = x.clone().requires_grad_(True)
        out = net.preprocess(xl, "cells.2.pre1", False, P, bn, True)
        R = torch.randn(out.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(8))
        (out * R).sum().backward(inputs=[xl] + list(P.values()))
        results.append((out.detach(), xl.grad, gW, bn.mean.clone(), bn.var.clone()))
    dops.set_backend("torch")
    for name_, a, b in zip(["out", "dx", "dW", "rm", "rv"], results[1], results[0]):
        _close(a, b, name_, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("capture", [False, True])
def test_search_step_matches_torch(capture):
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops

    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(11)
    tx = torch.randn(16, 3, 32, 32, device=dev, generator=gen)
    vx = torch.randn(16, 3, 32, 32, device=dev, generator=gen)
    ty = torch.randint(0, 10, (16,), device=dev, generator=gen)
    vy = torch.randint(0, 10, (16,), device=dev, generator=gen)
    res = {}
    for backend in ("torch", "hip"):
        dops.set_backend(backend)
        s = DartsSearch(layout, dev, capture=capture and backend == "hip")
        losses = [float(s.step(tx, ty, vx, vy)) for _ in range(2)]
        torch.cuda.synchronize()
        res[backend] = (losses, s.W.clone(), s.A.clone())
    dops.set_backend("torch")
    (lt, Wt, At), (lh, Wh, Ah) = res["torch"], res["hip"]
    assert abs(lt[0] - lh[0]) < 1e-4 * max(1.0, abs(lt[0]))
    assert abs(lt[1] - lh[1]) < 1e-3 * max(1.0, abs(lt[1]))
    _close(Wh, Wt, "W", rtol=1e-3, atol=1e-4)
    _close(Ah, At, "alpha", rtol=5e-2, atol=5e-5)


def test_search_trajectory_30_steps_matches_torch():
    """30 second-order search steps, HIP kernels in the captured graph vs the eager PyTorch oracle,
    on a learnable synthetic task (class-dependent channel means) with a larger alpha lr so the
    architecture moves by gradient signal rather than by init noise: same genotype, alpha
    trajectory within 5 % of its own displacement, weights within 1 %."""
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops

    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(21)
    proto = torch.randn(10, 3, 1, 1, device=dev, generator=gen)
    batches = []
    for _ in range(4):
        ty = torch.randint(0, 10, (32,), device=dev, generator=gen)
        vy = torch.randint(0, 10, (32,), device=dev, generator=gen)
        tx = proto[ty] + 0.5 * torch.randn(32, 3, 32, 32, device=dev, generator=gen)
        vx = proto[vy] + 0.5 * torch.randn(32, 3, 32, 32, device=dev, generator=gen)
        batches.append((tx, ty, vx, vy))
    res = {}
    for backend in ("torch", "hip"):
        dops.set_backend(backend)
        s = DartsSearch(layout, dev, capture=backend == "hip", settings={"alpha_lr": 3e-2})
        A0 = s.A.clone()
        losses = []
        for i in range(30):
            losses.append(float(s.step(*batches[i % 4])))
        torch.cuda.synchronize()
        res[backend] = (losses, s.W.clone(), s.A.clone(), A0, s.genotype())
    dops.set_backend("torch")
    (lt, Wt, At, A0, gt), (lh, Wh, Ah, _, gh) = res["torch"], res["hip"]
    assert str(gh) == str(gt), "genotype differs:\n hip   %s\n torch %s" % (gh, gt)
    moved = (At - A0).abs().max().item()
    assert moved > 1e-2, "alphas barely moved (%.3e): the test would not discriminate" % moved
    drift = (Ah - At).abs().max().item()
    assert drift <= 0.05 * moved, "alpha drift %.3e vs displacement %.3e" % (drift, moved)
    _close(Wh, Wt, "W", rtol=1e-2, atol=1e-3)
    assert max(abs(a - b) for a, b in zip(lt, lh)) < 1e-2


@pytest.mark.parametrize("N,C,H,K,registered", [(128, 48, 8, 10, False), (128, 256, 8, 10, True),
                                                 (7, 33, 5, 3, False), (64, 1024, 2, 64, True)])
def test_fused_head_matches_torch(N, C, H, K, registered):
    """hip_darts.head_loss (gap + linear + cross-entropy, fused forward/backward) against the
    fp32 PyTorch formula; weight grads through a registered replicated buffer and through the
    temporary-replica fallback."""
    from katib_amd.ops import hip_darts as hd

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(N + C)
    x = torch.randn(N, C, H, H, device=dev, generator=gen)
    y = torch.randint(0, K, (N,), device=dev, generator=gen)
    w0 = 0.1 * torch.randn(K, C, device=dev, generator=gen)
    b0 = 0.1 * torch.randn(K, device=dev, generator=gen)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w0, b0))
    logits_r = torch.nn.functional.linear(xr.mean((2, 3)), wr, br)
    loss_r = torch.nn.functional.cross_entropy(logits_r, y)
    (3.0 * loss_r).backward()
    if registered:
        rep = torch.zeros(hd.REP, K * C + K, device=dev)
        hd.register_grad_replicas(rep)
        w = rep.new_zeros(K * C + K)[:K * C].view(K, C).copy_(w0).requires_grad_(True)
        b = torch.empty(K, device=dev).copy_(b0).requires_grad_(True)
        w.grad = rep[0, :K * C].view(K, C)
        b.grad = rep[0, K * C:]
    else:
        w, b = w0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    xh = x.clone().requires_grad_(True)
    loss, logits = hd.head_loss(xh, w, b, y)
    assert not logits.requires_grad
    (3.0 * loss).backward()
    _close(logits, logits_r.detach(), "logits", rtol=1e-5, atol=1e-5)
    assert abs(float(loss) - float(loss_r)) < 1e-5 * max(1.0, abs(float(loss_r)))
    _close(xh.grad, xr.grad, "dx", rtol=1e-4, atol=1e-7)
    if registered:
        hd.fold(rep)
        gw, gb = rep[0, :K * C].view(K, C), rep[0, K * C:]
    else:
        gw, gb = w.grad, b.grad
    _close(gw, wr.grad, "dW", rtol=1e-4, atol=1e-6)
    _close(gb, br.grad, "db", rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("N,Cout,H", [(128, 4, 32), (128, 48, 32), (5, 7, 9)])
def test_stem_conv_bn_matches_torch(N, Cout, H):
    """hip_darts.stem_conv_bn (conv + BN statistics epilogue, combine BN apply, fused BN backward
    in the weight-gradient kernel) and stem_bn_eval against conv2d + batch_norm in fp32."""
    from katib_amd.ops import hip_darts as hd

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(N * Cout + H)
    x = torch.randn(N, 3, H, H, device=dev, generator=gen)
    w0 = 0.3 * torch.randn(Cout, 3, 3, 3, device=dev, generator=gen)
    g0 = 1.0 + 0.1 * torch.randn(Cout, device=dev, generator=gen)
    b0 = 0.1 * torch.randn(Cout, device=dev, generator=gen)
    R = torch.randn(N, Cout, H, H, device=dev, generator=gen)
    rm_r, rv_r = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    wr, gr, br = (t.clone().requires_grad_(True) for t in (w0, g0, b0))
    out_r = F.batch_norm(F.conv2d(x, wr, padding=1), rm_r, rv_r, gr, br, True, 0.1, 1e-5)
    (out_r * R).sum().backward()
    rm, rv = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    w, g, b = (t.clone().requires_grad_(True) for t in (w0, g0, b0))
    out = hd.stem_conv_bn(x, w, g, b, rm, rv, 0.1, 1e-5)
    (out * R).sum().backward()
    _close(out, out_r.detach(), "out", rtol=1e-4, atol=1e-5)
    _close(rm, rm_r, "running_mean", rtol=1e-5, atol=1e-6)
    _close(rv, rv_r, "running_var", rtol=1e-5, atol=1e-6)
    _close(w.grad, wr.grad, "dW", rtol=1e-3, atol=1e-4)
    _close(g.grad, gr.grad, "dgamma", rtol=1e-4, atol=1e-4)
    _close(b.grad, br.grad, "dbeta", rtol=1e-4, atol=1e-4)
    with torch.no_grad():
        ev = hd.stem_bn_eval(hd.stem_conv(x, w0), g0, b0, rm, rv, 1e-5)
        ev_r = F.batch_norm(F.conv2d(x, w0, padding=1), rm, rv, g0, b0, False, 0.1, 1e-5)
    _close(ev, ev_r, "eval", rtol=1e-4, atol=1e-5)


def test_evaluate_graph_matches_eager():
    """The HIP-graph validation forward (DartsSearch.evaluate with capture) equals the eager
    HIP forward and the torch-oracle forward on the same weights, across batch shapes and
    after the weights change between replays."""
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops

    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(5)
    tx = torch.randn(16, 3, 32, 32, device=dev, generator=gen)
    ty = torch.randint(0, 10, (16,), device=dev, generator=gen)
    dops.set_backend("hip")
    s = DartsSearch(layout, dev, capture=True)
    s.step(tx, ty, tx, ty)  # non-trivial running BN statistics
    for n in (16, 32, 16):
        vx = torch.randn(n, 3, 32, 32, device=dev, generator=gen)
        vy = torch.randint(0, 10, (n,), device=dev, generator=gen)
        got = [float(t) for t in s.evaluate(vx, vy)]
        want = [float(t) for t in s._evaluate(vx, vy)]
        dops.set_backend("torch")
        oracle = [float(t) for t in s._evaluate(vx, vy)]
        dops.set_backend("hip")
        assert abs(got[0] - want[0]) < 1e-5 * max(1.0, abs(want[0])) and got[1:] == want[1:]
        assert abs(got[0] - oracle[0]) < 1e-3 * max(1.0, abs(oracle[0]))
        s.step(tx, ty, tx, ty)  # weights move; the captured graph must read the live buffers
    assert len(s._eval_graphs) == 2
    dops.set_backend("torch")


def test_grouped_validation_matches_per_batch():
    """Validation batches merged per captured eval forward (models/darts_search.py eval_groups,
    used by the workload and bench.py) give the per-batch losses and correct counts: eval-mode BN
    normalises every sample with the running statistics."""
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch, eval_groups
    from katib_amd.ops import darts as dops

    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(9)
    tx = torch.randn(32, 3, 32, 32, device=dev, generator=gen)
    ty = torch.randint(0, 10, (32,), device=dev, generator=gen)
    dops.set_backend("hip")
    s = DartsSearch(layout, dev, capture=True)
    s.step(tx, ty, tx, ty)
    batches = [(torch.randn(32, 3, 32, 32, device=dev, generator=gen), torch.randint(0, 10, (32,), device=dev, generator=gen))
               for _ in range(6)]
    per = torch.zeros(2, dtype=torch.float64)
    for vx, vy in batches:
        loss, top1, _ = s.evaluate(vx, vy)
        per += torch.tensor([float(loss), float(top1)], dtype=torch.float64) * vy.numel()
    grouped = torch.zeros(2, dtype=torch.float64)
    shapes = []
    for vx, vy in eval_groups(batches, 4):  # groups of 4 and 2
        shapes.append(vx.shape[0])
        loss, top1, _ = s.evaluate(vx, vy)
        grouped += torch.tensor([float(loss), float(top1)], dtype=torch.float64) * vy.numel()
    assert shapes == [128, 64]
    assert abs(grouped[1] - per[1]) < 0.5  # correct counts (integers up to rounding of the fractions)
    assert abs(grouped[0] - per[0]) < 1e-4 * abs(per[0])
    dops.set_backend("torch")


@pytest.mark.parametrize("C,cell_idx,node,joint", [(4, 0, 1, False), (8, 1, 1, False), (16, 0, 2, False), (8, 1, 2, False),
                                                  (4, 0, 2, True), (8, 1, 2, True)])
def test_mixed_node_matches_torch(C, cell_idx, node, joint, monkeypatch):
    """All edges of a node in one edge-batched Function (mixed strides in reduction cells);
    ``joint``: the opt-in launch of the pools beside the stage-1 dw-pw bands (KATIB_HIP_JOINT_POOL)."""
    from katib_amd.models.darts import DartsNetwork
    from katib_amd.ops import darts as dops
    from katib_amd.ops import hip_darts

    monkeypatch.setattr(hip_darts, "JOINT_POOL", joint)

    layout, W, dev, BNState = _setup(C, N=3)
    cell = layout.cells[cell_idx]
    edges = [e for e in cell["edges"] if e["node"] == node]
    Cc = cell["C"]
    gen = torch.Generator(device=dev).manual_seed(9)
    H = 32
    states = []
    for j in range(2 + node):
        h = H if (j < 2 or not cell["reduction"]) else H // 2
        states.append(torch.randn(8, Cc, h, h, device=dev, generator=gen))
    w = torch.softmax(torch.randn(2 + node, len(layout.prims), device=dev, generator=gen), -1)
    Ho = H // 2 if cell["reduction"] else H
    R = torch.randn(8, Cc, Ho, Ho, device=dev, generator=gen)
    res = []
    for backend in ("torch", "hip"):
        dops.set_backend(backend)
        net = DartsNetwork(layout)
        Wl = W.clone()
        gW = torch.zeros_like(Wl)
        P, G = layout.views(Wl), layout.views(gW)
        for k, v in P.items():
            v.requires_grad_(True)
            v.grad = G[k]
        bn = BNState(layout, dev)
        xs = [s.clone().requires_grad_(True) for s in states]
        wl = w.clone().requires_grad_(True)
        out = net.mixed_node(xs, edges, P, wl, bn, True)
        (out * R).sum().backward(inputs=xs + [wl] + list(P.values()))
        torch.cuda.synchronize()
        res.append((out.detach(), [x.grad for x in xs], wl.grad, gW, bn.mean.clone(), bn.var.clone()))
    dops.set_backend("torch")
    (o_t, gx_t, gw_t, gW_t, m_t, v_t), (o_h, gx_h, gw_h, gW_h, m_h, v_h) = res
    _close(o_h, o_t, "out", rtol=1e-3, atol=1e-4)
    for i, (a, b) in enumerate(zip(gx_h, gx_t)):
        _close(a, b, "dx[%d]" % i, rtol=1e-3, atol=1e-4)
    _close(gw_h, gw_t, "dalpha", rtol=1e-3, atol=1e-4)
    _close(gW_h, gW_t, "dW", rtol=1e-3, atol=1e-4)
    _close(m_h, m_t, "running_mean", rtol=1e-3, atol=1e-5)
    _close(v_h, v_t, "running_var", rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("N,Cin,Cout,H", [(128, 3, 4, 32), (128, 3, 48, 32), (5, 3, 64, 7), (3, 1, 20, 28)])
def test_stem_conv_vs_torch(N, Cin, Cout, H):
    """Direct stem conv kernels (forward + weight gradient) vs F.conv2d in fp32."""
    import torch.nn.functional as F

    from katib_amd.ops import hip_darts as hd

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, Cin, H, H, generator=g).to(dev)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * 0.3).to(dev)
    dy = torch.randn(N, Cout, H, H, generator=g).to(dev)
    assert hd.stem_supported(x, w)
    w1 = w.clone().requires_grad_(True)
    y = hd.stem_conv(x, w1)
    y.backward(dy)
    w2 = w.clone().requires_grad_(True)
    yr = F.conv2d(x, w2, padding=1)
    yr.backward(dy)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w1.grad, w2.grad, rtol=1e-4, atol=1e-3 * (N * H * H) ** 0.5)
    # the input-gradient fallback path
    x1 = x.clone().requires_grad_(True)
    hd.stem_conv(x1, w).backward(dy)
    x2 = x.clone().requires_grad_(True)
    F.conv2d(x2, w, padding=1).backward(dy)
    torch.testing.assert_close(x1.grad, x2.grad, rtol=1e-4, atol=1e-4)


def _combine_case(nedge, nops, training, accumulate, offset, mean_shift):
    """Run combine_fwd on nedge edges x nops BN inputs (+ identity) with the operands placed at
    ``offset`` floats into their buffers (offset 1 defeats 16-byte alignment -> scalar path).
    Returns the kernel output, the updated running stats and an fp64 reference."""
    from katib_amd.ops import hip_darts as hd

    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    N, C, H, W = 4, 8, 16, 16
    n = N * C * H * W
    out0 = torch.randn(N, C, H, W, generator=g).to(dev)
    w = torch.softmax(torch.randn(nedge * (nops + 1), generator=g), 0).to(dev)
    calls, ref = [], out0.double().clone() if accumulate else torch.zeros(N, C, H, W, dtype=torch.float64, device=dev)
    rms, rvs, exp_rm, exp_rv = [], [], [], []
    mom = 0.1
    for e in range(nedge):
        zs, bns, widx = [], [], []
        for k in range(nops):
            base = torch.zeros(n + 4, device=dev)  # same values at either alignment
            base[offset:offset + n] = (torch.randn(n, generator=g) * 0.5 + mean_shift).to(dev)
            z = base[offset:offset + n].view(N, C, H, W)
            rm = (torch.randn(C, generator=g) * 0.1).to(dev)
            rv = (torch.rand(C, generator=g) + 0.5).to(dev)
            zd = z.double()
            if training:
                s1 = zd.sum((0, 2, 3))
                s2 = (zd * zd).sum((0, 2, 3))
                stats = torch.zeros(32 * 2 * C, dtype=torch.float64, device=dev)
                stats[:C], stats[C:2 * C] = s1, s2
                mean = s1 / (N * H * W)
                var = (s2 / (N * H * W) - mean * mean).clamp_min(0)
                cnt = N * H * W
                exp_rm.append((1 - mom) * rm.double() + mom * mean)
                exp_rv.append((1 - mom) * rv.double() + mom * var * cnt / (cnt - 1))
            else:
                stats, mean, var = None, rm.double(), rv.double()
                exp_rm.append(rm.double())
                exp_rv.append(rv.double())
            rms.append(rm)
            rvs.append(rv)
            bns.append(hd._bn(stats, rm, rv, N * H * W, training, 1e-5, C))
            zs.append(z)
            widx.append(e * (nops + 1) + k)
            ref += w[e * (nops + 1) + k].double() * (zd - mean[None, :, None, None]) / torch.sqrt(
                var[None, :, None, None] + 1e-5)
        xb = torch.zeros(n + 4, device=dev)
        xb[offset:offset + n] = torch.randn(n, generator=g).to(dev)
        x = xb[offset:offset + n].view(N, C, H, W)
        id_idx = e * (nops + 1) + nops
        ref += w[id_idx].double() * x.double()
        calls.append((zs, bns, widx, w, id_idx, x, []))
    out = out0.clone()
    hd._K.combine_fwd(calls, None, None, out, mom, training, accumulate)
    torch.cuda.synchronize()
    return out, rms, rvs, ref, exp_rm, exp_rv


@pytest.mark.parametrize("nedge,nops,training,accumulate,mean_shift",
                         [(1, 1, False, False, 0.0), (3, 3, True, True, 0.0), (2, 3, True, False, 0.0),
                          (3, 1, False, True, 0.0), (2, 2, True, True, 200.0)])
def test_combine_fwd_vector_and_scalar_paths(nedge, nops, training, accumulate, mean_shift):
    """combine_fwd takes the 16-byte vector path for aligned operands and the scalar path
    otherwise (offset 1 shifts every BN input and identity by one float). Both compute
    w * ((z - mean) * invstd), so they agree with each other to the last ulps and with the
    fp64 formula sum_e [sum_k w_ek BN(z_ek) + w_e,id x_e] (+ out when accumulating), over
    several edges, several BN inputs, training-mode statistics with running-stat updates,
    and a mean 400x the standard deviation."""
    res = [_combine_case(nedge, nops, training, accumulate, off, mean_shift) for off in (0, 1)]
    for out, rms, rvs, ref, exp_rm, exp_rv in res:
        torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4 if mean_shift else 2e-5)
        for a, b in zip(rms + rvs, exp_rm + exp_rv):
            torch.testing.assert_close(a.double(), b, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("selffold,edge", [(True, False), (False, True), (True, True)])
def test_selffold_and_edge_bwd_paths_match_torch(selffold, edge):
    """The A/B paths that are off by default (self-folding producers, fused per-edge input
    gradient) stay numerically equal to the PyTorch oracle on every node of a B5-shaped cell pair:
    3 captured search steps vs the eager torch step."""
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops
    from katib_amd.ops import hip_darts

    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(13)
    tx = torch.randn(16, 3, 32, 32, device=dev, generator=gen)
    vx = torch.randn(16, 3, 32, 32, device=dev, generator=gen)
    ty = torch.randint(0, 10, (16,), device=dev, generator=gen)
    vy = torch.randint(0, 10, (16,), device=dev, generator=gen)
    res = {}
    old_edge = hip_darts.EDGE_BWD
    try:
        for backend in ("torch", "hip"):
            dops.set_backend(backend)
            if backend == "hip":
                hip_darts.set_selffold(selffold)
                hip_darts.EDGE_BWD = edge
            s = DartsSearch(layout, dev, capture=backend == "hip")
            losses = [float(s.step(tx, ty, vx, vy)) for _ in range(3)]
            torch.cuda.synchronize()
            res[backend] = (losses, s.W.clone(), s.A.clone())
    finally:
        hip_darts.set_selffold(False)
        hip_darts.EDGE_BWD = old_edge
        dops.set_backend("torch")
    (lt, Wt, At), (lh, Wh, Ah) = res["torch"], res["hip"]
    assert max(abs(a - b) for a, b in zip(lt, lh)) < 1e-3
    _close(Wh, Wt, "W", rtol=1e-3, atol=1e-4)
    _close(Ah, At, "alpha", rtol=5e-2, atol=5e-5)


@pytest.mark.parametrize("leaf_alphas", [True, False])
def test_network_function_matches_per_cell_path(leaf_alphas):
    """The whole-network Function (hip_darts.network_loss: node-major cell outputs, first-writer
    gradient buffers, fused alpha softmax / alpha gradient) computes what the per-cell Functions
    under autograd compute: loss, logits, weight and alpha gradients, BN running statistics; with
    leaf alpha matrices (DartsSearch) the alpha gradient is written into the leaves' .grad, with
    per-node alpha rows it flows back through autograd."""
    from katib_amd.models.darts import BNState, DartsLayout, DartsNetwork
    from katib_amd.ops import darts as dops

    dops.set_backend("hip")
    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=3, num_nodes=3, stem_multiplier=1)
    g = torch.Generator().manual_seed(3)
    W = torch.zeros(layout.n_weights)
    layout.init_weights(W, g)
    A = 1e-1 * torch.randn(layout.n_alphas, generator=g)
    x = torch.randn(32, 3, 32, 32, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    out = {}
    for mode in (True, False):
        net = DartsNetwork(layout, ops=dops)
        net.net_function = mode
        Wl = W.to(dev).requires_grad_(True)
        P = layout.views(Wl)
        Al = A.to(dev)
        rows, K = layout.n_alpha_rows, len(layout.prims)
        an = Al[:rows * K].view(rows, K).clone().requires_grad_(True)
        ar = Al[rows * K:].view(rows, K).clone().requires_grad_(True)
        if leaf_alphas:
            an.grad, ar.grad = torch.zeros_like(an), torch.zeros_like(ar)
            na, ra = an, ar
        else:
            na, ra = list(an.split([2 + i for i in range(layout.N)])), list(ar.split([2 + i for i in range(layout.N)]))
        bn = BNState(layout, dev)
        loss, logits = net.forward_loss(x, y, P, na, ra, bn, training=True)
        loss.backward(inputs=[Wl, an, ar])
        torch.cuda.synchronize()
        out[mode] = (loss.detach(), logits.detach(), Wl.grad.clone(), an.grad.clone(), ar.grad.clone(), bn.buf.clone())
        dops.set_backend("hip")
    # both paths sum float atomics in a run-dependent order (and the gradient of a cell state in a
    # different order: first-writer buffers vs autograd additions): fp32 rounding-level differences
    for name_, a, b in zip(["loss", "logits", "gW", "ga_n", "ga_r", "bn"], out[True], out[False]):
        _close(a, b, name_, rtol=5e-3, atol=1e-5)
    dops.set_backend("torch")


@pytest.mark.parametrize("capture", [False, True])
def test_stacked_hessian_passes_match_concurrent_and_sequential(capture):
    """the +eps / -eps finite-difference passes recorded and issued as ONE pass of
    edge-batched launches (hip_darts.stacked_passes) compute what the two concurrent graph branches
    and the sequential in-place perturbation compute: weights, alphas and BN running statistics after
    3 second-order steps; and most launches of the pair really merge."""
    from katib_amd.models.darts import DartsLayout
    from katib_amd.models.darts_search import DartsSearch
    from katib_amd.ops import darts as dops

    dev = torch.device("cuda", 0)
    layout = DartsLayout(ALL, init_channels=4, num_layers=2, num_nodes=3, stem_multiplier=1)
    gen = torch.Generator(device=dev).manual_seed(5)
    batches = [(torch.randn(32, 3, 32, 32, device=dev, generator=gen), torch.randint(0, 10, (32,), device=dev, generator=gen),
                torch.randn(32, 3, 32, 32, device=dev, generator=gen), torch.randint(0, 10, (32,), device=dev, generator=gen))
               for _ in range(3)]
    dops.set_backend("hip")
    res = {}
    for mode in ("stacked", "concurrent", "sequential"):
        s = DartsSearch(layout, dev, capture=capture, hessian=mode)
        assert s.hessian == mode
        for b in batches:
            s.step(*b)
        torch.cuda.synchronize()
        res[mode] = (s.W.clone(), s.A.clone(), s.bn.mean.clone(), s.bn.var.clone(), s.stack_stats)
    dops.set_backend("torch")
    st = res["stacked"][4]
    assert st is not None and st["merged"] >= 40, st
    for other in ("concurrent", "sequential"):
        for name_, a, b in zip(["W", "alpha", "rm", "rv"], res["stacked"][:4], res[other][:4]):
            # alphas move by a finite difference over eps = 0.01 / ||dw'||: float-atomic summation order
            # (workgroup counts differ between the modes) shows up there first
            tol = dict(rtol=1e-3, atol=5e-5) if name_ == "alpha" else dict(rtol=1e-4, atol=1e-5)
            _close(a, b, "%s vs %s: %s" % ("stacked", other, name_), **tol)
