"""GPT-2 trial kernels (csrc/hip/transformer.hip) vs the fp32 PyTorch implementations of the
same contracts (ops/transformer.TorchOps) on the same bf16-rounded inputs, plus a whole
flat-model training step (HIP vs torch ops) and the graph-captured trial."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


@pytest.fixture(scope="module")
def ops():
    from katib_amd.ops.transformer import HipOps, TorchOps

    return HipOps(), TorchOps()


def _gen(seed=3):
    return torch.Generator(device=DEV).manual_seed(seed)


@pytest.mark.parametrize("D", [256, 768, 1024])
@pytest.mark.parametrize("residual", [False, True])
def test_layernorm_fwd_bwd(ops, D, residual):
    hip, ref = ops
    g = _gen()
    M = 333
    x = torch.randn(M, D, device=DEV, generator=g) * 2 + 0.5
    r = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16) if residual else None
    gamma = (1 + 0.1 * torch.randn(D, device=DEV, generator=g)).to(torch.bfloat16)
    beta = (0.1 * torch.randn(D, device=DEV, generator=g)).to(torch.bfloat16)
    xh, yh, mh, rh = hip.ln_fwd(x, r, gamma, beta)
    xr, yr, mr, rr = ref.ln_fwd(x, r, gamma, beta)
    assert _rel(xh, xr) < 1e-6 and _rel(mh, mr) < 1e-5 and _rel(rh, rr) < 1e-4
    assert _rel(yh, yr) < 1e-2
    dy = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    G0 = torch.randn(M, D, device=DEV, generator=g)
    outs = []
    for o in (hip, ref):
        G = G0.clone()
        dr = torch.empty(M, D, device=DEV, dtype=torch.bfloat16)
        dg = torch.empty(D, device=DEV, dtype=torch.bfloat16)
        db = torch.empty_like(dg)
        o.ln_bwd(dy, xr, mr, rr, gamma, G, dr, dg, db)
        outs.append((G, dr, dg, db))
    (Gh, drh, dgh, dbh), (Gr, drr, dgr, dbr) = outs
    assert _rel(Gh, Gr) < 1e-4
    assert _rel(drh, drr) < 1e-2
    assert _rel(dgh, dgr) < 1e-2 and _rel(dbh, dbr) < 1e-2


def test_gelu(ops):
    hip, ref = ops
    g = _gen()
    u = (torch.randn(4096 * 3 + 8 * 5, device=DEV, generator=g) * 3).to(torch.bfloat16)
    dy = torch.randn(u.shape, device=DEV, generator=g).to(torch.bfloat16)
    assert _rel(hip.gelu_fwd(u), ref.gelu_fwd(u)) < 1e-2
    assert _rel(hip.gelu_bwd(u, dy), ref.gelu_bwd(u, dy)) < 1e-2


@pytest.mark.parametrize("M", [256, 16384])
def test_dgrad_gelu_epilogue(ops, M):
    """gemm_lt NN dgrad with the GELU backward in its epilogue vs fp32 (dy @ w) * gelu'(u)."""
    hip, ref = ops
    g = _gen(7)
    D, F4 = 768, 3072
    dy = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(D, F4, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    u = (torch.randn(M, F4, device=DEV, generator=g) * 2).to(torch.bfloat16)
    du = hip.dgrad_gelu(dy, w, u)
    x = u.float()
    k0, k1 = math.sqrt(2.0 / math.pi), 0.044715
    t = torch.tanh(k0 * (x + k1 * x ** 3))
    d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
    want = (dy.float() @ w.float()) * d
    assert _rel(du, want) < 2e-2
    assert _rel(du, ref.dgrad_gelu(dy, w, u)) < 2e-2
    # the epilogue path really ran (same bits as a direct call)
    out = torch.empty_like(du)
    hip.k.gemm_lt(dy, False, w, True, None, out, 1, u)
    assert torch.equal(out, du)
    # + the bias gradient (default: colsum pass; the epilogue's per-64-row column sums directly)
    db = torch.empty(F4, device=DEV, dtype=torch.bfloat16)
    du2 = hip.dgrad_gelu(dy, w, u, db)
    assert torch.equal(du2, du)
    assert _rel(db, du.float().sum(0)) < 1e-2
    part = torch.empty(M // 64, F4, device=DEV, dtype=torch.float32)
    out2 = torch.empty_like(du)
    hip.k.gemm_lt(dy, False, w, True, None, out2, 1, u, part)
    assert torch.equal(out2, du)
    assert _rel(part.sum(0), du.float().sum(0)) < 1e-3
    dbr = torch.empty_like(db)
    ref.dgrad_gelu(dy, w, u, dbr)
    assert _rel(db, dbr) < 2e-2


@pytest.mark.parametrize("V,Vp", [(1000, 1024), (50257, 50304), (512, 512)])
def test_cross_entropy(ops, V, Vp):
    hip, ref = ops
    g = _gen()
    N = 67
    logits = (torch.randn(N, Vp, device=DEV, generator=g) * 3).to(torch.bfloat16)
    logits[:, V:] = 100.0  # pad columns must be ignored
    tgt = torch.randint(0, V, (N,), device=DEV, generator=g)
    lh, sh = hip.xent_fwd(logits, tgt, V)
    lr, sr = ref.xent_fwd(logits, tgt, V)
    assert _rel(lh, lr) < 1e-4 and _rel(sh, sr) < 1e-5
    gs = torch.full((1,), 0.7, device=DEV)
    dh = hip.xent_bwd(logits.clone(), tgt, sh, gs, V)
    dr = ref.xent_bwd(logits.clone(), tgt, sr, gs, V)
    assert _rel(dh, dr) < 1e-2
    assert V == Vp or float(dh[:, V:].abs().max()) == 0.0
    # one-pass training form (forward + backward over a single read of the logits)
    lf, sf, df = hip.xent_train(logits.clone(), tgt, gs, V)
    assert _rel(lf, lr) < 1e-4 and _rel(sf, sr) < 1e-5
    assert _rel(df, dr) < 1e-2
    assert V == Vp or float(df[:, V:].abs().max()) == 0.0


@pytest.mark.parametrize("V,Vp", [(1000, 1024), (50257, 50304), (512, 512)])
def test_cross_entropy_eval(ops, V, Vp):
    """the validation loss + top-1 of the PBT member in one pass over the bf16
    logits (xent_eval_k) against F.cross_entropy / argmax on the fp32 copy; includes tied maxima
    (torch.argmax picks the lowest index) and pad columns that must be ignored."""
    hip, ref = ops
    g = _gen(V)
    N = 131
    logits = (torch.randn(N, Vp, device=DEV, generator=g) * 3).to(torch.bfloat16)
    logits[:, V:] = 100.0
    tgt = torch.randint(0, V, (N,), device=DEV, generator=g)
    am = logits[:, :V].float().argmax(-1)
    tgt[:40] = am[:40]  # hits
    logits[40:50, 7] = logits[40:50, :V].float().max(-1).values.to(torch.bfloat16) + 1.0
    logits[40:50, V - 3] = logits[40:50, 7]  # a tie: index 7 wins
    tgt[40:45] = 7
    tgt[45:50] = V - 3
    lh, ch = hip.xent_eval(logits, tgt, V)
    lr, cr = ref.xent_eval(logits, tgt, V)
    assert abs(float(lh) - float(lr)) <= 1e-4 * abs(float(lr))
    assert float(ch) == float(cr) and float(cr) >= 45


@pytest.mark.parametrize("B,T,H", [(2, 128, 3), (1, 512, 2), (2, 256, 4)])
def test_attention_fwd_bwd(ops, B, T, H):
    hip, ref = ops
    g = _gen(B * T + H)
    qkv = torch.randn(B * T, 3 * H * 64, device=DEV, generator=g).to(torch.bfloat16)
    oh, lh = hip.attn_fwd(qkv, B, T, H)
    orf, lr = ref.attn_fwd(qkv, B, T, H)
    assert _rel(oh, orf) < 2e-2, _rel(oh, orf)
    assert float((lh - lr).abs().max()) < 1e-2
    do = torch.randn(B * T, H * 64, device=DEV, generator=g).to(torch.bfloat16)
    dh = hip.attn_bwd(qkv, oh, do, lh, B, T, H)
    dr = ref.attn_bwd(qkv, orf, do, lr, B, T, H)
    d5h, d5r = dh.view(B, T, 3, H, 64), dr.view(B, T, 3, H, 64)
    for part in range(3):
        assert _rel(d5h[:, :, part], d5r[:, :, part]) < 3e-2, (part, _rel(d5h[:, :, part], d5r[:, :, part]))


def test_attention_forced_rescale(ops):
    """A key whose score jumps far above the running max in a late tile forces the online
    softmax rescale (guide rule 26): one query row attends almost only to that key."""
    hip, ref = ops
    B, T, H = 1, 256, 1
    g = _gen(11)
    x = torch.randn(B * T, 3 * 64, device=DEV, generator=g) * 0.5
    q, k = x[:, :64], x[:, 64:128]
    q[200] = 2.0
    k[190] = 2.0  # tile 2 (keys 128..191): score 2*2*64/8 = 32 >> the first tiles' max
    qkv = x.to(torch.bfloat16)
    oh, lh = hip.attn_fwd(qkv, B, T, H)
    orf, lr = ref.attn_fwd(qkv, B, T, H)
    assert _rel(oh, orf) < 2e-2
    assert float((lh - lr).abs().max()) < 1e-2


def test_adamw(ops):
    hip, ref = ops
    g = _gen()
    n = 4096 + 8 * 13
    p0 = torch.randn(n, device=DEV, generator=g)
    gr = torch.randn(n, device=DEV, generator=g).to(torch.bfloat16)
    res = []
    for o in (hip, ref):
        p, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        w16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
        lr, step, ss = torch.full((1,), 1e-2, device=DEV), torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
        for _ in range(3):
            step += 1
            o.adamw(p, gr, m, v, w16, lr, step, 0.9, 0.95, 1e-8, 0.1, 1.0, ss)
        res.append((p, m, v, w16, ss))
    for a, b in zip(*res):
        assert _rel(a, b) < 1e-4


def _cfg():
    from katib_amd.workloads.gpt2_pbt import GPTConfig

    return GPTConfig(vocab=1000, ctx=128, n_layer=2, n_head=4, d=256)


def test_flat_gpt_step_hip_vs_torch(ops):
    from katib_amd.models.gpt2 import GPT2Flat

    hip, ref = ops
    cfg = _cfg()
    g = _gen()
    idx = torch.randint(0, cfg.vocab, (2, 128), device=DEV, generator=g)
    tgt = torch.randint(0, cfg.vocab, (2, 128), device=DEV, generator=g)
    mh = GPT2Flat(cfg, DEV, hip, seed=5)
    mr = GPT2Flat(cfg, DEV, ref, seed=5)
    lh = mh.forward_backward(idx, tgt)
    lr = mr.forward_backward(idx, tgt)
    assert abs(float(lh) - float(lr)) < 2e-2 * abs(float(lr))
    for n in ("wte.weight", "blocks.0.qkv.weight", "blocks.1.fc2.weight", "blocks.0.ln1.weight", "wpe.weight"):
        assert _rel(mh.g[n], mr.g[n]) < 6e-2, (n, _rel(mh.g[n], mr.g[n]))
    mh.optimizer_step()
    mr.optimizer_step()
    assert _rel(mh.p32, mr.p32) < 1e-3


def test_gpt2_trial_captured_flat(tmp_path):
    """The trial on the flat HIP model (graph-captured) learns like the nn.Module + autograd
    implementation, and its checkpoint loads into the module implementation."""
    from katib_amd.workloads import gpt2_pbt

    gpt2_pbt.PRESETS["gpu-test"] = _cfg()
    common = ["--model", "gpu-test", "--batch-size", "8", "--lr", "3e-3", "--num-tokens", "200000", "--p2p", "0"]
    ck = str(tmp_path / "ck")
    v_flat = gpt2_pbt.main(common + ["--steps", "40", "--checkpoint-dir", ck, "--impl", "flat"])
    v_mod = gpt2_pbt.main(common + ["--steps", "40", "--checkpoint-dir", str(tmp_path / "ck2"), "--impl", "module"])
    v_cont = gpt2_pbt.main(common + ["--steps", "5", "--checkpoint-dir", ck, "--impl", "module"])
    assert all(math.isfinite(v) for v in (v_flat, v_mod, v_cont))
    assert v_flat < math.log(1000) - 0.3 and v_mod < math.log(1000) - 0.3
    assert abs(v_flat - v_mod) < 0.15, (v_flat, v_mod)
    assert v_cont < math.log(1000) - 1.0  # continued from the flat checkpoint (5 steps from scratch: ~6.8)


@pytest.mark.parametrize("M,N,K", [(16384, 768, 768), (16384, 3072, 768), (4096, 768, 3072), (300, 64, 40)])
def test_wgrad_and_colsum(ops, M, N, K):
    hip, _ = ops
    g = _gen()
    dy = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    out = torch.empty(N, K, device=DEV, dtype=torch.bfloat16)
    hip.wgrad(dy, x, out)
    ref = dy.float().t() @ x.float()
    assert _rel(out, ref) < 1e-2
    b = torch.empty(N, device=DEV, dtype=torch.bfloat16)
    hip.colsum(dy, b)
    assert _rel(b, dy.float().sum(0)) < 1e-2
