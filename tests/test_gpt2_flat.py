"""Flat-buffer GPT-2 (models/gpt2.py) with its hand-written backward vs autograd through the
nn.Module GPT of the trial (fp32, torch ops backend): loss, every parameter gradient and one
clipped AdamW step. Plus the trial program on both implementations with checkpoint carry."""
import math

import torch
import torch.nn.functional as F


def test_flat_gpt_matches_autograd():
    from katib_amd.models.gpt2 import GPT2Flat
    from katib_amd.ops.transformer import TorchOps
    from katib_amd.workloads.gpt2_pbt import GPT, GPTConfig

    torch.manual_seed(0)
    cfg = GPTConfig(vocab=100, ctx=32, n_layer=2, n_head=2, d=128)
    ref = GPT(cfg)
    flat = GPT2Flat(cfg, "cpu", TorchOps(), dtype=torch.float32)
    flat.load_state_dict(ref.state_dict())
    idx = torch.randint(0, 100, (3, 32))
    tgt = torch.randint(0, 100, (3, 32))
    loss_ref = F.cross_entropy(ref(idx).view(-1, 100), tgt.view(-1))
    loss_ref.backward()
    loss = flat.forward_backward(idx, tgt)
    assert abs(float(loss) - float(loss_ref)) < 1e-5
    for n, p in ref.named_parameters():
        gf = flat.g[n][:p.shape[0]]
        assert float((gf - p.grad).abs().max()) <= 1e-4 * float(p.grad.abs().max()) + 1e-9, n
    assert float(flat.g["wte.weight"][100:].abs().max()) == 0.0  # vocabulary pad rows
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, betas=(0.9, 0.95), weight_decay=0.1, eps=1e-8)
    torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
    opt.step()
    flat.lr_t.fill_(1e-3)
    flat.optimizer_step(max_norm=0.5)
    sd = flat.state_dict()
    for n, p in ref.named_parameters():
        assert float((sd[n] - p.detach()).abs().max()) < 5e-5, n


def test_gpt2_trial_flat_and_module_cpu(tmp_path):
    from katib_amd.workloads import gpt2_pbt

    ck = str(tmp_path / "ck")
    common = ["--model", "tiny", "--batch-size", "4", "--num-tokens", "50000", "--checkpoint-dir", ck]
    v1 = gpt2_pbt.main(common + ["--steps", "6", "--impl", "flat"])
    v2 = gpt2_pbt.main(common + ["--steps", "3", "--impl", "module"])
    v3 = gpt2_pbt.main(common + ["--steps", "3", "--impl", "flat"])
    assert all(math.isfinite(v) for v in (v1, v2, v3))
    st = torch.load(tmp_path / "ck" / "optim.pt", weights_only=True)
    assert int(st["step"]) == 12
