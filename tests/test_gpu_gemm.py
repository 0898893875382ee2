"""bf16 NT GEMM (gemm_bf16.hip) vs the fp32 PyTorch formula: C = A W^T (+ bias) (+ tanh GELU), the
GPT-2-small projection shapes (rows cut to keep the test short), asymmetric data so a transposed
or mis-swizzled tile cannot pass, and the GPT-2 forward through the HIP ops vs the torch ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _k():
    from katib_amd import _hipload

    return _hipload.hipkern()


@pytest.mark.parametrize("M,N,K,bias,gelu", [(128, 128, 64, True, False), (256, 2304, 768, True, False),
                                             (512, 768, 768, True, False), (256, 3072, 768, True, True),
                                             (384, 768, 3072, True, False), (128, 50304, 768, False, False),
                                             (1024, 256, 128, False, True)])
def test_gemm_nt_matches_fp32(M, N, K, bias, gelu):
    k = _k()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    # asymmetric structure: a row ramp in A and a column ramp in W
    A += (torch.arange(M, device=dev)[:, None] % 7 * 0.1).to(torch.bfloat16)
    W += (torch.arange(K, device=dev)[None, :] % 5 * 0.01).to(torch.bfloat16)
    b = (torch.randn(N, device=dev, generator=g) * 0.1).to(torch.bfloat16) if bias else None
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    G = torch.empty_like(C) if gelu else None
    k.gemm_nt(A, W, b, C, G)
    ref = A.float() @ W.float().t() + (b.float() if bias else 0.0)
    torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()) ** 0.5)
    if gelu:
        refg = F.gelu(C.float(), approximate="tanh")
        torch.testing.assert_close(G.float(), refg, rtol=2e-2, atol=1e-2)


def test_gpt2_forward_hip_gemm_matches_torch_ops():
    """Every forward projection of a small GPT-2 (qkv, proj, fc + fused GELU, fc2, the tied LM
    head: vocab 1024 so it takes the HIP GEMM too) against the torch ops."""
    from katib_amd.models.gpt2 import GPT2Flat
    from katib_amd.ops.transformer import get_ops
    from katib_amd.workloads.gpt2_pbt import GPTConfig

    dev = torch.device("cuda", 0)
    cfg = GPTConfig(vocab=1024, ctx=128, n_layer=2, n_head=4, d=256)
    idx = torch.randint(0, 1024, (2, 128), device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    hip = get_ops("hip", dev)
    hip.gemm = "all"  # every projection on gemm_bf16, not only the shapes where it wins
    assert hip._gemm_ok(torch.empty(256, 256, device=dev, dtype=torch.bfloat16),
                                     torch.empty(1024, 256, device=dev, dtype=torch.bfloat16))
    outs = []
    for ops in (get_ops("torch", dev), hip):
        m = GPT2Flat(cfg, dev, ops, seed=0)
        outs.append(m.forward(idx).float())
    torch.testing.assert_close(outs[1], outs[0], rtol=5e-2, atol=5e-2)


@pytest.mark.parametrize("a_mn,b_mn", [(False, True), (True, True), (True, False), (False, False)])
@pytest.mark.parametrize("M,N,K,splitk", [(128, 128, 64, 1), (256, 768, 2304, 1), (768, 768, 4096, 4),
                                          (384, 256, 1024, 2), (3072, 768, 2048, 8)])
def test_gemm_lt_layouts_match_fp32(a_mn, b_mn, M, N, K, splitk):
    """Layout-native GEMM (gemm_lt_kernel): NN (dgrad), TN (wgrad), NT and TT operand layouts, the
    MN-contiguous operands read through ds_read_b64_tr_b16 with the swizzled LDS image; bf16 output
    (splitk 1) or fp32 split-K slabs summed here. Asymmetric data so a transposed fragment fails."""
    k = _k()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M * 3 + N * 5 + K + 7 * splitk)
    opA = torch.randn(M, K, device=dev, generator=g) + (torch.arange(M, device=dev)[:, None] % 7) * 0.1
    opB = (torch.randn(K, N, device=dev, generator=g) + (torch.arange(N, device=dev)[None, :] % 5) * 0.05) * 0.05
    opA, opB = opA.to(torch.bfloat16), opB.to(torch.bfloat16)
    A = opA.t().contiguous() if a_mn else opA  # stored [K][M] or [M][K]
    B = opB.contiguous() if b_mn else opB.t().contiguous()  # stored [K][N] or [N][K]
    ref = opA.float() @ opB.float()
    tol = dict(rtol=2e-2, atol=2e-2 * float(ref.abs().max()) ** 0.5)
    if splitk == 1:
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        k.gemm_lt(A, a_mn, B, b_mn, None, C)
        torch.testing.assert_close(C.float(), ref, **tol)
    C32 = torch.empty(splitk, M, N, device=dev, dtype=torch.float32)
    k.gemm_lt(A, a_mn, B, b_mn, None, C32, splitk)
    torch.testing.assert_close(C32.sum(0), ref, rtol=1e-3, atol=1e-3 * float(ref.abs().max()))


def test_gemm_lt_bias_and_errors():
    k = _k()
    dev = torch.device("cuda", 0)
    A = torch.randn(256, 512, device=dev).to(torch.bfloat16)
    B = torch.randn(512, 384, device=dev).to(torch.bfloat16)
    b = torch.randn(384, device=dev).to(torch.bfloat16)
    C = torch.empty(256, 384, device=dev, dtype=torch.bfloat16)
    k.gemm_lt(A, False, B, True, b, C)
    ref = A.float() @ B.float() + b.float()
    torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=0.2)
    with pytest.raises(RuntimeError):
        k.gemm_lt(A, False, B[:, :100].contiguous(), True, None, C)  # N % 128
    with pytest.raises(RuntimeError):
        k.gemm_lt(A, False, B, True, None, C, 2)  # bf16 output with split-K


@pytest.mark.parametrize("a_mn,b_mn", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K,splitk", [(256, 256, 64, 1), (512, 768, 768, 1), (384, 640, 192, 1),
                                          (256, 2304, 3072, 1), (768, 768, 4096, 4), (1280, 384, 2048, 8)])
def test_gemm256_layouts_match_fp32(a_mn, b_mn, M, N, K, splitk):
    """256x256-tile 8-wave ping-pong GEMM (gemm256.hip): forward (K, K), dgrad (K, MN), wgrad (MN, MN)
    and the fourth layout; one K-tile (K 64: the prologue-only path), M / N that leave a half-outside
    last tile (384, 640, 1280: clamped staging, skipped stores), bf16 output or fp32 split-K slabs.
    Asymmetric data so a transposed or mis-swizzled fragment fails."""
    k = _k()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M * 3 + N * 5 + K + 7 * splitk + 11 * a_mn + 13 * b_mn)
    opA = torch.randn(M, K, device=dev, generator=g) + (torch.arange(M, device=dev)[:, None] % 7) * 0.1
    opB = (torch.randn(K, N, device=dev, generator=g) + (torch.arange(N, device=dev)[None, :] % 5) * 0.05) * 0.05
    opA, opB = opA.to(torch.bfloat16), opB.to(torch.bfloat16)
    A = opA.t().contiguous() if a_mn else opA
    B = opB.contiguous() if b_mn else opB.t().contiguous()
    ref = opA.float() @ opB.float()
    if splitk == 1:
        C = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        k.gemm256(A, a_mn, B, b_mn, None, C)
        torch.testing.assert_close(C.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()) ** 0.5)
    C32 = torch.full((splitk, M, N), float("nan"), device=dev, dtype=torch.float32)
    k.gemm256(A, a_mn, B, b_mn, None, C32, None, splitk)
    torch.testing.assert_close(C32.sum(0), ref, rtol=1e-3, atol=1e-3 * float(ref.abs().max()))


@pytest.mark.parametrize("M,N,K", [(512, 3072, 768), (256, 50304, 768), (384, 384, 128)])
def test_gemm256_bias_gelu_epilogue(M, N, K):
    """Forward epilogues: bias, and U = A W^T + b with G = gelu_tanh(U) (the fc layer); N = 50304 is
    the padded GPT-2 vocabulary (a half-outside last column tile)."""
    k = _k()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    A = (torch.randn(M, K, device=dev, generator=g) + (torch.arange(M, device=dev)[:, None] % 7) * 0.1).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = (torch.randn(N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    U = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    G = torch.empty_like(U)
    k.gemm256(A, False, W, False, b, U, G)
    ref = A.float() @ W.float().t() + b.float()
    torch.testing.assert_close(U.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()) ** 0.5)
    torch.testing.assert_close(G.float(), F.gelu(U.float(), approximate="tanh"), rtol=2e-2, atol=1e-2)
    with pytest.raises(RuntimeError):
        k.gemm256(A, False, W[:100].contiguous(), False, None, U[:, :100].contiguous())  # N % 128
