// GPT-2 trial kernels for gfx950 (transformer.hip): fused residual-add + LayerNorm,
// tanh-GELU, vocabulary cross-entropy, flat-buffer AdamW with global-norm clipping,
// and causal flash attention (forward, dQ, dK/dV) on v_mfma_f32_16x16x32_bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace katib_hip {
namespace tfm {

typedef __hip_bfloat16 bf16;

// LayerNorm over rows of D (D % 256 == 0, D <= 4096). x32: fp32 residual stream.
// If r != nullptr: xo = x32 + r (written), LN input = xo; else LN input = x32.
hipError_t ln_fwd(const float* x32, const bf16* r, float* xo, const bf16* gamma, const bf16* beta, bf16* y,
                  float* mean, float* rstd, int M, int D, float eps, hipStream_t st);
// dx = LN'(dy) (+ dres if given), written fp32 (may alias dres); dr = bf16(dx) if given;
// per-block dgamma/dbeta partials [nblk][D] (fp32) -> ln_reduce_params writes bf16 grads.
int ln_bwd_blocks(int M);
hipError_t ln_bwd(const bf16* dy, const float* xin, const float* mean, const float* rstd, const bf16* gamma,
                  const float* dres, float* dx, bf16* dr, float* part_g, float* part_b, int M, int D,
                  hipStream_t st, float* part_r = nullptr);
// part_r / dbias (optional): column sums of the bf16 dr output -> the bias gradient of the linear
// layer whose output gradient dr is.
hipError_t ln_reduce_params(const float* part_g, const float* part_b, int nblk, int D, bf16* dgamma, bf16* dbeta,
                            hipStream_t st, const float* part_r = nullptr, bf16* dbias = nullptr);

// tanh-approximate GELU on bf16 (n % 8 == 0).
hipError_t gelu_fwd(const bf16* u, bf16* g, int64_t n, hipStream_t st);
hipError_t gelu_bwd(const bf16* u, const bf16* dy, bf16* du, int64_t n, hipStream_t st);

// Cross-entropy over the first V columns of rows of stride Vp (Vp % 8 == 0).
// evaluation: per-row loss (lse - logit[tgt]) and top-1 hit (argmax == tgt, ties to the lowest index)
hipError_t xent_eval(const bf16* logits, const int64_t* tgt, float* loss, float* hit, int N, int V, int Vp,
                     hipStream_t st);
hipError_t xent_fwd(const bf16* logits, const int64_t* tgt, float* loss, float* lse, int N, int V, int Vp,
                    hipStream_t st);
// dlogits = (softmax - onehot) * (*gscale) * inv_n, written in place over logits (pad columns -> 0).
hipError_t xent_bwd(bf16* logits, const int64_t* tgt, const float* lse, const float* gscale, float inv_n, int N,
                    int V, int Vp, hipStream_t st);
// Training cross-entropy in one pass: per-row loss and lse, and the gradient written in place over the
// logits (Vp <= 53248); hipErrorInvalidValue for wider rows (use xent_fwd + xent_bwd).
hipError_t xent_fused(bf16* logits, const int64_t* tgt, float* loss, float* lse, const float* gscale, float inv_n,
                      int N, int V, int Vp, hipStream_t st);

// sumsq[0] += sum(g^2) over a flat bf16 gradient (caller zeroes sumsq).
hipError_t grad_sumsq(const bf16* g, int64_t n, float* sumsq, hipStream_t st);
// AdamW over flat buffers; clip scale = min(1, max_norm / (sqrt(*sumsq) + 1e-6)) (max_norm <= 0: none);
// lr and the step count are device scalars so a captured graph replays with new values.
hipError_t adamw(float* p, const bf16* g, float* m, float* v, bf16* w16, int64_t n, const float* lr,
                 const float* step, float beta1, float beta2, float eps, float wd, const float* sumsq,
                 float max_norm, hipStream_t st);

// out[c] = bf16(sum_r part[r][c]) (split-K / partial-sum reduction), n % 4 == 0.
hipError_t reduce_rows(const float* part, int R, int64_t n, bf16* out, hipStream_t st);
// out[c] = bf16(sum_r x[r][c]) for x [M, N] bf16 (N % 8 == 0); part: fp32 [colsum_chunks(M, N)][N] scratch.
int colsum_chunks(int M, int N);
hipError_t colsum(const bf16* x, int M, int N, float* part, bf16* out, hipStream_t st);

// Causal flash attention, head dim 64. qkv [B, T, 3, H, 64] bf16; o [B, T, H, 64] bf16;
// lse [B, H, T] fp32 in the log2 domain of the scaled scores. T % 128 == 0.
hipError_t attn_fwd(const bf16* qkv, bf16* o, float* lse, int B, int T, int H, float sm_scale, hipStream_t st);
// dqkv [B, T, 3, H, 64] bf16 (fully written); delta [B, H, T] fp32 scratch.
hipError_t attn_bwd(const bf16* qkv, const bf16* o, const bf16* dout, const float* lse, float* delta, bf16* dqkv,
                    int B, int T, int H, float sm_scale, hipStream_t st);

}  // namespace tfm
}  // namespace katib_hip
