// Fused MLP training kernels (mlp.hip): bf16 activations/weight shadows, fp32 masters.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace katib_hip {
namespace mlp {

typedef __hip_bfloat16 bf16;

// y[M][N] = epi(x[idx?][K] . w[N][K]^T); epi = + bias (may be null), ReLU if relu, * [mask > 0] if mask.
hipError_t lin_fwd(const bf16* x, const int64_t* idx, const bf16* w, const float* bias, const bf16* mask, bf16* y,
                   int M, int N, int K, int relu, hipStream_t st);
// dW = dy^T x (x rows through idx when given) and SGD with momentum on w (fp32 [N][K]), its momentum
// buffer, bf16 shadows w16 [N][K] / w16t [K][N]; bias (+ its buffer) updated from the column sums of dy.
hipError_t lin_wgrad_sgd(const bf16* dy, const bf16* x, const int64_t* idx, int M, int N, int K, float* w, float* wm,
                         bf16* w16, bf16* w16t, float* bias, float* bm, const float* lr, float momentum,
                         hipStream_t st);
// softmax cross-entropy over the first C of ld columns; dl = (softmax - onehot) / M; stats += (mean loss, correct).
hipError_t xent_small(const bf16* logits, const int64_t* y, const int64_t* idx, bf16* dl, int M, int C, int ld,
                      float* stats, hipStream_t st);

}  // namespace mlp
}  // namespace katib_hip
