// NHWC bf16 BatchNorm (+ residual + ReLU) kernels (batchnorm.hip). x, y, residual: [P, C]
// bf16 (P = N*H*W, C % 8 == 0); statistics and parameters fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

namespace katib_hip {
namespace bn {

typedef __hip_bfloat16 bf16;

// Row-chunk plan of the statistics passes: part must hold R * 2 * C floats.
void plan(int P, int C, int* R, int* rows, int* cvb);

// Training forward: batch statistics (mean, invstd out), running stats updated in place when
// rmean != nullptr, ss = [scale; shift] (2C), y = relu?(x * scale + shift + res?).
hipError_t fwd_train(const bf16* x, const bf16* res, bf16* y, const float* gamma, const float* beta, float* rmean,
                     float* rvar, float* mean, float* invstd, float* ss, float* part, int P, int C, float eps,
                     float momentum, int relu, hipStream_t st, long long* counter = nullptr);
// Inference forward with the running statistics.
hipError_t fwd_eval(const bf16* x, const bf16* res, bf16* y, const float* gamma, const float* beta,
                    const float* rmean, const float* rvar, float* ss, int P, int C, float eps, int relu,
                    hipStream_t st);
// Backward. y (the forward output) masks dy when the forward applied ReLU (nullptr: no ReLU);
// dres (may be nullptr) receives the masked gradient that flows to the residual input.
// accumulate: dgamma / dbeta += instead of = (persistent gradient buffers).
hipError_t bwd(const bf16* dy, const bf16* y, const bf16* x, const float* gamma, const float* mean,
               const float* invstd, bf16* dx, bf16* dres, float* dgamma, float* dbeta, float* coef, float* part, int P,
               int C, hipStream_t st, int accumulate = 0);

// Per-channel sum of a [P, C] bf16 activation into out[C] fp32 (bias gradients): the statistics
// pass into part (R * 2 * C floats) + one finalize launch; deterministic, no atomics and no
// zero-initialised workspace, so it replays correctly from a HIP graph.
hipError_t channel_sum(const bf16* x, float* out, float* part, int P, int C, hipStream_t st);

}  // namespace bn
}  // namespace katib_hip
