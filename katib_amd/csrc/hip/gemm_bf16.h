// bf16 NT GEMM with fused bias / bias + GELU epilogue (gemm_bf16.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {
namespace gemm {

bool supported(int M, int N, int K);  // M, N multiples of 128, K of 64
// C[M][N] = A[M][K] W[N][K]^T (+ bias[N]); G != nullptr: C = pre-activation, G = gelu_tanh(C)
hipError_t launch_nt(const void* A, const void* W, const void* bias, void* C, void* G, int M, int N, int K,
                     hipStream_t st);

// Layout-native GEMM: C = op(A) op(B), op(A)[M][K] from A stored [M][K] (a_mn false) or [K][M]
// (a_mn true), op(B)[K][N] from B stored [N][K] (b_mn false) or [K][N] (b_mn true); lda / ldb are
// the stored row strides (elements). out_f32: C is an fp32 slab [splitk][M][N] (one slab per K
// slice), else bf16 [M][N] (+ bias[N], splitk 1). M, N multiples of 128, K of 64 * splitk.
// gelu_u (bf16 output only): C = (product + bias) * gelu_tanh'(gelu_u[M][N]) - the GELU backward of the
// MLP folded into its dgrad epilogue. colpart (bf16 output only): fp32 column sums of the stored C per
// 64-row block, colpart[M / 64][N] (reduced over blocks by the caller: the bias gradient).
hipError_t launch_lt(const void* A, int lda, bool a_mn, const void* B, int ldb, bool b_mn, const void* bias, void* C,
                     bool out_f32, int splitk, int M, int N, int K, hipStream_t st, const void* gelu_u = nullptr,
                     float* colpart = nullptr);

// 256 x 256-tile, 8-wave ping-pong GEMM (gemm256.hip): the same operand layouts as launch_lt; C bf16
// [M][N] (+ bias) with G = gelu_tanh(C) when G is given (forward fc), or fp32 slabs [splitk][M][N]
// (out_f32). M, N multiples of 128 (a half-outside last tile is clamped), K of 64 * splitk.
bool supported256(int M, int N, int K, int splitk);
hipError_t launch_g256(const void* A, int lda, bool a_mn, const void* B, int ldb, bool b_mn, const void* bias, void* C,
                       void* G, bool out_f32, int splitk, int M, int N, int K, hipStream_t st);
// measurement only (wrong results): 1 no DMA in the K loop, 2 no fragment reads, 3 neither, 4 no stagger
hipError_t launch_g256_ablate(const void* A, const void* B, void* C, int M, int N, int K, int variant, hipStream_t st);

}  // namespace gemm
}  // namespace katib_hip
