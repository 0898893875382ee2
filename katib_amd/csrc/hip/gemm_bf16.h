// bf16 NT GEMM with fused bias / bias + GELU epilogue (gemm_bf16.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {
namespace gemm {

bool supported(int M, int N, int K);  // M, N multiples of 128, K of 64
// C[M][N] = A[M][K] W[N][K]^T (+ bias[N]); G != nullptr: C = pre-activation, G = gelu_tanh(C)
hipError_t launch_nt(const void* A, const void* W, const void* bias, void* C, void* G, int M, int N, int K,
                     hipStream_t st);

}  // namespace gemm
}  // namespace katib_hip
