// Implicit-GEMM convolution on MFMA (bf16 in, fp32 accumulate), NHWC activations.
// Used by the ResNet-18 trial (HyperBand config) and the ENAS child networks
// (SURVEY §2.13 K1/K20 and the ResNet-18 "new scope" row). See conv_igemm.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdint>

namespace katib_hip {
namespace conv {

struct ConvGeom {
  int N, H, W, C;       // input  (NHWC)
  int K, R, S;          // filters [K][R][S][C]
  int OH, OW;           // output (NHWC, K channels)
  int sh, sw, ph, pw, dh, dw;
};

// y[N*OH*OW][K] = conv(x, w), x [N*H*W][C], w [K][R*S*C]; C % 8 == 0.
// out_f32 != nullptr: fp32 output instead of bf16 (y ignored).
hipError_t launch_fwd(const ConvGeom& g, const __hip_bfloat16* x, const __hip_bfloat16* w, __hip_bfloat16* y,
                      float* out_f32, hipStream_t stream);
// dx[N*H*W][C] = conv_transpose(dy, w); wt = w transposed to [C][R*S*K]; K % 8 == 0.
// add_d != nullptr: the epilogue adds a second gradient of x ([N*H*W][C] bf16) - the residual
// branch of a ResNet block - masked by add_y > 0 when add_y != nullptr (the ReLU after the add),
// so the two branch gradients meet in one store instead of an extra add pass.
hipError_t launch_dgrad(const ConvGeom& g, const __hip_bfloat16* dy, const __hip_bfloat16* wt, __hip_bfloat16* dx,
                        hipStream_t stream, const __hip_bfloat16* add_d = nullptr,
                        const __hip_bfloat16* add_y = nullptr);
// dw32[K][R*S*C] += sum over output pixels dy (x) im2col(x); dw32 must be zeroed by the caller.
hipError_t launch_wgrad(const ConvGeom& g, const __hip_bfloat16* x, const __hip_bfloat16* dy, float* dw32,
                        hipStream_t stream);

}  // namespace conv
}  // namespace katib_hip
