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
hipError_t launch_dgrad(const ConvGeom& g, const __hip_bfloat16* dy, const __hip_bfloat16* wt, __hip_bfloat16* dx,
                        hipStream_t stream);
// dw32[K][R*S*C] += sum over output pixels dy (x) im2col(x); dw32 must be zeroed by the caller.
hipError_t launch_wgrad(const ConvGeom& g, const __hip_bfloat16* x, const __hip_bfloat16* dy, float* dw32,
                        hipStream_t stream);

}  // namespace conv
}  // namespace katib_hip
