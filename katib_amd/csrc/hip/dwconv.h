// Depthwise 2-D convolution, NHWC bf16 activations, fp32 weights and accumulation
// (ENAS child networks: depthwise_convolution / the depthwise half of separable_convolution,
// reference examples/v1beta1/trial-images/enas-cnn-cifar10/op_library.py:22-155).
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

namespace katib_hip {
namespace dwconv {

struct Geom {
  int N, H, W, C;  // input, C % 8 == 0
  int DM;          // depth multiplier: output channel o reads input channel o / DM (1 or 2)
  int K;           // square kernel, odd, <= 7
  int S;           // stride 1 or 2
  int pt, pl;      // top / left padding (TF 'same' puts the odd pixel bottom / right)
  int OH, OW;
};

// y[n,oy,ox,o] = bias[o] + sum_taps x[n, oy*S - pt + ky, ox*S - pl + kx, o / DM] * w[o][ky*K + kx]
hipError_t launch_fwd(const Geom& g, const __hip_bfloat16* x, const float* w, const float* bias, __hip_bfloat16* y,
                      hipStream_t st);
// gx[n,iy,ix,c] = sum_m sum_taps gy[n,oy,ox,c*DM + m] * w[c*DM + m][tap]  (oy*S = iy + pt - ky)
hipError_t launch_dgrad(const Geom& g, const __hip_bfloat16* gy, const float* w, __hip_bfloat16* gx, hipStream_t st);
// gw_part[b][o][tap]: per-workgroup partial sums over the workgroup's output rows; the caller
// sums the rows (deterministic, no float atomics). Returns the number of partial rows in *rows.
hipError_t launch_wgrad(const Geom& g, const __hip_bfloat16* x, const __hip_bfloat16* gy, float* gw_part, int rows,
                        hipStream_t st);
int wgrad_rows(const Geom& g);

}  // namespace dwconv
}  // namespace katib_hip
