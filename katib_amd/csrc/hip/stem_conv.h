// Direct 3x3 / pad-1 / stride-1 convolution for the DARTS stem (few input channels,
// fp32 NCHW): forward and weight gradient. See stem_conv.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace katib_hip {
namespace stem {

constexpr int kMaxCout = 64;  // LDS weight slab: kMaxCout * 9 * CIN floats

// y[N][Cout][H][W] = conv3x3(x[N][Cin][H][W], w[Cout][Cin][3][3]), zero padding 1.
void launch_fwd(const float* x, const float* w, float* y, int N, int Cin, int Cout, int H, int W, hipStream_t s);

// dw[Cout][Cin][3][3] = sum_{n,h,w} dy[n][co][h][w] * x[n][ci][h+kh-1][w+kw-1].
// `partial` holds chunks * Cout * Cin * 9 floats (per-chunk sums, reduced in a fixed order).
void launch_wgrad(const float* x, const float* dy, float* partial, float* dw, int N, int Cin, int Cout, int H, int W,
                  int chunks, hipStream_t s);

}  // namespace stem
}  // namespace katib_hip
