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

// Stem BatchNorm (affine, training) fused into the convolution kernels:
// forward: the conv also accumulates per-channel (sum, sum of squares) of y into kRep fp64
// replicas stats[r][2*Cout] (replica = workgroup % kRep; folded by the caller before use).
void launch_fwd_stats(const float* x, const float* w, float* y, double* stats, int N, int Cin, int Cout, int H, int W,
                      hipStream_t s);

// weight gradient through the BN backward: dy is the gradient of the BN OUTPUT; per element the
// kernel forms dz = gamma istd (dy - S1/M - zhat S2/M), zhat = (z - mean) istd, from the folded
// reductions red = (S1 = sum dy, S2 = sum dy zhat) and the folded forward statistics; dgamma += S2
// and dbeta += S1 (single writer per channel) when the pointers are given.
struct BnBwd {
  const float* z;        // conv output (pre-BN) [N][Cout][H][W]
  const double* red;     // folded [S1[Cout], S2[Cout]]
  const double* stats;   // folded [sum[Cout], sumsq[Cout]]
  const float* gamma;
  float inv_count;       // 1 / (N H W)
  float eps;
  float* dgamma;         // nullable
  float* dbeta;          // nullable
  float red_scale;       // 1, or 1 / world under SyncBN (red then sums every rank's dy: d gamma / d beta stay per rank)
};
// accumulate: dw += the weight gradient (a registered gradient row) instead of dw =
void launch_wgrad_bn(const float* x, const float* dy, const BnBwd& bn, float* partial, float* dw, int N, int Cin,
                     int Cout, int H, int W, int chunks, hipStream_t s, bool accumulate = false);

}  // namespace stem
}  // namespace katib_hip
