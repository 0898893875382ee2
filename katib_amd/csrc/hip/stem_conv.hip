// DARTS stem convolution (model.py:90-93 in the reference's darts-cnn-cifar10 trial:
// Conv2d(3, C_stem, 3, padding=1, bias=False)) as two direct kernels for gfx950.
//
// With 3 input channels the conv is a K=27 reduction - far too thin for MFMA tiles and
// a poor fit for the library's fp32 Winograd kernels (0.43 ms / 5 ms launches in eager
// traces, plus find-mode tuning on first use). Both directions are HBM-bound here
// (measured: forward 7 us, weight gradient 17 us on 128x3x32x32 -> 4 channels):
//   forward: one thread per output pixel keeps its 27-value input patch in registers
//            and sweeps every output channel against a weight slab broadcast from LDS;
//            stores are coalesced along W for each output plane.
//   wgrad:   grid (pixel chunk, output channel); each thread accumulates the 27 partial
//            products of its pixels in registers, a 64-lane shuffle tree + LDS folds the
//            4 waves, and a second launch (one wave per weight) sums the chunk partials in a fixed order
//            (deterministic, no float atomics).
// The input image never needs a gradient, so there is no data-gradient kernel.
#include "darts_ops.h"  // kRep
#include "stem_conv.h"

namespace katib_hip {
namespace stem {
namespace {

constexpr int kThreads = 256;

template <int CIN>
__device__ __forceinline__ void load_patch(const float* __restrict__ x, int n, int h, int w, int H, int W,
                                           float (&v)[CIN * 9]) {
#pragma unroll
  for (int ci = 0; ci < CIN; ++ci) {
    const float* plane = x + ((size_t)n * CIN + ci) * H * W;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int hh = h + kh - 1;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ww = w + kw - 1;
        const bool in = hh >= 0 && hh < H && ww >= 0 && ww < W;
        v[ci * 9 + kh * 3 + kw] = in ? plane[hh * W + ww] : 0.f;
      }
    }
  }
}

template <int CIN>
__global__ __launch_bounds__(kThreads) void stem_fwd_kernel(const float* __restrict__ x, const float* __restrict__ wt,
                                                             float* __restrict__ y, int N, int Cout, int H, int W) {
  __shared__ float ws[kMaxCout * CIN * 9];
  for (int i = threadIdx.x; i < Cout * CIN * 9; i += kThreads) ws[i] = wt[i];
  __syncthreads();
  const int HW = H * W;
  const int p = blockIdx.x * kThreads + threadIdx.x;
  if (p >= N * HW) return;
  const int n = p / HW, r = p - n * HW, h = r / W, w = r - (r / W) * W;
  float v[CIN * 9];
  load_patch<CIN>(x, n, h, w, H, W, v);
  float* out = y + (size_t)n * Cout * HW + r;
  for (int co = 0; co < Cout; ++co) {
    const float* wc = ws + co * CIN * 9;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k) acc = fmaf(wc[k], v[k], acc);
    out[(size_t)co * HW] = acc;
  }
}

__device__ __forceinline__ float wsum64(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// forward + BN statistics: every thread of the grid takes part in the per-channel wave sums
// (out-of-range pixels contribute zeros), waves fold into LDS, the workgroup into replica
// blockIdx.x % kRep of stats[kRep][2*Cout] = (sum, sum of squares).
template <int CIN>
__global__ __launch_bounds__(kThreads) void stem_fwd_stats_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ wt,
                                                                   float* __restrict__ y, double* __restrict__ stats,
                                                                   int N, int Cout, int H, int W) {
  __shared__ float ws[kMaxCout * CIN * 9];
  __shared__ float st[2 * kMaxCout];
  for (int i = threadIdx.x; i < Cout * CIN * 9; i += kThreads) ws[i] = wt[i];
  for (int i = threadIdx.x; i < 2 * Cout; i += kThreads) st[i] = 0.f;
  __syncthreads();
  const int HW = H * W;
  const int p = blockIdx.x * kThreads + threadIdx.x;
  const bool valid = p < N * HW;
  const int q = valid ? p : 0;
  const int n = q / HW, r = q - n * HW, h = r / W, w = r - (r / W) * W;
  float v[CIN * 9];
  load_patch<CIN>(x, n, h, w, H, W, v);
  float* out = y + (size_t)n * Cout * HW + r;
  const int lane = threadIdx.x & 63;
  for (int co = 0; co < Cout; ++co) {
    const float* wc = ws + co * CIN * 9;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < CIN * 9; ++k) acc = fmaf(wc[k], v[k], acc);
    if (valid) out[(size_t)co * HW] = acc;
    const float a = valid ? acc : 0.f;
    const float s1 = wsum64(a), s2 = wsum64(a * a);
    if (lane == 0) {
      atomicAdd(&st[co], s1);
      atomicAdd(&st[Cout + co], s2);
    }
  }
  __syncthreads();
  double* rep = stats + (size_t)(blockIdx.x % kRep) * 2 * Cout;
  for (int i = threadIdx.x; i < 2 * Cout; i += kThreads) atomicAdd(rep + i, (double)st[i]);
}

template <int CIN, bool BN>
__global__ __launch_bounds__(kThreads) void stem_wgrad_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ dy, BnBwd bn,
                                                               float* __restrict__ partial, int N, int Cout, int H,
                                                               int W, int per_chunk) {
  constexpr int K = CIN * 9;
  __shared__ float red[kThreads / 64][K];
  const int co = blockIdx.y, HW = H * W, P = N * HW;
  const int p0 = blockIdx.x * per_chunk, p1 = min(P, p0 + per_chunk);
  // BN backward coefficients: dz = k1 * (dy - m1 - zhat * m2), zhat = (z - mean) * istd
  float mean = 0.f, istd = 0.f, k1 = 1.f, m1 = 0.f, m2 = 0.f;
  if (BN) {
    const double m = bn.stats[co] * (double)bn.inv_count;
    double var = bn.stats[Cout + co] * (double)bn.inv_count - m * m;
    if (var < 0) var = 0;
    mean = (float)m;
    istd = rsqrtf((float)var + bn.eps);
    k1 = bn.gamma[co] * istd;
    m1 = (float)(bn.red[co] * (double)bn.inv_count);
    m2 = (float)(bn.red[Cout + co] * (double)bn.inv_count);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (bn.dgamma) bn.dgamma[co] += (float)(bn.red[Cout + co] * (double)bn.red_scale);
      if (bn.dbeta) bn.dbeta[co] += (float)(bn.red[co] * (double)bn.red_scale);
    }
  }
  float acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0.f;
  for (int p = p0 + threadIdx.x; p < p1; p += kThreads) {
    const int n = p / HW, r = p - n * HW, h = r / W, w = r - (r / W) * W;
    const size_t idx = ((size_t)n * Cout + co) * HW + r;
    float d = dy[idx];
    if (BN) d = k1 * (d - m1 - (bn.z[idx] - mean) * istd * m2);
    float v[K];
    load_patch<CIN>(x, n, h, w, H, W, v);
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = fmaf(d, v[k], acc[k]);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float s = acc[k];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) red[wave][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) s += red[i][threadIdx.x];
    partial[((size_t)blockIdx.x * Cout + co) * K + threadIdx.x] = s;
  }
}

// one wave per weight element: lanes stride over the chunk partials, then a shuffle tree
// (fixed order for a given chunk count -> deterministic)
__global__ __launch_bounds__(64) void chunk_sum_kernel(const float* __restrict__ partial, float* __restrict__ out,
                                                        int n, int chunks, int accumulate) {
  const int i = blockIdx.x;
  float s = 0.f;
  for (int c = threadIdx.x; c < chunks; c += 64) s += partial[(size_t)c * n + i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (threadIdx.x == 0) out[i] = accumulate ? out[i] + s : s;  // accumulate: into a gradient row
}

}  // namespace

void launch_fwd(const float* x, const float* w, float* y, int N, int Cin, int Cout, int H, int W, hipStream_t s) {
  const int blocks = (N * H * W + kThreads - 1) / kThreads;
  if (Cin == 3)
    hipLaunchKernelGGL(stem_fwd_kernel<3>, dim3(blocks), dim3(kThreads), 0, s, x, w, y, N, Cout, H, W);
  else
    hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(blocks), dim3(kThreads), 0, s, x, w, y, N, Cout, H, W);
}

namespace {

template <bool BN>
void wgrad_impl(const float* x, const float* dy, const BnBwd& bn, float* partial, float* dw, int N, int Cin, int Cout,
                int H, int W, int chunks, hipStream_t s, bool accumulate = false) {
  const int P = N * H * W;
  const int per_chunk = (P + chunks - 1) / chunks;
  if (Cin == 3)
    hipLaunchKernelGGL((stem_wgrad_kernel<3, BN>), dim3(chunks, Cout), dim3(kThreads), 0, s, x, dy, bn, partial, N,
                       Cout, H, W, per_chunk);
  else
    hipLaunchKernelGGL((stem_wgrad_kernel<1, BN>), dim3(chunks, Cout), dim3(kThreads), 0, s, x, dy, bn, partial, N,
                       Cout, H, W, per_chunk);
  const int n = Cout * Cin * 9;
  hipLaunchKernelGGL(chunk_sum_kernel, dim3(n), dim3(64), 0, s, partial, dw, n, chunks, accumulate ? 1 : 0);
}

}  // namespace

void launch_wgrad(const float* x, const float* dy, float* partial, float* dw, int N, int Cin, int Cout, int H, int W,
                  int chunks, hipStream_t s) {
  wgrad_impl<false>(x, dy, BnBwd{}, partial, dw, N, Cin, Cout, H, W, chunks, s);
}

void launch_wgrad_bn(const float* x, const float* dy, const BnBwd& bn, float* partial, float* dw, int N, int Cin,
                     int Cout, int H, int W, int chunks, hipStream_t s, bool accumulate) {
  wgrad_impl<true>(x, dy, bn, partial, dw, N, Cin, Cout, H, W, chunks, s, accumulate);
}

void launch_fwd_stats(const float* x, const float* w, float* y, double* stats, int N, int Cin, int Cout, int H, int W,
                      hipStream_t s) {
  const int blocks = (N * H * W + kThreads - 1) / kThreads;
  if (Cin == 3)
    hipLaunchKernelGGL(stem_fwd_stats_kernel<3>, dim3(blocks), dim3(kThreads), 0, s, x, w, y, stats, N, Cout, H, W);
  else
    hipLaunchKernelGGL(stem_fwd_stats_kernel<1>, dim3(blocks), dim3(kThreads), 0, s, x, w, y, stats, N, Cout, H, W);
}

}  // namespace stem
}  // namespace katib_hip
