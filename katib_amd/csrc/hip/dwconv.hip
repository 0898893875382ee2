// Depthwise 2-D convolution for the ENAS child networks: NHWC bf16 activations, fp32 weights
// ([K*K][Co] tap-major on the device) and fp32 accumulation.
//
// Every thread owns 8 consecutive channels of one pixel, so each tap is one 16-byte bf16 load
// (8 B at depth multiplier 2, where 8 output channels read 4 input channels) and two 16-byte
// weight loads that the whole wave reads as one contiguous 512-byte row of the tap; the taps'
// input pixels of neighbouring threads overlap, which L1/L2 serve. TF 'same' padding is the
// (pt, pl) offset plus bounds checks in the gathers. The weight gradient is a per-workgroup
// partial over a band of output rows, written without atomics and summed by the caller.
#include "dwconv.h"

#include <algorithm>

namespace katib_hip {
namespace dwconv {

namespace {

__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  f[0] = bf_lo(v.x), f[1] = bf_hi(v.x), f[2] = bf_lo(v.y), f[3] = bf_hi(v.y);
  f[4] = bf_lo(v.z), f[5] = bf_hi(v.z), f[6] = bf_lo(v.w), f[7] = bf_hi(v.w);
}

__device__ __forceinline__ unsigned short to_bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);  // round to nearest even, NaN preserved
  return *reinterpret_cast<unsigned short*>(&b);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = to_bf(f[0]) | ((unsigned)to_bf(f[1]) << 16);
  v.y = to_bf(f[2]) | ((unsigned)to_bf(f[3]) << 16);
  v.z = to_bf(f[4]) | ((unsigned)to_bf(f[5]) << 16);
  v.w = to_bf(f[6]) | ((unsigned)to_bf(f[7]) << 16);
  return v;
}

// 8 input channels' worth of activations feeding output channels [o0, o0 + 8)
template <int DM>
__device__ __forceinline__ void load_in8(const __hip_bfloat16* p, float* xv) {
  if (DM == 1) {
    unpack8(*reinterpret_cast<const uint4*>(p), xv);
  } else {  // 4 input channels, each feeding two consecutive output channels
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    xv[0] = xv[1] = bf_lo(v.x);
    xv[2] = xv[3] = bf_hi(v.x);
    xv[4] = xv[5] = bf_lo(v.y);
    xv[6] = xv[7] = bf_hi(v.y);
  }
}

template <int K, int DM>
__global__ void __launch_bounds__(256) dw_fwd_kernel(Geom g, const __hip_bfloat16* __restrict__ x,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     __hip_bfloat16* __restrict__ y) {
  // thread = (4 consecutive output pixels of a row, 8 channels): each tap's 8 weights are
  // loaded once for the 4 pixels
  constexpr int PX = 4;
  const int Co = g.C * DM, G = Co / 8, QW = (g.OW + PX - 1) / PX;
  const long total = (long)g.N * g.OH * QW * G;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int gg = (int)(idx % G);
    long p = idx / G;
    const int ox0 = (int)(p % QW) * PX;
    p /= QW;
    const int oy = (int)(p % g.OH), n = (int)(p / g.OH);
    const int o0 = gg * 8, c0 = o0 / DM;
    float acc[PX][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float b0 = bias ? bias[o0 + j] : 0.f;
#pragma unroll
      for (int q = 0; q < PX; ++q) acc[q][j] = b0;
    }
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int iy = oy * g.S - g.pt + ky;
      if (iy < 0 || iy >= g.H) continue;
      const __hip_bfloat16* xrow = x + (((long)n * g.H + iy) * g.W) * g.C + c0;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const float4* wt = reinterpret_cast<const float4*>(w + (ky * K + kx) * Co + o0);
        const float4 wa = wt[0], wb = wt[1];
        const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
        for (int q = 0; q < PX; ++q) {
          const int ix = (ox0 + q) * g.S - g.pl + kx;
          if (ox0 + q >= g.OW || ix < 0 || ix >= g.W) continue;
          float xv[8];
          load_in8<DM>(xrow + (long)ix * g.C, xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[q][j] += xv[j] * wv[j];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PX; ++q)
      if (ox0 + q < g.OW)
        *reinterpret_cast<uint4*>(y + (((long)n * g.OH + oy) * g.OW + ox0 + q) * Co + o0) = pack8(acc[q]);
  }
}

template <int K, int DM>
__global__ void __launch_bounds__(256) dw_dgrad_kernel(Geom g, const __hip_bfloat16* __restrict__ gy,
                                                       const float* __restrict__ w, __hip_bfloat16* __restrict__ gx) {
  const int Co = g.C * DM, G = g.C / 8;
  const long total = (long)g.N * g.H * g.W * G;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int gg = (int)(idx % G);
    long p = idx / G;
    const int ix = (int)(p % g.W);
    p /= g.W;
    const int iy = (int)(p % g.H), n = (int)(p / g.H);
    const int c0 = gg * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int ty = iy + g.pt - ky;
      if (ty < 0 || ty % g.S) continue;
      const int oy = ty / g.S;
      if (oy >= g.OH) continue;
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        const int tx = ix + g.pl - kx;
        if (tx < 0 || tx % g.S) continue;
        const int ox = tx / g.S;
        if (ox >= g.OW) continue;
        const __hip_bfloat16* src = gy + (((long)n * g.OH + oy) * g.OW + ox) * Co + c0 * DM;
        const float* wt = w + (ky * K + kx) * Co + c0 * DM;
#pragma unroll
        for (int h = 0; h < DM; ++h) {  // output channels c0*DM + [8h, 8h + 8)
          float gv[8];
          unpack8(*reinterpret_cast<const uint4*>(src + 8 * h), gv);
          const float4 wa = reinterpret_cast<const float4*>(wt + 8 * h)[0];
          const float4 wb = reinterpret_cast<const float4*>(wt + 8 * h)[1];
          const float prod[8] = {gv[0] * wa.x, gv[1] * wa.y, gv[2] * wa.z, gv[3] * wa.w,
                                 gv[4] * wb.x, gv[5] * wb.y, gv[6] * wb.z, gv[7] * wb.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[(8 * h + j) / DM] += prod[j];
        }
      }
    }
    *reinterpret_cast<uint4*>(gx + (((long)n * g.H + iy) * g.W + ix) * g.C + c0) = pack8(acc);
  }
}

// one workgroup per band of output rows (flattened n*OH + oy); job = (channel group, tap):
// acc[8] over the band's pixels, one partial row per workgroup. (A (channel group, kernel row)
// job with K column accumulators reads gy once per K taps but leaves most threads idle at these
// channel counts: measured 2x slower at K = 5.)
template <int K, int DM>
__global__ void __launch_bounds__(256) dw_wgrad_kernel(Geom g, const __hip_bfloat16* __restrict__ x,
                                                       const __hip_bfloat16* __restrict__ gy,
                                                       float* __restrict__ part, int rows_per_block) {
  const int Co = g.C * DM, G = Co / 8, KK = K * K;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(g.N * g.OH, r0 + rows_per_block);
  float* out = part + (long)blockIdx.x * Co * KK;
  for (int job = threadIdx.x; job < G * KK; job += 256) {
    const int gg = job % G, tap = job / G, ky = tap / K, kx = tap - ky * K;
    const int o0 = gg * 8, c0 = o0 / DM;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = r0; r < r1; ++r) {
      const int n = r / g.OH, oy = r - n * g.OH, iy = oy * g.S - g.pt + ky;
      if (iy < 0 || iy >= g.H) continue;
      const __hip_bfloat16* gyr = gy + ((long)r * g.OW) * Co + o0;
      const __hip_bfloat16* xr = x + (((long)n * g.H + iy) * g.W) * g.C + c0;
      for (int ox = 0; ox < g.OW; ++ox) {
        const int ix = ox * g.S - g.pl + kx;
        if (ix < 0 || ix >= g.W) continue;
        float gv[8], xv[8];
        unpack8(*reinterpret_cast<const uint4*>(gyr + (long)ox * Co), gv);
        load_in8<DM>(xr + (long)ix * g.C, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += gv[j] * xv[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) out[(o0 + j) * KK + tap] = acc[j];
  }
}

int grid_for(long total) { return (int)std::max<long>(1, std::min<long>((total + 255) / 256, 8192)); }

}  // namespace

int wgrad_rows(const Geom& g) {
  // ~16 MB of fp32 partials at most, between 32 and 1024 workgroups
  const long per = (long)g.C * g.DM * g.K * g.K * 4;
  const int want = (int)std::max<long>(32, std::min<long>(1024, (16l << 20) / std::max<long>(per, 1)));
  const int rows = g.N * g.OH;
  const int rpb = (rows + want - 1) / want;
  return (rows + rpb - 1) / rpb;
}

#define KATIB_DW_DISPATCH(KER, ...)                                                   \
  switch (g.K * 10 + g.DM) {                                                          \
    case 31: hipLaunchKernelGGL((KER<3, 1>), __VA_ARGS__); break;                     \
    case 32: hipLaunchKernelGGL((KER<3, 2>), __VA_ARGS__); break;                     \
    case 51: hipLaunchKernelGGL((KER<5, 1>), __VA_ARGS__); break;                     \
    case 52: hipLaunchKernelGGL((KER<5, 2>), __VA_ARGS__); break;                     \
    case 71: hipLaunchKernelGGL((KER<7, 1>), __VA_ARGS__); break;                     \
    case 72: hipLaunchKernelGGL((KER<7, 2>), __VA_ARGS__); break;                     \
    default: return hipErrorInvalidValue;                                             \
  }

hipError_t launch_fwd(const Geom& g, const __hip_bfloat16* x, const float* w, const float* bias, __hip_bfloat16* y,
                      hipStream_t st) {
  const long total = (long)g.N * g.OH * ((g.OW + 3) / 4) * (g.C * g.DM / 8);
  KATIB_DW_DISPATCH(dw_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, g, x, w, bias, y)
  return hipGetLastError();
}

hipError_t launch_dgrad(const Geom& g, const __hip_bfloat16* gy, const float* w, __hip_bfloat16* gx, hipStream_t st) {
  const long total = (long)g.N * g.H * g.W * (g.C / 8);
  KATIB_DW_DISPATCH(dw_dgrad_kernel, dim3(grid_for(total)), dim3(256), 0, st, g, gy, w, gx)
  return hipGetLastError();
}

hipError_t launch_wgrad(const Geom& g, const __hip_bfloat16* x, const __hip_bfloat16* gy, float* gw_part, int rows,
                        hipStream_t st) {
  const int nrows = g.N * g.OH, rpb = (nrows + rows - 1) / rows;
  KATIB_DW_DISPATCH(dw_wgrad_kernel, dim3(rows), dim3(256), 0, st, g, x, gy, gw_part, rpb)
  return hipGetLastError();
}

}  // namespace dwconv
}  // namespace katib_hip
