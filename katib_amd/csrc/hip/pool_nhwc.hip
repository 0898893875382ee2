// NHWC bf16 pooling for the ENAS child network's `reduction` op (reference
// examples/v1beta1/trial-images/enas-cnn-cifar10/op_library.py:127-150: Keras MaxPooling2D /
// AveragePooling2D, pool P, stride S, padding 'valid'), forward and backward, so the child's
// train step has no MIOpen pooling (and no PyTorch kernel) left in its captured graph.
//
// One thread per (pixel, 8-channel group): every tap is one 16-byte load of 8 bf16 channels, so a
// wave reads 64 consecutive channel groups of consecutive pixels (fully coalesced in NHWC).
//   forward : y = max / mean over the P x P window; max also stores the winning tap (uint8, the
//             first maximum in row-major order, as torch.max_pool2d) per output element;
//   backward: each input pixel GATHERS from the outputs whose window covers it (no atomics,
//             every input element written exactly once, zeros where no window reaches).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cmath>
#include <cstdint>

#include "pool_nhwc.h"

namespace katib_hip {
namespace poolnhwc {

namespace {

struct alignas(16) BF8 {
  __hip_bfloat16 v[8];
};
struct alignas(8) U8x8 {
  unsigned char v[8];
};

template <bool MAX>
__global__ void __launch_bounds__(256) pool_fwd_kernel(Geom g, const BF8* __restrict__ x, BF8* __restrict__ y,
                                                       U8x8* __restrict__ arg) {
  const int CG = g.C / 8;
  const int64_t total = (int64_t)g.N * g.OH * g.OW * CG;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int cg = (int)(t % CG);
    int64_t r = t / CG;
    const int ox = (int)(r % g.OW);
    r /= g.OW;
    const int oy = (int)(r % g.OH);
    const int n = (int)(r / g.OH);
    float acc[8];
    unsigned char am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[j] = MAX ? -INFINITY : 0.f;
      am[j] = 0;
    }
    for (int ky = 0; ky < g.P; ++ky) {
      const int iy = oy * g.S + ky;
      for (int kx = 0; kx < g.P; ++kx) {
        const int ix = ox * g.S + kx;
        const BF8 v = x[(((int64_t)n * g.H + iy) * g.W + ix) * CG + cg];
        const unsigned char tap = (unsigned char)(ky * g.P + kx);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = __bfloat162float(v.v[j]);
          if (MAX) {
            if (f > acc[j] || (f != f && acc[j] == acc[j])) {
              acc[j] = f;
              am[j] = tap;
            }
          } else {
            acc[j] += f;
          }
        }
      }
    }
    BF8 o;
    const float inv = 1.f / (float)(g.P * g.P);
#pragma unroll
    for (int j = 0; j < 8; ++j) o.v[j] = __float2bfloat16(MAX ? acc[j] : acc[j] * inv);
    y[t] = o;
    if (MAX) {
      U8x8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) a.v[j] = am[j];
      arg[t] = a;
    }
  }
}

template <bool MAX>
__global__ void __launch_bounds__(256) pool_bwd_kernel(Geom g, const BF8* __restrict__ gy,
                                                       const U8x8* __restrict__ arg, BF8* __restrict__ gx) {
  const int CG = g.C / 8;
  const int64_t total = (int64_t)g.N * g.H * g.W * CG;
  const float inv = 1.f / (float)(g.P * g.P);
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int cg = (int)(t % CG);
    int64_t r = t / CG;
    const int ix = (int)(r % g.W);
    r /= g.W;
    const int iy = (int)(r % g.H);
    const int n = (int)(r / g.H);
    // outputs whose window [o*S, o*S + P) contains the pixel
    const int oy0 = iy - g.P + 1 <= 0 ? 0 : (iy - g.P + 1 + g.S - 1) / g.S, oy1 = min(iy / g.S, g.OH - 1);
    const int ox0 = ix - g.P + 1 <= 0 ? 0 : (ix - g.P + 1 + g.S - 1) / g.S, ox1 = min(ix / g.S, g.OW - 1);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int64_t o = (((int64_t)n * g.OH + oy) * g.OW + ox) * CG + cg;
        const BF8 v = gy[o];
        if (MAX) {
          const U8x8 a = arg[o];
          const unsigned char tap = (unsigned char)((iy - oy * g.S) * g.P + (ix - ox * g.S));
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (a.v[j] == tap) acc[j] += __bfloat162float(v.v[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += __bfloat162float(v.v[j]) * inv;
        }
      }
    BF8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out.v[j] = __float2bfloat16(acc[j]);
    gx[t] = out;
  }
}

int blocks_for(int64_t items) {
  const int64_t b = (items + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

hipError_t launch_fwd(const Geom& g, bool is_max, const void* x, void* y, void* arg, hipStream_t st) {
  const int64_t items = (int64_t)g.N * g.OH * g.OW * (g.C / 8);
  if (is_max)
    hipLaunchKernelGGL(pool_fwd_kernel<true>, dim3(blocks_for(items)), dim3(256), 0, st, g,
                       static_cast<const BF8*>(x), static_cast<BF8*>(y), static_cast<U8x8*>(arg));
  else
    hipLaunchKernelGGL(pool_fwd_kernel<false>, dim3(blocks_for(items)), dim3(256), 0, st, g,
                       static_cast<const BF8*>(x), static_cast<BF8*>(y), nullptr);
  return hipGetLastError();
}

hipError_t launch_bwd(const Geom& g, bool is_max, const void* gy, const void* arg, void* gx, hipStream_t st) {
  const int64_t items = (int64_t)g.N * g.H * g.W * (g.C / 8);
  if (is_max)
    hipLaunchKernelGGL(pool_bwd_kernel<true>, dim3(blocks_for(items)), dim3(256), 0, st, g,
                       static_cast<const BF8*>(gy), static_cast<const U8x8*>(arg), static_cast<BF8*>(gx));
  else
    hipLaunchKernelGGL(pool_bwd_kernel<false>, dim3(blocks_for(items)), dim3(256), 0, st, g,
                       static_cast<const BF8*>(gy), nullptr, static_cast<BF8*>(gx));
  return hipGetLastError();
}

}  // namespace poolnhwc
}  // namespace katib_hip
