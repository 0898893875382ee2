// BatchNorm (+ residual add + ReLU) for NHWC bf16 activations on gfx950.
//
// The ResNet-18 trial (BASELINE config 3) spent ~45 % of its GPU time in MIOpen's NCHW-
// oriented batch-norm kernels on channels-last bf16 tensors (profiles/resnet_torch_baseline_
// kernel_stats.txt: FwdTrainSpatialNorm, BwdSpatialDX, BwdSpatialDScaleDBias, and an
// inference kernel at 385 us per call). A BN over [P = N*H*W, C] rows is two streaming
// passes, so the kernels here are built for HBM bandwidth:
//
//  fwd   stats    per-channel sum / sum of squares, 16-byte loads, fp32 partials per row chunk
//        finalize mean, 1/std, running-stat update (unbiased var), folded scale/shift
//        apply    y = relu(x * scale + shift [+ residual])           (one read, one write)
//  bwd   stats    sum g and sum g*xhat, g = dy * [y > 0]             (ReLU mask from the output)
//        finalize dgamma, dbeta and the three dx coefficients
//        apply    dx = scale * (g - mean(g) - xhat * mean(g xhat)); dres = g
//
// Channel counts are multiples of 8 (16-byte vectors of 8 bf16).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "batchnorm.h"

namespace katib_hip {
namespace bn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16;

__device__ __forceinline__ float lo2f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi2f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }
__device__ __forceinline__ void unpack8(const u32x4& q, float* v) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = lo2f(q[k]);
    v[2 * k + 1] = hi2f(q[k]);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* v) {
  return u32x4{pack2(v[0], v[1]), pack2(v[2], v[3]), pack2(v[4], v[5]), pack2(v[6], v[7])};
}

// Partial per-channel sums over a chunk of rows. Block: cvb column vectors (8 channels) x
// (256 / cvb) row groups. MODE 0: (sum x, sum x^2). MODE 1: (sum g, sum g * xhat) with
// g = dy masked by y > 0 when y != nullptr.
template <int MODE>
__global__ __launch_bounds__(256) void stats_k(const u16* __restrict__ x, const u16* __restrict__ dy,
                                               const u16* __restrict__ y, const float* __restrict__ mean,
                                               const float* __restrict__ invstd, int P, int C, int rows, int cvb,
                                               float* __restrict__ part) {
  __shared__ float red[256 * 16];  // [row group][cvb][16]
  const int tx = threadIdx.x % cvb, ty = threadIdx.x / cvb, rg = 256 / cvb;
  const int cv = blockIdx.x * cvb + tx, c0 = cv * 8;
  const int r0 = blockIdx.y * rows, r1 = min(P, r0 + rows);
  float a[8], b[8], mu[8], is[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = b[e] = 0.f;
  const bool active = ty < rg && c0 < C;
  if (active) {
    if (MODE == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        mu[e] = mean[c0 + e];
        is[e] = invstd[c0 + e];
      }
    }
    for (int r = r0 + ty; r < r1; r += rg) {
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(x + (int64_t)r * C + c0), v);
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a[e] += v[e];
          b[e] += v[e] * v[e];
        }
      } else {
        float g[8];
        unpack8(*reinterpret_cast<const u32x4*>(dy + (int64_t)r * C + c0), g);
        if (y) {
          float yy[8];
          unpack8(*reinterpret_cast<const u32x4*>(y + (int64_t)r * C + c0), yy);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = yy[e] > 0.f ? g[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          a[e] += g[e];
          b[e] += g[e] * (v[e] - mu[e]) * is[e];
        }
      }
    }
  }
  if (ty < rg) {
    float* o = red + (ty * cvb + tx) * 16;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = a[e];
      o[8 + e] = b[e];
    }
  }
  __syncthreads();
  // one thread per (column vector, value): cvb * 16 <= 256
  if (threadIdx.x < cvb * 16) {
    const int c = threadIdx.x >> 4, k = threadIdx.x & 15;
    float s = 0.f;
    for (int t = 0; t < rg; ++t) s += red[(t * cvb + c) * 16 + k];
    const int ch = (blockIdx.x * cvb + c) * 8 + (k & 7);
    if (ch < C) part[((int64_t)blockIdx.y * 2 + (k >> 3)) * C + ch] = s;
  }
}

// Sum the R partial rows of (a, b) per channel: block = 64 channels x 4 row groups.
__device__ __forceinline__ void sum_parts(const float* __restrict__ part, int R, int C, float& a, float& b,
                                          float (*red)[4][64]) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6, c = blockIdx.x * 64 + tx;
  float s = 0.f, q = 0.f;
  if (c < C) {
#pragma unroll 8
    for (int r = ty; r < R; r += 4) {
      s += part[(int64_t)(2 * r) * C + c];
      q += part[(int64_t)(2 * r + 1) * C + c];
    }
  }
  red[0][ty][tx] = s;
  red[1][ty][tx] = q;
  __syncthreads();
  a = (red[0][0][tx] + red[0][1][tx]) + (red[0][2][tx] + red[0][3][tx]);
  b = (red[1][0][tx] + red[1][1][tx]) + (red[1][2][tx] + red[1][3][tx]);
}

__global__ __launch_bounds__(256) void fwd_finalize_k(const float* __restrict__ part, int R, int C, int P,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      float eps, float momentum, float* __restrict__ rmean,
                                                      float* __restrict__ rvar, float* __restrict__ mean,
                                                      float* __restrict__ invstd, float* __restrict__ ss,
                                                      long long* __restrict__ counter) {
  __shared__ float red[2][4][64];
  float s, q;
  // nn.BatchNorm2d's num_batches_tracked += 1, folded in here instead of its own framework launch
  if (counter != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *counter += 1;
  sum_parts(part, R, C, s, q, red);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (threadIdx.x >= 64 || c >= C) return;
  const float m = s / P;
  const float var = fmaxf(q / P - m * m, 0.f);
  const float is = rsqrtf(var + eps);
  mean[c] = m;
  invstd[c] = is;
  const float sc = gamma[c] * is;
  ss[c] = sc;
  ss[C + c] = beta[c] - m * sc;
  if (rmean) {
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * m;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (P > 1 ? var * P / (P - 1) : var);
  }
}

__global__ __launch_bounds__(256) void sum_finalize_k(const float* __restrict__ part, int R, int C,
                                                      float* __restrict__ out) {
  __shared__ float red[2][4][64];
  float s, q;
  sum_parts(part, R, C, s, q, red);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (threadIdx.x < 64 && c < C) out[c] = s;
}

__global__ void eval_coef_k(const float* __restrict__ rmean, const float* __restrict__ rvar,
                            const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int C,
                            float* __restrict__ ss) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sc = gamma[c] * rsqrtf(rvar[c] + eps);
  ss[c] = sc;
  ss[C + c] = beta[c] - rmean[c] * sc;
}

__global__ __launch_bounds__(256) void apply_k(const u16* __restrict__ x, const u16* __restrict__ res,
                                               u16* __restrict__ y, const float* __restrict__ ss, int64_t n8, int C,
                                               int relu) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int c0 = (int)((i * 8) % C);
    float v[8];
    unpack8(reinterpret_cast<const u32x4*>(x)[i], v);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(ss + c0), s1 = *reinterpret_cast<const f32x4*>(ss + c0 + 4);
    const f32x4 h0 = *reinterpret_cast<const f32x4*>(ss + C + c0), h1 = *reinterpret_cast<const f32x4*>(ss + C + c0 + 4);
    const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (res) unpack8(reinterpret_cast<const u32x4*>(res)[i], r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = v[e] * sc[e] + sh[e] + r[e];
      if (relu) v[e] = fmaxf(v[e], 0.f);
    }
    reinterpret_cast<u32x4*>(y)[i] = pack8(v);
  }
}

__global__ __launch_bounds__(256) void bwd_finalize_k(const float* __restrict__ part, int R, int C, int P,
                                                      const float* __restrict__ gamma,
                                                      const float* __restrict__ invstd, float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta, float* __restrict__ coef,
                                                      int accumulate) {
  __shared__ float red[2][4][64];
  float sg, sgx;
  sum_parts(part, R, C, sg, sgx, red);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  if (threadIdx.x >= 64 || c >= C) return;
  // accumulate: add into persistent gradient buffers (zeroed by the fused optimizer after use)
  dgamma[c] = accumulate ? dgamma[c] + sgx : sgx;
  dbeta[c] = accumulate ? dbeta[c] + sg : sg;
  coef[c] = gamma[c] * invstd[c];
  coef[C + c] = sg / P;
  coef[2 * C + c] = sgx / P;
}

__global__ __launch_bounds__(256) void bwd_apply_k(const u16* __restrict__ dy, const u16* __restrict__ y,
                                                   const u16* __restrict__ x, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd, const float* __restrict__ coef,
                                                   u16* __restrict__ dx, u16* __restrict__ dres, int64_t n8, int C) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int c0 = (int)((i * 8) % C);
    float g[8], v[8];
    unpack8(reinterpret_cast<const u32x4*>(dy)[i], g);
    if (y) {
      float yy[8];
      unpack8(reinterpret_cast<const u32x4*>(y)[i], yy);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = yy[e] > 0.f ? g[e] : 0.f;
    }
    if (dres) reinterpret_cast<u32x4*>(dres)[i] = pack8(g);
    unpack8(reinterpret_cast<const u32x4*>(x)[i], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      const float xh = (v[e] - mean[c]) * invstd[c];
      v[e] = coef[c] * (g[e] - coef[C + c] - xh * coef[2 * C + c]);
    }
    reinterpret_cast<u32x4*>(dx)[i] = pack8(v);
  }
}

inline int ew_grid(int64_t n8) {
  const int64_t b = (n8 + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

void plan(int P, int C, int* R, int* rows, int* cvb) {
  *cvb = C / 8 < 16 ? C / 8 : 16;
  const int cblocks = (C / 8 + *cvb - 1) / *cvb;
  int r = 1024 / cblocks;
  const int rg = 256 / *cvb;
  const int max_r = (P + rg - 1) / rg;  // >= one row per row group
  r = r < 1 ? 1 : (r > 128 ? 128 : r);
  r = r > max_r ? max_r : r;
  *R = r;
  *rows = (P + r - 1) / r;
}

hipError_t fwd_train(const bf16* x, const bf16* res, bf16* y, const float* gamma, const float* beta, float* rmean,
                     float* rvar, float* mean, float* invstd, float* ss, float* part, int P, int C, float eps,
                     float momentum, int relu, hipStream_t st, long long* counter) {
  int R, rows, cvb;
  plan(P, C, &R, &rows, &cvb);
  const u16* xx = reinterpret_cast<const u16*>(x);
  hipLaunchKernelGGL(stats_k<0>, dim3((C / 8 + cvb - 1) / cvb, R), dim3(256), 0, st, xx, nullptr, nullptr, nullptr,
                     nullptr, P, C, rows, cvb, part);
  hipLaunchKernelGGL(fwd_finalize_k, dim3((C + 63) / 64), dim3(256), 0, st, part, R, C, P, gamma, beta, eps,
                     momentum, rmean, rvar, mean, invstd, ss, counter);
  const int64_t n8 = (int64_t)P * C / 8;
  hipLaunchKernelGGL(apply_k, dim3(ew_grid(n8)), dim3(256), 0, st, xx, reinterpret_cast<const u16*>(res),
                     reinterpret_cast<u16*>(y), ss, n8, C, relu);
  return hipGetLastError();
}

hipError_t channel_sum(const bf16* x, float* out, float* part, int P, int C, hipStream_t st) {
  int R, rows, cvb;
  plan(P, C, &R, &rows, &cvb);
  hipLaunchKernelGGL(stats_k<0>, dim3((C / 8 + cvb - 1) / cvb, R), dim3(256), 0, st, reinterpret_cast<const u16*>(x),
                     nullptr, nullptr, nullptr, nullptr, P, C, rows, cvb, part);
  hipLaunchKernelGGL(sum_finalize_k, dim3((C + 63) / 64), dim3(256), 0, st, part, R, C, out);
  return hipGetLastError();
}

hipError_t fwd_eval(const bf16* x, const bf16* res, bf16* y, const float* gamma, const float* beta,
                    const float* rmean, const float* rvar, float* ss, int P, int C, float eps, int relu,
                    hipStream_t st) {
  hipLaunchKernelGGL(eval_coef_k, dim3((C + 255) / 256), dim3(256), 0, st, rmean, rvar, gamma, beta, eps, C, ss);
  const int64_t n8 = (int64_t)P * C / 8;
  hipLaunchKernelGGL(apply_k, dim3(ew_grid(n8)), dim3(256), 0, st, reinterpret_cast<const u16*>(x),
                     reinterpret_cast<const u16*>(res), reinterpret_cast<u16*>(y), ss, n8, C, relu);
  return hipGetLastError();
}

hipError_t bwd(const bf16* dy, const bf16* y, const bf16* x, const float* gamma, const float* mean,
               const float* invstd, bf16* dx, bf16* dres, float* dgamma, float* dbeta, float* coef, float* part, int P,
               int C, hipStream_t st, int accumulate) {
  int R, rows, cvb;
  plan(P, C, &R, &rows, &cvb);
  const u16* d = reinterpret_cast<const u16*>(dy);
  const u16* yy = reinterpret_cast<const u16*>(y);
  const u16* xx = reinterpret_cast<const u16*>(x);
  hipLaunchKernelGGL(stats_k<1>, dim3((C / 8 + cvb - 1) / cvb, R), dim3(256), 0, st, xx, d, yy, mean, invstd, P, C,
                     rows, cvb, part);
  hipLaunchKernelGGL(bwd_finalize_k, dim3((C + 63) / 64), dim3(256), 0, st, part, R, C, P, gamma, invstd, dgamma,
                     dbeta, coef, accumulate);
  const int64_t n8 = (int64_t)P * C / 8;
  hipLaunchKernelGGL(bwd_apply_k, dim3(ew_grid(n8)), dim3(256), 0, st, d, yy, xx, mean, invstd, coef,
                     reinterpret_cast<u16*>(dx), reinterpret_cast<u16*>(dres), n8, C);
  return hipGetLastError();
}

}  // namespace bn
}  // namespace katib_hip
