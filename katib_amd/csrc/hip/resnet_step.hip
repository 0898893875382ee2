// Fused ResNet-18 step kernels: input gather, classifier head, multi-tensor SGD (resnet_step.h).
//
// Reference parity: the trial is the reference's PyTorch ResNet-18 CIFAR job of BASELINE
// config 3 (HyperBand + median-stop, examples/v1beta1/trial-images - a torchvision-style
// training loop: SGD + Nesterov momentum + weight decay, cross-entropy on a linear head after
// global average pooling). The math here is that loop's; the launches are shaped for gfx950:
// one workgroup per sample for the head, fixed-order batch reductions, and a single SGD launch
// over every parameter tensor (64 x 64 LDS tiles per filter slice so the transposed bf16 image
// is written with coalesced rows).
#include <cmath>

#include "resnet_step.h"

namespace katib_hip {
namespace rn {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16;

constexpr int kThreads = 256;
constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// ------------------------------------------------------------------ gather + pad
__global__ __launch_bounds__(kThreads) void gather_k(const u16* __restrict__ tx, const int64_t* __restrict__ idx,
                                                     u16* __restrict__ xb, int B, int HW, int C, int C8,
                                                     int64_t n_src) {
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;  // one (sample, pixel)
  if (t >= (int64_t)B * HW) return;
  const int b = (int)(t / HW), p = (int)(t - (int64_t)b * HW);
  const int64_t j = idx[b];
  const bool ok = j >= 0 && j < n_src;  // out-of-range index -> zero image, no out-of-bounds read
  const u16* src = tx + ((ok ? j : 0) * HW + p) * C;
  u16* dst = xb + t * C8;
  for (int c0 = 0; c0 < C8; c0 += 8) {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 2 * q;
      const uint32_t lo = (ok && c < C) ? src[c] : 0u, hi = (ok && c + 1 < C) ? src[c + 1] : 0u;
      w[q] = lo | (hi << 16);
    }
    *reinterpret_cast<u32x4*>(dst + c0) = u32x4{w[0], w[1], w[2], w[3]};
  }
}

// ------------------------------------------------------------------ head (one workgroup per sample)
__global__ __launch_bounds__(kThreads) void head_k(HeadArgs a) {
  __shared__ float sp[kHeadMaxC];
  __shared__ float sdx[kHeadMaxC];
  __shared__ float sl[kHeadMaxK];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid % kWave, wid = tid / kWave;
  const int C = a.C, K = a.K, HW = a.HW, CV = C / 8;
  for (int c = tid; c < C; c += kThreads) sp[c] = 0.f;
  __syncthreads();
  const u16* xb = reinterpret_cast<const u16*>(a.x) + (int64_t)b * HW * C;
  // sum over pixels: a thread's vectors share one channel group when CV divides 256 (flush on change)
  {
    float acc[8];
    int cur = -1;
    for (int v = tid; v < HW * CV; v += kThreads) {
      const int c0 = (v % CV) * 8;
      if (c0 != cur) {
        if (cur >= 0)
          for (int e = 0; e < 8; ++e) atomicAdd(&sp[cur + e], acc[e]);
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
        cur = c0;
      }
      const u32x4 q = *reinterpret_cast<const u32x4*>(xb + (int64_t)v * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(q[k] << 16);
        acc[2 * k + 1] += __uint_as_float(q[k] & 0xffff0000u);
      }
    }
    if (cur >= 0)
      for (int e = 0; e < 8; ++e) atomicAdd(&sp[cur + e], acc[e]);
  }
  __syncthreads();
  const float inv_hw = 1.0f / HW;
  for (int c = tid; c < C; c += kThreads) {
    const float v = sp[c] * inv_hw;
    sp[c] = v;
    a.pooled[(int64_t)b * C + c] = v;
  }
  __syncthreads();
  for (int k = wid; k < K; k += kThreads / kWave) {
    float s = 0.f;
    for (int c = lane; c < C; c += kWave) s += sp[c] * a.w[(int64_t)k * C + c];
    s = wave_sum(s);
    if (lane == 0) sl[k] = s + a.bias[k];
  }
  __syncthreads();
  if (tid == 0) {
    float m = sl[0];
    for (int k = 1; k < K; ++k) m = fmaxf(m, sl[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(sl[k] - m);
    const float lse = m + logf(se);
    const int64_t j = a.idx[b];
    const int64_t t = (j >= 0 && j < a.n_labels) ? a.ty[j] : -1;
    const bool ok = t >= 0 && t < K;  // bad label -> NaN loss (visible), no out-of-bounds read
    a.loss_n[b] = ok ? lse - sl[ok ? t : 0] : NAN;
    const float inv_b = 1.0f / a.B;
    for (int k = 0; k < K; ++k) {
      const float d = (expf(sl[k] - lse) - (k == t ? 1.f : 0.f)) * inv_b;
      sl[k] = d;
      a.dl[(int64_t)b * K + k] = d;
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += kThreads) {
    float d = 0.f;
    for (int k = 0; k < K; ++k) d += sl[k] * a.w[(int64_t)k * C + c];
    sdx[c] = d * inv_hw;
  }
  __syncthreads();
  u16* dxb = reinterpret_cast<u16*>(a.dx) + (int64_t)b * HW * C;
  for (int v = tid; v < HW * CV; v += kThreads) {
    const int c0 = (v % CV) * 8;
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(sdx[c0 + 2 * q]) | ((uint32_t)f2bf(sdx[c0 + 2 * q + 1]) << 16);
    *reinterpret_cast<u32x4*>(dxb + (int64_t)v * 8) = u32x4{w[0], w[1], w[2], w[3]};
  }
}

// batch reductions: blocks [0, nb) 64 weight-gradient elements each, the batch split over the 4
// waves (a serial 256-sample chain per thread was 61 us), summed in a fixed order through LDS;
// block nb: bias + loss
__global__ __launch_bounds__(kThreads) void head_reduce_k(HeadArgs a) {
  const int nb = (a.K * a.C + kWave - 1) / kWave, tid = threadIdx.x;
  if ((int)blockIdx.x < nb) {
    __shared__ float part[kThreads / kWave][kWave];
    const int lane = tid % kWave, w = tid / kWave;
    const int e = blockIdx.x * kWave + lane;
    float s = 0.f;
    if (e < a.K * a.C) {
      const int k = e / a.C, c = e - k * a.C;
#pragma unroll 8
      for (int b = w; b < a.B; b += kThreads / kWave) s += a.dl[(int64_t)b * a.K + k] * a.pooled[(int64_t)b * a.C + c];
    }
    part[w][lane] = s;
    __syncthreads();
    if (w == 0 && e < a.K * a.C) a.gw[e] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    return;
  }
  if (tid < a.K) {
    float s = 0.f;
#pragma unroll 8
    for (int b = 0; b < a.B; ++b) s += a.dl[(int64_t)b * a.K + tid];
    a.gb[tid] = s;
  }
  if (a.loss_acc != nullptr && tid >= kWave && tid < 2 * kWave) {
    float s = 0.f;
    for (int b = tid - kWave; b < a.B; b += kWave) s += a.loss_n[b];
    s = wave_sum(s);
    if (tid == kWave) *a.loss_acc += s / a.B;
  }
}

// ------------------------------------------------------------------ multi-tensor SGD
constexpr int kFlatTile = 4096;
constexpr int kT = 64;  // filter tile: 64 output channels x 64 input channels of one (r, s)

__device__ __forceinline__ void sgd_update(float& p, float g, float& m, float lr, float mom, float wd, int nesterov) {
  const float d = g + wd * p;
  m = mom * m + d;
  p -= lr * (nesterov ? d + mom * m : m);
}

__global__ __launch_bounds__(kThreads) void sgd_k(const SgdSeg* __restrict__ segs, int nseg, float lr, float mom,
                                                  float wd, int nesterov, int update) {
  __shared__ u16 tile[kT * (kT + 1)];
  const int t = blockIdx.x, tid = threadIdx.x;
  int lo = 0, hi = nseg - 1;  // last segment with tile0 <= t
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].tile0 <= t)
      lo = mid;
    else
      hi = mid - 1;
  }
  const SgdSeg s = segs[lo];
  const int lt = t - s.tile0;
  if (s.wk == nullptr) {
    if (!update) return;
    const int base = lt * kFlatTile;
#pragma unroll 4
    for (int j = 0; j < kFlatTile / kThreads; ++j) {
      const int i = base + tid + kThreads * j;
      if (i < s.n) {
        float p = s.p[i], m = s.m[i];
        sgd_update(p, s.g[i], m, lr, mom, wd, nesterov);
        s.p[i] = p;
        s.m[i] = m;
        s.g[i] = 0.f;
      }
    }
    return;
  }
  const int tiles_k = (s.K + kT - 1) / kT;
  const int rs = lt % s.RS, r2 = lt / s.RS, kt = r2 % tiles_k, ct = r2 / tiles_k;
  const int cl = tid & (kT - 1), c = ct * kT + cl;
#pragma unroll 4
  for (int j = 0; j < kT * kT / kThreads; ++j) {
    const int kl = (tid >> 6) + (kThreads / kT) * j, k = kt * kT + kl;
    float w = 0.f;
    if (k < s.K && c < s.C8) {
      const int64_t row = (int64_t)k * s.RS + rs;
      if (c < s.C) {
        const int64_t pi = row * s.C + c;
        float p = s.p[pi];
        if (update) {
          float m = s.m[pi];
          sgd_update(p, s.g[row * s.C8 + c], m, lr, mom, wd, nesterov);
          s.p[pi] = p;
          s.m[pi] = m;
          s.g[row * s.C8 + c] = 0.f;
        }
        w = p;
      } else if (update) {
        s.g[row * s.C8 + c] = 0.f;
      }
      reinterpret_cast<u16*>(s.wk)[row * s.C8 + c] = f2bf(w);
    }
    tile[cl * (kT + 1) + kl] = f2bf(w);
  }
  if (s.wt == nullptr) return;  // uniform per workgroup
  __syncthreads();
  const int kl = tid & (kT - 1), k = kt * kT + kl;
#pragma unroll 4
  for (int j = 0; j < kT * kT / kThreads; ++j) {
    const int cl2 = (tid >> 6) + (kThreads / kT) * j, c2 = ct * kT + cl2;
    if (c2 < s.C8 && k < s.K)
      reinterpret_cast<u16*>(s.wt)[((int64_t)c2 * s.RS + rs) * s.K + k] = tile[cl2 * (kT + 1) + kl];
  }
}

}  // namespace

hipError_t launch_gather(const bf16* tx, const int64_t* idx, bf16* xb, int B, int HW, int C, int C8, int64_t n_src,
                         hipStream_t st) {
  const int64_t n = (int64_t)B * HW;
  hipLaunchKernelGGL(gather_k, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                     reinterpret_cast<const u16*>(tx), idx, reinterpret_cast<u16*>(xb), B, HW, C, C8, n_src);
  return hipGetLastError();
}

hipError_t launch_head(const HeadArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(head_k, dim3(a.B), dim3(kThreads), 0, st, a);
  const int nb = (a.K * a.C + kWave - 1) / kWave;
  hipLaunchKernelGGL(head_reduce_k, dim3(nb + 1), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

int sgd_tiles(const SgdSeg& s) {
  if (s.wk == nullptr) return (s.n + kFlatTile - 1) / kFlatTile;
  return s.RS * ((s.K + kT - 1) / kT) * ((s.C8 + kT - 1) / kT);
}

hipError_t launch_sgd(const SgdSeg* segs_dev, int nseg, int total_tiles, float lr, float momentum, float wd,
                      int nesterov, int update, hipStream_t st) {
  hipLaunchKernelGGL(sgd_k, dim3(total_tiles), dim3(kThreads), 0, st, segs_dev, nseg, lr, momentum, wd, nesterov,
                     update);
  return hipGetLastError();
}

}  // namespace rn
}  // namespace katib_hip
