// Fused DARTS head: gap + classifier + cross-entropy, forward and backward - see darts_head.h.
#include <cmath>

#include "darts_head.h"
#include "darts_ops.h"  // kRep (weight-gradient replica rows)

namespace katib_hip {
namespace head {
namespace {

constexpr int kThreads = 256;
constexpr int kWave = 64;
constexpr int kWaves = kThreads / kWave;
constexpr int kU = 8;  // channels / classes per wave with loads in flight together

__device__ inline float wave_sum(float v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// one workgroup per sample; wave w pools channels w, w+4, ... with its lanes over the pixels
__global__ void __launch_bounds__(kThreads) head_fwd_kernel(FwdArgs a) {
  __shared__ float sp[kMaxC];
  __shared__ float sl[kMaxK];
  const int n = blockIdx.x, lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
  const float inv_hw = 1.0f / a.HW;
  // kU channels per wave in flight: all loads issue before the first reduction (the chain of
  // one load -> wave sum per channel was latency-bound)
  for (int c0 = wid; c0 < a.C; c0 += kWaves * kU) {
    float s[kU];
    if (a.HW <= kWave) {  // one pixel per lane: straight-line loads
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int c = c0 + u * kWaves;
        s[u] = (c < a.C && lane < a.HW) ? a.x[plane_off(n, c, a.N, a.C, a.nodes, a.HW) + lane] : 0.0f;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int c = c0 + u * kWaves;
        float v = 0.0f;
        if (c < a.C) {
          const float* xc = a.x + plane_off(n, c, a.N, a.C, a.nodes, a.HW);
          for (int p = lane; p < a.HW; p += kWave) v += xc[p];
        }
        s[u] = v;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int c = c0 + u * kWaves;
      const float v = wave_sum(s[u]) * inv_hw;
      if (lane == 0 && c < a.C) sp[c] = v;
    }
  }
  __syncthreads();
  // the pooled features leave after the pooling loop: a global store inside it could alias x, which
  // kept every channel group's loads behind the previous group's stores (a round trip per group)
  for (int c = threadIdx.x; c < a.C; c += kThreads) a.pooled[(size_t)n * a.C + c] = sp[c];
  for (int k0 = wid; k0 < a.K; k0 += kWaves * kU) {
    float s[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int k = k0 + u * kWaves;
      float v = 0.0f;
      if (k < a.K) {
        if (a.C <= kWave) {
          v = lane < a.C ? sp[lane] * a.w[(size_t)k * a.C + lane] : 0.0f;
        } else {
          for (int c = lane; c < a.C; c += kWave) v += sp[c] * a.w[(size_t)k * a.C + c];
        }
      }
      s[u] = v;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int k = k0 + u * kWaves;
      const float v = wave_sum(s[u]);
      if (lane == 0 && k < a.K) {
        const float l = v + a.b[k];
        sl[k] = l;
        a.logits[(size_t)n * a.K + k] = l;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = sl[0];
    for (int k = 1; k < a.K; ++k) m = fmaxf(m, sl[k]);
    float se = 0.0f;
    for (int k = 0; k < a.K; ++k) se += expf(sl[k] - m);
    const float lse = m + logf(se);
    const int64_t t = a.y[n];
    const bool ok = t >= 0 && t < a.K;  // out-of-range label -> NaN loss, no out-of-bounds read
    a.loss_n[n] = ok ? lse - sl[t] : NAN;
    const float inv_n = 1.0f / a.N;
    for (int k = 0; k < a.K; ++k)
      a.dl[(size_t)n * a.K + k] = (expf(sl[k] - lse) - (k == t ? 1.0f : 0.0f)) * inv_n;
  }
}

__global__ void __launch_bounds__(kThreads) head_loss_kernel(const float* __restrict__ loss_n, int N,
                                                             float* __restrict__ loss) {
  __shared__ float sh[kWaves];
  float s = 0.0f;
  for (int i = threadIdx.x; i < N; i += kThreads) s += loss_n[i];
  s = wave_sum(s);
  if (threadIdx.x % kWave == 0) sh[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.0f;
    for (int i = 0; i < kWaves; ++i) t += sh[i];
    *loss = t / N;
  }
}

__global__ void __launch_bounds__(kThreads) head_bwd_kernel(BwdArgs a) {
  __shared__ float sd[kMaxK];
  const int n = blockIdx.x, lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
  const float g = *a.gout;
  if (threadIdx.x < a.K) sd[threadIdx.x] = g * a.dl[(size_t)n * a.K + threadIdx.x];
  __syncthreads();
  if (a.dx != nullptr) {
    // d[c] = (dl W)[c] / HW for every channel first (weight loads only, all in flight), then the
    // broadcast stores: interleaving each channel's stores with the next channel's weight loads
    // (which may alias dx for the compiler) serialised one round trip per channel - 64 per
    // workgroup on the darts-gpu.yaml head (47.6 us per launch)
    __shared__ float sdx[kMaxC];
    const float inv_hw = 1.0f / a.HW;
    for (int c = threadIdx.x; c < a.C; c += kThreads) {
      float d = 0.0f;
      for (int k = 0; k < a.K; ++k) d += sd[k] * a.w[(size_t)k * a.C + c];
      sdx[c] = d * inv_hw;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.C * a.HW; i += kThreads) {
      const int c = i / a.HW, p = i - c * a.HW;
      a.dx[plane_off(n, c, a.N, a.C, a.nodes, a.HW) + p] = sdx[c];
    }
  }
  const int rep = n % kRep;
  if (a.gw != nullptr) {
    const float* pn = a.pooled + (size_t)n * a.C;
    float* gw = a.gw + (size_t)rep * a.gw_stride;
    for (int i = threadIdx.x; i < a.K * a.C; i += kThreads) atomicAdd(gw + i, sd[i / a.C] * pn[i % a.C]);
  }
  if (a.gb != nullptr && threadIdx.x < a.K) atomicAdd(a.gb + (size_t)rep * a.gb_stride + threadIdx.x, sd[threadIdx.x]);
}

}  // namespace

void launch_fwd(const FwdArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a.N), dim3(kThreads), 0, st, a);
}

void launch_loss(const float* loss_n, int N, float* loss, hipStream_t st) {
  hipLaunchKernelGGL(head_loss_kernel, dim3(1), dim3(kThreads), 0, st, loss_n, N, loss);
}

void launch_bwd(const BwdArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(head_bwd_kernel, dim3(a.N), dim3(kThreads), 0, st, a);
}

}  // namespace head
}  // namespace katib_hip
