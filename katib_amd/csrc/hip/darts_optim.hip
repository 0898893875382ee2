// DARTS search-step optimizer kernels - see darts_optim.h.
#include <algorithm>

#include "darts_optim.h"
#include "darts_ops.h"  // kRep

namespace katib_hip {
namespace optim {
namespace {

constexpr int kWave = 64;

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Fixed-order reduction of the sumsq partials by wave 0, broadcast through LDS.
__device__ inline double total_of(const double* parts, int nparts) {
  __shared__ double sh;
  if (threadIdx.x < kWave) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < kMaxParts / kWave; ++k) {
      const int i = threadIdx.x + k * kWave;
      if (i < nparts) v += parts[i];
    }
    v = wave_sum(v);
    if (threadIdx.x == 0) sh = v;
  }
  __syncthreads();
  return sh;
}

int grid_for(int n) { return std::max(1, std::min((n + kThreads - 1) / kThreads, 1024)); }

__global__ void __launch_bounds__(kThreads) sumsq_kernel(const float* __restrict__ x, int n,
                                                         double* __restrict__ parts) {
  __shared__ double sh[kThreads / kWave];
  double acc = 0.0;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
    const double v = x[i];
    acc += v * v;
  }
  acc = wave_sum(acc);
  const int lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
  if (lane == 0) sh[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kThreads / kWave; ++k) s += sh[k];
    parts[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(kThreads) virtual_step_kernel(VirtualStepArgs a) {
  const float lr = *a.lr;
  const int stride = gridDim.x * kThreads;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < a.n; i += stride) {
    const float w = a.w[i];
    // v = (mu * m + g) + wd * w;  w' = w + (-lr) * v   (architect.py:30-47 operation order)
    const float v = __fadd_rn(__fadd_rn(__fmul_rn(a.mom[i], a.mu), a.g[i]), __fmul_rn(w, a.wd));
    a.wv[i] = __fadd_rn(__fmul_rn(v, -lr), w);
    if (a.g_zero) a.g_zero[i] = 0.0f;  // same thread, after its read of g[i]
  }
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < a.n_zero_w; i += stride) a.zero_w[i] = 0.0f;
  if (blockIdx.x == 0) {
    for (int i = threadIdx.x; i < a.na; i += kThreads) {
      a.av[i] = a.a[i];
      a.zero_a[i] = 0.0f;
    }
  }
}

__global__ void __launch_bounds__(kThreads) hessian_kernel(HessianArgs a) {
  float eps;
  const int stride = gridDim.x * kThreads, i0 = blockIdx.x * kThreads + threadIdx.x;
  if (a.phase == 3) {  // concurrent form: both perturbed weight vectors at once, w untouched
    eps = __fdiv_rn(0.01f, static_cast<float>(sqrt(total_of(a.parts, a.nparts))));
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.eps = eps;
    const float m2 = -__fmul_rn(2.0f, eps);
    for (int i = i0; i < a.n; i += stride) {
      const float wp = __fadd_rn(a.w[i], __fmul_rn(a.d[i], eps));
      a.wp[i] = wp;
      a.wm[i] = __fadd_rn(wp, __fmul_rn(a.d[i], m2));
    }
    for (int i = i0; i < a.nbn; i += stride) {
      const float v = a.bn[i];
      a.bn_plus[i] = v;
      a.bn_zero[i] = v;
    }
    if (blockIdx.x == 0)
      for (int i = threadIdx.x; i < a.na; i += kThreads) a.ga[i] = a.gap[i] = 0.0f;
    return;
  }
  if (a.phase == 2 && a.nbn > 0) {
    const float k = 1.0f - a.bn_momentum;
    for (int i = i0; i < a.nbn; i += stride)
      a.bn[i] = __fsub_rn(__fadd_rn(__fmul_rn(k, a.bn_plus[i]), a.bn[i]), __fmul_rn(k, a.bn_zero[i]));
  }
  if (a.phase == 0) {
    const float norm = static_cast<float>(sqrt(total_of(a.parts, a.nparts)));
    eps = __fdiv_rn(0.01f, norm);
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.eps = eps;
  } else {
    eps = *a.eps;
  }
  const float scale = a.phase == 1 ? -__fmul_rn(2.0f, eps) : eps;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < a.n; i += gridDim.x * kThreads)
    a.w[i] = __fadd_rn(a.w[i], __fmul_rn(a.d[i], scale));
  if (blockIdx.x == 0) {
    if (a.phase == 0) {
      for (int i = threadIdx.x; i < a.na; i += kThreads) a.ga[i] = 0.0f;
    } else if (a.phase == 1) {
      for (int i = threadIdx.x; i < a.na; i += kThreads) {
        a.gap[i] = a.ga[i];
        a.ga[i] = 0.0f;
      }
    } else {
      const float lr = *a.lr, two_eps = __fmul_rn(2.0f, eps);
      for (int i = threadIdx.x; i < a.na; i += kThreads) {
        const float h = __fdiv_rn(__fsub_rn(a.gap[i], a.ga[i]), two_eps);
        a.alpha_grad[i] = __fsub_rn(a.gav[i], __fmul_rn(h, lr));
      }
    }
  }
}

// single workgroup (the step counter is read by every thread, then advanced once)
__global__ void __launch_bounds__(kThreads) adam_kernel(AdamArgs a) {
  const float t = *a.t + 1.0f;
  __syncthreads();
  if (threadIdx.x == 0) *a.t = t;
  const float bc1 = 1.0f - powf(a.b1, t), bc2 = 1.0f - powf(a.b2, t);
  const float sbc2 = sqrtf(bc2), step = a.lr / bc1;
  for (int i = threadIdx.x; i < a.n; i += kThreads) {
    const float g = a.grad[i] + a.wd * a.a[i];
    const float m = a.b1 * a.m[i] + (1.0f - a.b1) * g;
    const float v = a.b2 * a.v[i] + (1.0f - a.b2) * g * g;
    a.m[i] = m;
    a.v[i] = v;
    a.a[i] -= m / (sqrtf(v) / sbc2 + a.eps) * step;
  }
  for (int i = threadIdx.x; i < a.nzero; i += kThreads) a.zero[i] = 0.0f;
}

__global__ void __launch_bounds__(kThreads) sgd_clip_kernel(SgdArgs a) {
  const float total = static_cast<float>(sqrt(total_of(a.parts, a.nparts)));
  const float coef = fminf(__fdiv_rn(a.clip, total + 1e-6f), 1.0f);
  const float lr = *a.lr;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < a.n; i += gridDim.x * kThreads) {
    const float g = __fmul_rn(a.g[i], coef);
    const float w = a.w[i];
    a.g[i] = a.zero_g ? 0.0f : g;
    const float m = __fadd_rn(__fmul_rn(a.mom[i], a.mu), __fadd_rn(g, __fmul_rn(w, a.wd)));
    a.mom[i] = m;
    a.w[i] = __fsub_rn(w, __fmul_rn(m, lr));
  }
}

__global__ void __launch_bounds__(kThreads) alpha_softmax_kernel(AlphaSoftmaxArgs a) {
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < a.nzero; i += (long long)gridDim.x * kThreads)
    a.zero[i] = 0.0;
  if (blockIdx.x != 0) return;
  for (int m = 0; m < a.nmat; ++m) {
    for (int r = threadIdx.x; r < a.rows[m]; r += kThreads) {
      const float* x = a.a[m] + (size_t)r * a.K;
      float mx = x[0];
      for (int k = 1; k < a.K; ++k) mx = fmaxf(mx, x[k]);
      float s = 0.0f;
      for (int k = 0; k < a.K; ++k) s += expf(x[k] - mx);
      float* w = a.w[m] + (size_t)r * a.K;
      for (int k = 0; k < a.K; ++k) w[k] = expf(x[k] - mx) / s;
    }
  }
}

// one workgroup per destination row; thread (j, k) = (the row's j-th entry, primitive k): its kRep
// replica loads all in flight at once (a thread walking them serially waited ~2000 dependent
// memory round trips per launch), the entry's dot product over k by a 16-lane shuffle, and the
// entries of the row summed in a fixed order (deterministic)
__global__ void __launch_bounds__(kThreads) alpha_grad_kernel(AlphaGradArgs a) {
  constexpr int KP = 16, EP = kThreads / KP;  // lanes per entry, entries per pass
  __shared__ double sD[EP][KP];
  const int r = blockIdx.x, t = threadIdx.x, j = t / KP, k = t % KP;
  const int e0 = a.row_start[r], e1 = a.row_start[r + 1];
  double acc = 0.0;  // thread k < K of pass-owner j == 0 accumulates the row
  for (int base = e0; base < e1; base += EP) {
    const int e = base + j;
    const bool ok = e < e1 && k < a.K;
    double g = 0.0, w = 0.0;
    if (ok) {
      const double* p = a.g[e] + k;
      const int rs = a.rstride[e];
      double v[katib_hip::kRep];
#pragma unroll
      for (int q = 0; q < katib_hip::kRep; ++q) v[q] = p[(size_t)q * rs];
#pragma unroll
      for (int q = 0; q < katib_hip::kRep; ++q) g += v[q];
      w = (double)a.w[e][k];
    }
    double dot = w * g;
#pragma unroll
    for (int o = KP / 2; o > 0; o >>= 1) dot += __shfl_xor(dot, o, KP);
    sD[j][k] = ok ? w * (g - dot) : 0.0;
    __syncthreads();
    if (t < a.K)
      for (int jj = 0; jj < EP && base + jj < e1; ++jj) acc += sD[jj][t];
    __syncthreads();
  }
  if (t < a.K) {
    float* d = a.dst[r];
    d[t] = a.accumulate ? d[t] + (float)acc : (float)acc;
  }
}

}  // namespace

void launch_alpha_softmax(const AlphaSoftmaxArgs& a, hipStream_t st) {
  const int blocks = std::max(1, (int)std::min<long long>((a.nzero + kThreads - 1) / kThreads, 1024));
  hipLaunchKernelGGL(alpha_softmax_kernel, dim3(blocks), dim3(kThreads), 0, st, a);
}

void launch_alpha_grad(const AlphaGradArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(alpha_grad_kernel, dim3(a.nrows), dim3(kThreads), 0, st, a);
}

int sumsq_parts(int n) { return std::max(1, std::min((n + kThreads * 8 - 1) / (kThreads * 8), kMaxParts)); }

void launch_sumsq(const float* x, int n, double* parts, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(sumsq_parts(n)), dim3(kThreads), 0, st, x, n, parts);
}

void launch_virtual_step(const VirtualStepArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(virtual_step_kernel, dim3(grid_for(std::max(a.n, a.n_zero_w))), dim3(kThreads), 0, st, a);
}

void launch_hessian(const HessianArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(hessian_kernel, dim3(grid_for(std::max(a.n, a.nbn))), dim3(kThreads), 0, st, a);
}

void launch_adam(const AdamArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(1), dim3(kThreads), 0, st, a);
}

void launch_sgd_clip(const SgdArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sgd_clip_kernel, dim3(grid_for(a.n)), dim3(kThreads), 0, st, a);
}

}  // namespace optim
}  // namespace katib_hip
