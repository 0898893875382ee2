// GPT-2 trial kernels for gfx950 (BASELINE config 5: PBT on GPT-2 small).
//
// The torch-op profile of the trial (profiles/gpt2_torch_baseline_kernel_stats.txt) spends
// ~35 % in hipBLASLt GEMMs and the rest in attention, an fp32 vocabulary softmax (forward
// and backward, 50257 columns), dtype casts of every weight and activation, LayerNorm and
// AdamW. These kernels replace everything except the plain GEMMs:
//
//  * ln_fwd / ln_bwd        residual add fused into LayerNorm; one wave per row, the row
//                           in registers (D % 256 == 0), fp32 residual stream, bf16 out.
//  * gelu_fwd / gelu_bwd    tanh GELU, 16-byte vectors.
//  * xent_fwd / xent_bwd    cross-entropy over the (padded) vocabulary straight from the
//                           bf16 logits: online max/sum in the forward, the gradient
//                           written in place over the logits in the backward.
//  * grad_sumsq / adamw     global-norm clip + AdamW over one flat fp32 master buffer,
//                           emitting the bf16 shadow weights the GEMMs read.
//  * attn_fwd / attn_bwd    causal flash attention for head dim 64 on
//                           v_mfma_f32_16x16x32_bf16. The score tile is computed
//                           transposed (key on the accumulator row, query on the lane),
//                           so the online softmax is lane-local except for two
//                           cross-lane steps, and the bf16 probabilities feed the P.V
//                           MFMA as B operands with no data movement; V (and K, dO, Q in
//                           the backward) are consumed column-wise through the gfx950
//                           transposing LDS read ds_read_b64_tr_b16.
#include <cstdlib>
#include "transformer.h"

#include <math.h>

namespace katib_hip {
namespace tfm {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16;

__device__ __forceinline__ float bf2f(u16 b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ float lo2f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi2f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ uint32_t pack2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ============================================================== LayerNorm
template <int V>  // D = 256 * V; one wave per row, lane owns columns 256 i + 4 lane .. + 3
__global__ __launch_bounds__(256) void ln_fwd_k(const float* __restrict__ x32, const u16* __restrict__ r,
                                                float* __restrict__ xo, const u16* __restrict__ gamma,
                                                const u16* __restrict__ beta, u16* __restrict__ y,
                                                float* __restrict__ mean, float* __restrict__ rstd, int M,
                                                float eps) {
  constexpr int D = 256 * V;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int64_t base = (int64_t)row * D;
  f32x4 v[V];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 256 * i + 4 * lane;
    f32x4 t = *reinterpret_cast<const f32x4*>(x32 + base + c);
    if (r) {
      const u32x2 rr = *reinterpret_cast<const u32x2*>(r + base + c);
      t[0] += lo2f(rr[0]);
      t[1] += hi2f(rr[0]);
      t[2] += lo2f(rr[1]);
      t[3] += hi2f(rr[1]);
      *reinterpret_cast<f32x4*>(xo + base + c) = t;
    }
    v[i] = t;
    s += (t[0] + t[1]) + (t[2] + t[3]);
  }
  const float mu = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = v[i][k] - mu;
      q += d * d;
    }
  const float rs = rsqrtf(wave_sum(q) * (1.f / D) + eps);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int c = 256 * i + 4 * lane;
    const u32x2 gg = *reinterpret_cast<const u32x2*>(gamma + c);
    const u32x2 bb = *reinterpret_cast<const u32x2*>(beta + c);
    u32x2 o;
    o[0] = pack2((v[i][0] - mu) * rs * lo2f(gg[0]) + lo2f(bb[0]), (v[i][1] - mu) * rs * hi2f(gg[0]) + hi2f(bb[0]));
    o[1] = pack2((v[i][2] - mu) * rs * lo2f(gg[1]) + lo2f(bb[1]), (v[i][3] - mu) * rs * hi2f(gg[1]) + hi2f(bb[1]));
    *reinterpret_cast<u32x2*>(y + base + c) = o;
  }
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

constexpr int kLnBwdBlocks = 256;

template <int V>
__global__ __launch_bounds__(256) void ln_bwd_k(const u16* __restrict__ dy, const float* __restrict__ xin,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                const u16* __restrict__ gamma, const float* dres, float* dx,
                                                u16* __restrict__ dr, float* __restrict__ part_g,
                                                float* __restrict__ part_b, float* __restrict__ part_r, int M) {
  constexpr int D = 256 * V;
  __shared__ float red[2][4][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // part_r != nullptr: also the column sums of the bf16 gradient written to dr - the bias gradient
  // of the linear layer whose output dr is (GPT-2: attn proj / fc2), so no separate column-sum pass
  f32x4 ag[V], ab[V], ar[V], gv[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    ag[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    ab[i] = ag[i];
    ar[i] = ag[i];
    const u32x2 gg = *reinterpret_cast<const u32x2*>(gamma + 256 * i + 4 * lane);
    gv[i] = f32x4{lo2f(gg[0]), hi2f(gg[0]), lo2f(gg[1]), hi2f(gg[1])};
  }
  // two rows per wave per iteration: both rows' loads issue before either row's reductions (one row
  // per iteration left each wave with a serial load -> wave_sum -> store chain at one wave per SIMD)
  constexpr int RR = 2;
  const int stride = gridDim.x * 4;
  for (int row0 = blockIdx.x * 4 + w; row0 < M; row0 += RR * stride) {
    f32x4 xh[RR][V], g[RR][V], rd[RR][V];
    float s1[RR], s2[RR], mu[RR], rs[RR];
    bool ok[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      const int row = row0 + r * stride;
      ok[r] = row < M;
      const int rw = ok[r] ? row : row0;
      const int64_t base = (int64_t)rw * D;
      mu[r] = mean[rw];
      rs[r] = rstd[rw];
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = 256 * i + 4 * lane;
        xh[r][i] = *reinterpret_cast<const f32x4*>(xin + base + c);
        const u32x2 d2 = *reinterpret_cast<const u32x2*>(dy + base + c);
        g[r][i] = f32x4{lo2f(d2[0]), hi2f(d2[0]), lo2f(d2[1]), hi2f(d2[1])};
        rd[r][i] = dres ? *reinterpret_cast<const f32x4*>(dres + base + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      s1[r] = 0.f;
      s2[r] = 0.f;
#pragma unroll
      for (int i = 0; i < V; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          xh[r][i][k] = (xh[r][i][k] - mu[r]) * rs[r];
          const float dxh = g[r][i][k] * gv[i][k];
          s1[r] += dxh;
          s2[r] += dxh * xh[r][i][k];
          if (ok[r]) {
            ag[i][k] += g[r][i][k] * xh[r][i][k];
            ab[i][k] += g[r][i][k];
          }
        }
    }
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      s1[r] = wave_sum(s1[r]) * (1.f / D);
      s2[r] = wave_sum(s2[r]) * (1.f / D);
    }
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      if (!ok[r]) continue;  // wave-uniform
      const int64_t base = (int64_t)(row0 + r * stride) * D;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int c = 256 * i + 4 * lane;
        f32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = rs[r] * (g[r][i][k] * gv[i][k] - s1[r] - xh[r][i][k] * s2[r]);
        o += rd[r][i];
        *reinterpret_cast<f32x4*>(dx + base + c) = o;
        if (dr) {
          const u32x2 ob = u32x2{pack2(o[0], o[1]), pack2(o[2], o[3])};
          *reinterpret_cast<u32x2*>(dr + base + c) = ob;
          if (part_r) ar[i] += f32x4{lo2f(ob[0]), hi2f(ob[0]), lo2f(ob[1]), hi2f(ob[1])};  // what colsum(dr) sums
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    *reinterpret_cast<f32x4*>(&red[0][w][256 * i + 4 * lane]) = ag[i];
    *reinterpret_cast<f32x4*>(&red[1][w][256 * i + 4 * lane]) = ab[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    part_g[(int64_t)blockIdx.x * D + c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
    part_b[(int64_t)blockIdx.x * D + c] = (red[1][0][c] + red[1][1][c]) + (red[1][2][c] + red[1][3][c]);
  }
  if (part_r == nullptr) return;  // uniform
  __syncthreads();  // red[0] is reused (a third [4][D] array would pass the 64 KB static LDS limit at D = 2048)
#pragma unroll
  for (int i = 0; i < V; ++i) *reinterpret_cast<f32x4*>(&red[0][w][256 * i + 4 * lane]) = ar[i];
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256)
    part_r[(int64_t)blockIdx.x * D + c] = (red[0][0][c] + red[0][1][c]) + (red[0][2][c] + red[0][3][c]);
}

// sum nblk partial rows per column: block = 64 columns x 4 row groups
// block = 64 columns x 16 row groups (1024 threads): only D / 64 workgroups exist, so each needs
// many loads in flight; the optional third array (bias gradient) is read in the same loop
constexpr int kLnRedGroups = 16;
__global__ __launch_bounds__(64 * kLnRedGroups) void ln_reduce_k(const float* __restrict__ pg,
                                                                 const float* __restrict__ pb,
                                                                 const float* __restrict__ pr, int nblk, int D,
                                                                 u16* __restrict__ dg, u16* __restrict__ db,
                                                                 u16* __restrict__ dbias) {
  __shared__ float red[3][kLnRedGroups][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6, c = blockIdx.x * 64 + tx;
  float sg = 0.f, sb = 0.f, sr = 0.f;
  if (c < D) {
    if (pr) {
#pragma unroll 4
      for (int r = ty; r < nblk; r += kLnRedGroups) {
        sg += pg[(int64_t)r * D + c];
        sb += pb[(int64_t)r * D + c];
        sr += pr[(int64_t)r * D + c];
      }
    } else {
#pragma unroll 4
      for (int r = ty; r < nblk; r += kLnRedGroups) {
        sg += pg[(int64_t)r * D + c];
        sb += pb[(int64_t)r * D + c];
      }
    }
  }
  red[0][ty][tx] = sg;
  red[1][ty][tx] = sb;
  red[2][ty][tx] = sr;
  __syncthreads();
  if (ty < 3 && c < D) {  // one wave per output array, fixed summation order
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kLnRedGroups; ++k) t += red[ty][k][tx];
    u16* out = ty == 0 ? dg : (ty == 1 ? db : dbias);
    if (out) out[c] = f2bf(t);
  }
}

// ============================================================== GELU (tanh form)
constexpr float kGeluK0 = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kGeluK1 = 0.044715f;

__device__ __forceinline__ float tanh_fast(float z) {  // hardware exp2 + reciprocal (no IEEE divide)
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z * 2.8853900817779268f) + 1.f);  // 2 log2(e)
}
__device__ __forceinline__ float gelu_f(float u) {
  return 0.5f * u * (1.f + tanh_fast(kGeluK0 * (u + kGeluK1 * u * u * u)));
}
__device__ __forceinline__ float gelu_df(float u) {
  const float t = tanh_fast(kGeluK0 * (u + kGeluK1 * u * u * u));
  return 0.5f * (1.f + t) + 0.5f * u * (1.f - t * t) * kGeluK0 * (1.f + 3.f * kGeluK1 * u * u);
}

__global__ __launch_bounds__(256) void gelu_fwd_k(const u16* __restrict__ u, u16* __restrict__ g, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const u32x4 a = reinterpret_cast<const u32x4*>(u)[i];
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = pack2(gelu_f(lo2f(a[k])), gelu_f(hi2f(a[k])));
    reinterpret_cast<u32x4*>(g)[i] = o;
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_k(const u16* __restrict__ u, const u16* __restrict__ dy,
                                                  u16* __restrict__ du, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const u32x4 a = reinterpret_cast<const u32x4*>(u)[i];
    const u32x4 d = reinterpret_cast<const u32x4*>(dy)[i];
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = pack2(lo2f(d[k]) * gelu_df(lo2f(a[k])), hi2f(d[k]) * gelu_df(hi2f(a[k])));
    reinterpret_cast<u32x4*>(du)[i] = o;
  }
}

// ============================================================== cross-entropy
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ void block_max_sum(float& m, float& s, float* sh) {
  // combine (max, sum-of-exp2) pairs across the 4 waves of a 256-thread block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = (mn == -INFINITY) ? 0.f : s * exp2f(m - mn) + s2 * exp2f(m2 - mn);
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[2 * w] = m;
    sh[2 * w + 1] = s;
  }
  __syncthreads();
  float mm = sh[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) mm = fmaxf(mm, sh[2 * i]);
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) ss += sh[2 * i + 1] * exp2f(sh[2 * i] - mm);
  m = mm;
  s = ss;
}

__global__ __launch_bounds__(256) void xent_fwd_k(const u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                  float* __restrict__ loss, float* __restrict__ lse, int V, int Vp) {
  __shared__ float sh[8];
  const int row = blockIdx.x;
  const u16* L = logits + (int64_t)row * Vp;
  const int nch = Vp >> 3;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < nch; c += 256) {
    const u32x4 q = reinterpret_cast<const u32x4*>(L)[c];
    float x[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[2 * k] = lo2f(q[k]) * kLog2e;
      x[2 * k + 1] = hi2f(q[k]) * kLog2e;
    }
    if (8 * c + 8 > V) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (8 * c + e >= V) x[e] = -INFINITY;
    }
    float cm = x[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) cm = fmaxf(cm, x[e]);
    const float mn = fmaxf(m, cm);
    if (mn == -INFINITY) continue;
    float cs = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) cs += exp2f(x[e] - mn);
    s = s * exp2f(m - mn) + cs;
    m = mn;
  }
  block_max_sum(m, s, sh);
  if (threadIdx.x == 0) {
    const float l = (m + log2f(s)) * kLn2;
    const int64_t t = tgt[row];
    const float xt = (t >= 0 && t < V) ? bf2f(L[t]) : 0.f;
    lse[row] = l;
    loss[row] = l - xt;
  }
}

// Evaluation: per-row loss and top-1 hit in ONE pass over the bf16 logits row (the validation metric
// PBT ranks members on) - instead of an fp32 copy of the logits, a softmax / NLL and an argmax reduce.
// argmax ties resolve to the lowest index (torch.argmax's choice).
__global__ __launch_bounds__(256) void xent_eval_k(const u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                   float* __restrict__ loss, float* __restrict__ hit, int V, int Vp) {
  __shared__ float sh[8];
  __shared__ float shv[4];
  __shared__ int shi[4];
  const int row = blockIdx.x;
  const u16* L = logits + (int64_t)row * Vp;
  const int nch = Vp >> 3;
  float m = -INFINITY, s = 0.f, bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = threadIdx.x; c < nch; c += 256) {
    const u32x4 q = reinterpret_cast<const u32x4*>(L)[c];
    float r[8], x[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r[2 * k] = lo2f(q[k]);
      r[2 * k + 1] = hi2f(q[k]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (8 * c + e >= V) r[e] = -INFINITY;
      x[e] = r[e] * kLog2e;
      if (r[e] > bv) {  // strictly greater: the first index of a tie stays (columns ascend per thread)
        bv = r[e];
        bi = 8 * c + e;
      }
    }
    float cm = x[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) cm = fmaxf(cm, x[e]);
    const float mn = fmaxf(m, cm);
    if (mn == -INFINITY) continue;
    float cs = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) cs += exp2f(x[e] - mn);
    s = s * exp2f(m - mn) + cs;
    m = mn;
  }
  block_max_sum(m, s, sh);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(bv, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (v2 > bv || (v2 == bv && i2 < bi)) {
      bv = v2;
      bi = i2;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    shv[threadIdx.x >> 6] = bv;
    shi[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bv = shv[0];
    bi = shi[0];
#pragma unroll
    for (int w = 1; w < 4; ++w)
      if (shv[w] > bv || (shv[w] == bv && shi[w] < bi)) {
        bv = shv[w];
        bi = shi[w];
      }
    const float l = (m + log2f(s)) * kLn2;
    const int64_t t = tgt[row];
    const float xt = (t >= 0 && t < V) ? bf2f(L[t]) : 0.f;
    loss[row] = l - xt;
    hit[row] = (t == (int64_t)bi) ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(256) void xent_bwd_k(u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                  const float* __restrict__ lse, const float* __restrict__ gscale,
                                                  float inv_n, int V, int Vp) {
  const int row = blockIdx.x;
  u16* L = logits + (int64_t)row * Vp;
  const int nch = Vp >> 3;
  const float l2 = lse[row] * kLog2e;
  const float sc = gscale[0] * inv_n;
  const int64_t t = tgt[row];
  for (int c = threadIdx.x; c < nch; c += 256) {
    u32x4 q = reinterpret_cast<u32x4*>(L)[c];
    float g[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      g[2 * k] = exp2f(lo2f(q[k]) * kLog2e - l2);
      g[2 * k + 1] = exp2f(hi2f(q[k]) * kLog2e - l2);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = 8 * c + e;
      g[e] = col >= V ? 0.f : (g[e] - (col == t ? 1.f : 0.f)) * sc;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = pack2(g[2 * k], g[2 * k + 1]);
    reinterpret_cast<u32x4*>(L)[c] = q;
  }
}

// Forward + backward in one pass over the row (training): the row's 8-bf16 vectors are held in
// registers between the (max, sum) reduction and the gradient write, so the logits are read from HBM
// once instead of twice (xent_fwd_k then xent_bwd_k: 1.6 GB read twice per GPT-2 step at 16k tokens).
template <int NV>  // vectors of 8 bf16 per thread: Vp <= 8 * kXentThreads * NV
__global__ __launch_bounds__(512, 4) void xent_fused_k(u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                    float* __restrict__ loss, float* __restrict__ lse,
                                                    const float* __restrict__ gscale, float inv_n, int V, int Vp) {
  constexpr int kT = 512, kW = kT / 64;  // 8 waves: ~13 vectors per thread for GPT-2's 50304 columns
  __shared__ float sh[2 * kW];
  const int row = blockIdx.x;
  u16* L = logits + (int64_t)row * Vp;
  const int nch = Vp >> 3;
  const int64_t t = tgt[row];
  const bool tok = t >= 0 && t < V;
  const float xt = (threadIdx.x == 0 && tok) ? bf2f(L[t]) : 0.f;  // read before any thread overwrites the row
  u32x4 q[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = threadIdx.x + kT * j;
    q[j] = c < nch ? reinterpret_cast<const u32x4*>(L)[c] : u32x4{0u, 0u, 0u, 0u};
  }
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = threadIdx.x + kT * j;
    if (c >= nch) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = 8 * c + 2 * k;
      if (col < V) m = fmaxf(m, lo2f(q[j][k]));
      if (col + 1 < V) m = fmaxf(m, hi2f(q[j][k]));
    }
  }
  // block max, then the sum of exp2 against it (two reductions; no online rescaling needed)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  m = sh[0];
#pragma unroll
  for (int i = 1; i < kW; ++i) m = fmaxf(m, sh[i]);
  m *= kLog2e;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = threadIdx.x + kT * j;
    if (c >= nch) continue;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int col = 8 * c + 2 * k;
      if (col < V) s += __builtin_amdgcn_exp2f(lo2f(q[j][k]) * kLog2e - m);
      if (col + 1 < V) s += __builtin_amdgcn_exp2f(hi2f(q[j][k]) * kLog2e - m);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) sh[kW + (threadIdx.x >> 6)] = s;
  __syncthreads();
  s = 0.f;
#pragma unroll
  for (int i = 0; i < kW; ++i) s += sh[kW + i];
  const float l2 = m + log2f(s);  // log2-domain lse
  if (threadIdx.x == 0) {
    lse[row] = l2 * kLn2;
    loss[row] = l2 * kLn2 - xt;  // xt = 0 for an out-of-range target, as in xent_fwd_k
  }
  const float sc = gscale[0] * inv_n;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = threadIdx.x + kT * j;
    if (c >= nch) continue;
    float g[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      g[2 * k] = __builtin_amdgcn_exp2f(lo2f(q[j][k]) * kLog2e - l2);
      g[2 * k + 1] = __builtin_amdgcn_exp2f(hi2f(q[j][k]) * kLog2e - l2);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = 8 * c + e;
      g[e] = col >= V ? 0.f : (g[e] - (col == t ? 1.f : 0.f)) * sc;
    }
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = pack2(g[2 * k], g[2 * k + 1]);
    reinterpret_cast<u32x4*>(L)[c] = o;
  }
}

// ============================================================== AdamW
__global__ __launch_bounds__(256) void sumsq_k(const u16* __restrict__ g, int64_t n8, float* __restrict__ out) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const u32x4 a = reinterpret_cast<const u32x4*>(g)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x0 = lo2f(a[k]), x1 = hi2f(a[k]);
      s += x0 * x0 + x1 * x1;
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (sh[0] + sh[1]) + (sh[2] + sh[3]));
}

__global__ __launch_bounds__(256) void adamw_k(float* __restrict__ p, const u16* __restrict__ g,
                                               float* __restrict__ m, float* __restrict__ v, u16* __restrict__ w16,
                                               int64_t n4, const float* __restrict__ lr_p,
                                               const float* __restrict__ step_p, float b1, float b2, float eps,
                                               float wd, const float* __restrict__ sumsq, float max_norm) {
  const float lr = lr_p[0], t = step_p[0];
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1, rbc2 = rsqrtf(bc2), decay = 1.f - lr * wd;
  float clip = 1.f;
  if (max_norm > 0.f) clip = fminf(1.f, max_norm / (sqrtf(sumsq[0]) + 1e-6f));
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    const u32x2 gg = reinterpret_cast<const u32x2*>(g)[i];
    const float gr[4] = {lo2f(gg[0]) * clip, hi2f(gg[0]) * clip, lo2f(gg[1]) * clip, hi2f(gg[1]) * clip};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] = b1 * mm[k] + (1.f - b1) * gr[k];
      vv[k] = b2 * vv[k] + (1.f - b2) * gr[k] * gr[k];
      pp[k] = pp[k] * decay - step_size * mm[k] / (sqrtf(vv[k]) * rbc2 + eps);
    }
    reinterpret_cast<f32x4*>(p)[i] = pp;
    reinterpret_cast<f32x4*>(m)[i] = mm;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    reinterpret_cast<u32x2*>(w16)[i] = u32x2{pack2(pp[0], pp[1]), pack2(pp[2], pp[3])};
  }
}

// ============================================================== column sums / split-K partial reduction
// out[c] = bf16(sum_r part[r][c]); n % 4 == 0
__global__ __launch_bounds__(256) void reduce_rows_k(const float* __restrict__ part, int R, int64_t n,
                                                     u16* __restrict__ out) {
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 s = reinterpret_cast<const f32x4*>(part)[i];
#pragma unroll 8
    for (int r = 1; r < R; ++r) s += reinterpret_cast<const f32x4*>(part + (int64_t)r * n)[i];
    reinterpret_cast<u32x2*>(out)[i] = u32x2{pack2(s[0], s[1]), pack2(s[2], s[3])};
  }
}

// part[chunk][c] = sum over the chunk's rows of x[r][c]; block = 16 column vectors (8 bf16) x 16 row groups
__global__ __launch_bounds__(256) void colsum_k(const u16* __restrict__ x, int M, int N, int rows,
                                                float* __restrict__ part) {
  __shared__ f32x4 red[16][16][2];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int cv = blockIdx.x * 16 + tx;
  const int r0 = blockIdx.y * rows, r1 = min(M, r0 + rows);
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a;
  if (cv * 8 < N) {
#pragma unroll 4
    for (int r = r0 + ty; r < r1; r += 16) {
      const u32x4 q = *reinterpret_cast<const u32x4*>(x + (int64_t)r * N + cv * 8);
      a += f32x4{lo2f(q[0]), hi2f(q[0]), lo2f(q[1]), hi2f(q[1])};
      b += f32x4{lo2f(q[2]), hi2f(q[2]), lo2f(q[3]), hi2f(q[3])};
    }
  }
  red[ty][tx][0] = a;
  red[ty][tx][1] = b;
  __syncthreads();
  if (threadIdx.x < 32) {
    const int c = threadIdx.x & 15, h = threadIdx.x >> 4;
    f32x4 s = red[0][c][h];
#pragma unroll
    for (int k = 1; k < 16; ++k) s += red[k][c][h];
    if ((blockIdx.x * 16 + c) * 8 < N) reinterpret_cast<f32x4*>(part + (int64_t)blockIdx.y * N + (blockIdx.x * 16 + c) * 8)[h] = s;
  }
}

// ============================================================== flash attention (head dim 64)
constexpr int HD = 64;
constexpr int LDK = HD + 8;  // LDS row pitch in bf16 (144 B: 16-B padded rows)
constexpr int QB = 128;      // query rows per workgroup (4 waves x 32)
constexpr int KT = 64;       // keys per LDS tile

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ bf16x8 ld8(const u16* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(p));
}
// transposing read: rows r0 + 0..3 and r0 + 16 + 0..3 of columns c0 + 0..15 -> 8 bf16 per lane
// (lane 4q + p of each 16-lane group addresses row q, columns 4p .. 4p + 3)
__device__ __forceinline__ bf16x8 ld_tr(const u16* tile, int r0, int c0, int li) {
  const u16* a = tile + (r0 + (li >> 2)) * LDK + c0 + 4 * (li & 3);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 16 * LDK));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (__bf16)a[0];
  r[1] = (__bf16)a[1];
  r[2] = (__bf16)a[2];
  r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0];
  r[5] = (__bf16)b[1];
  r[6] = (__bf16)b[2];
  r[7] = (__bf16)b[3];
  return r;
}
#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// Stage 64 rows x 64 bf16 of two row-strided sources into LDS tiles (register staged).
struct TileLoader {
  u32x4 r[4];
  __device__ __forceinline__ void load(const u16* s0, const u16* s1, int64_t stride, int row0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = threadIdx.x + 256 * k, which = idx >> 9, rem = idx & 511, row = rem >> 3, ch = rem & 7;
      const u16* s = which ? s1 : s0;
      r[k] = *reinterpret_cast<const u32x4*>(s + (int64_t)(row0 + row) * stride + ch * 8);
    }
  }
  __device__ __forceinline__ void store(u16* t0, u16* t1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = threadIdx.x + 256 * k, which = idx >> 9, rem = idx & 511, row = rem >> 3, ch = rem & 7;
      *reinterpret_cast<u32x4*>((which ? t1 : t0) + row * LDK + ch * 8) = r[k];
    }
  }
};

// grid: (T / QB) * B * H blocks, heaviest (last) query blocks first; block -> bh = id % BH
// keeps all query blocks of one (batch, head) on one XCD group when BH % 8 == 0 (K/V in one L2).
__global__ __launch_bounds__(256) void attn_fwd_k(const u16* __restrict__ qkv, u16* __restrict__ o,
                                                  float* __restrict__ lse, int T, int H, int BH, float c) {
  __shared__ __align__(16) u16 sm[2][2][KT * LDK];
  const int nqb = T / QB;
  const int bh = blockIdx.x % BH, qb = nqb - 1 - blockIdx.x / BH;
  const int b = bh / H, h = bh - b * H;
  const int C = H * HD;
  const int64_t C3 = 3 * C;
  const u16* base = qkv + (int64_t)b * T * C3 + h * HD;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int q0 = qb * QB, q0w = q0 + 32 * w;

  bf16x8 qf[2][2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[r][ks] = ld8(base + (int64_t)(q0w + 16 * r + li) * C3 + 8 * g + 32 * ks);

  float mrow[2] = {-1e30f, -1e30f}, lrow[2] = {0.f, 0.f};
  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) acc[r][mm] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ntiles = (q0 + QB) / KT;
  TileLoader ld;
  ld.load(base + C, base + 2 * C, C3, 0);
  ld.store(sm[0][0], sm[0][1]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, kv0 = t * KT;
    if (t + 1 < ntiles) ld.load(base + C, base + 2 * C, C3, kv0 + KT);
    if (kv0 <= q0w + 31) {
      const u16* Ks = sm[buf][0];
      const u16* Vs = sm[buf][1];
      f32x4 s[2][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        s[0][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        s[1][n] = s[0][n];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = ld8(Ks + (16 * n + li) * LDK + 8 * g + 32 * ks);
          s[0][n] = MFMA(kf, qf[0][ks], s[0][n]);
          s[1][n] = MFMA(kf, qf[1][ks], s[1][n]);
        }
      }
      // Online softmax in the log2 domain, trimmed for the VALU: the mask only on diagonal tiles (a
      // wave-uniform branch), the scale folded into one FMA per score, v_exp_f32 directly (exp2f's
      // denormal range reduction tripled the exp cost; probabilities below 2^-126 are 0 here anyway),
      // and lazy rescaling: the running max moves only when a tile's max exceeds it by more than
      // kLazy (probabilities then stay <= 2^kLazy, safe in fp32 / bf16), so after the first tiles the
      // 32 accumulator rescales of a tile are skipped unless some lane of the wave needs them.
      constexpr float kLazy = 8.f;
      const bool diag = kv0 + KT - 1 > q0w;
      bf16x8 pb[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int q = q0w + 16 * r + li;
        if (diag) {
#pragma unroll
          for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (kv0 + 16 * n + 4 * g + j > q) s[r][n][j] = -INFINITY;
        }
        float mx = -INFINITY;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) mx = fmaxf(mx, s[r][n][j]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mxc = mx * c;  // c > 0: max commutes with the scale
        const float mn = mxc > mrow[r] + kLazy ? mxc : mrow[r];
        const float alpha = __builtin_amdgcn_exp2f(mrow[r] - mn);
        mrow[r] = mn;
        float rs = 0.f;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r][n][j], c, -mn));
            s[r][n][j] = p;
            rs += p;
          }
        rs += __shfl_xor(rs, 16, 64);
        rs += __shfl_xor(rs, 32, 64);
        lrow[r] = lrow[r] * alpha + rs;
        if (__builtin_amdgcn_read_exec() & __ballot(alpha != 1.f)) {
#pragma unroll
          for (int mm = 0; mm < 4; ++mm) acc[r][mm] *= alpha;
        }
        pb[r][0] = pack8(s[r][0], s[r][1]);
        pb[r][1] = pack8(s[r][2], s[r][3]);
      }
#pragma unroll
      for (int mm = 0; mm < 4; ++mm)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 vt = ld_tr(Vs, 32 * ks + 4 * g, 16 * mm, li);
          acc[0][mm] = MFMA(vt, pb[0][ks], acc[0][mm]);
          acc[1][mm] = MFMA(vt, pb[1][ks], acc[1][mm]);
        }
    }
    if (t + 1 < ntiles) ld.store(sm[buf ^ 1][0], sm[buf ^ 1][1]);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int q = q0w + 16 * r + li;
    const float inv = 1.f / lrow[r];
    u16* orow = o + ((int64_t)(b * T + q) * H + h) * HD;
#pragma unroll
    for (int mm = 0; mm < 4; ++mm)
      *reinterpret_cast<u32x2*>(orow + 16 * mm + 4 * g) =
          u32x2{pack2(acc[r][mm][0] * inv, acc[r][mm][1] * inv), pack2(acc[r][mm][2] * inv, acc[r][mm][3] * inv)};
    if (g == 0) lse[(int64_t)bh * T + q] = mrow[r] + log2f(lrow[r]);
  }
}

// delta[bh][q] = sum_d dO * O
__global__ __launch_bounds__(256) void attn_delta_k(const u16* __restrict__ o, const u16* __restrict__ dout,
                                                    float* __restrict__ delta, int T, int H, int64_t n) {
  const int64_t i = blockIdx.x * 256ll + threadIdx.x;  // (b, q, h)
  if (i >= n) return;
  const u32x4* a = reinterpret_cast<const u32x4*>(o + i * HD);
  const u32x4* d = reinterpret_cast<const u32x4*>(dout + i * HD);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < HD / 8; ++k) {
    const u32x4 x = a[k], y = d[k];
#pragma unroll
    for (int e = 0; e < 4; ++e) s += lo2f(x[e]) * lo2f(y[e]) + hi2f(x[e]) * hi2f(y[e]);
  }
  const int h = (int)(i % H);
  const int64_t bq = i / H;
  const int q = (int)(bq % T), b = (int)(bq / T);
  delta[((int64_t)b * H + h) * T + q] = s;
}

// dQ: per query block (like the forward), S^T and dP^T with the query on the lane.
__global__ __launch_bounds__(256) void attn_dq_k(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                 const float* __restrict__ lse, const float* __restrict__ delta,
                                                 u16* __restrict__ dqkv, int T, int H, int BH, float c,
                                                 float sm_scale) {
  __shared__ __align__(16) u16 sm[2][2][KT * LDK];
  const int nqb = T / QB;
  const int bh = blockIdx.x % BH, qb = nqb - 1 - blockIdx.x / BH;
  const int b = bh / H, h = bh - b * H;
  const int C = H * HD;
  const int64_t C3 = 3 * C;
  const u16* base = qkv + (int64_t)b * T * C3 + h * HD;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int q0 = qb * QB, q0w = q0 + 32 * w;

  bf16x8 qf[2][2], df[2][2];
  float lq[2], dq_[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int q = q0w + 16 * r + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[r][ks] = ld8(base + (int64_t)q * C3 + 8 * g + 32 * ks);
      df[r][ks] = ld8(dout + ((int64_t)(b * T + q) * H + h) * HD + 8 * g + 32 * ks);
    }
    lq[r] = lse[(int64_t)bh * T + q];
    dq_[r] = delta[(int64_t)bh * T + q];
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) acc[r][mm] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ntiles = (q0 + QB) / KT;
  TileLoader ld;
  ld.load(base + C, base + 2 * C, C3, 0);
  ld.store(sm[0][0], sm[0][1]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, kv0 = t * KT;
    if (t + 1 < ntiles) ld.load(base + C, base + 2 * C, C3, kv0 + KT);
    if (kv0 <= q0w + 31) {
      const u16* Ks = sm[buf][0];
      const u16* Vs = sm[buf][1];
      f32x4 s[2][4], dp[2][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        s[0][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        s[1][n] = s[0][n];
        dp[0][n] = s[0][n];
        dp[1][n] = s[0][n];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kf = ld8(Ks + (16 * n + li) * LDK + 8 * g + 32 * ks);
          const bf16x8 vf = ld8(Vs + (16 * n + li) * LDK + 8 * g + 32 * ks);
          s[0][n] = MFMA(kf, qf[0][ks], s[0][n]);
          s[1][n] = MFMA(kf, qf[1][ks], s[1][n]);
          dp[0][n] = MFMA(vf, df[0][ks], dp[0][n]);
          dp[1][n] = MFMA(vf, df[1][ks], dp[1][n]);
        }
      }
      const bool diag = kv0 + KT - 1 > q0w;
      bf16x8 dsb[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int q = q0w + 16 * r + li;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r][n][j], c, -lq[r]));  // v_exp_f32, see attn_fwd_k
            if (diag && kv0 + 16 * n + 4 * g + j > q) p = 0.f;
            s[r][n][j] = p * (dp[r][n][j] - dq_[r]);
          }
        dsb[r][0] = pack8(s[r][0], s[r][1]);
        dsb[r][1] = pack8(s[r][2], s[r][3]);
      }
#pragma unroll
      for (int mm = 0; mm < 4; ++mm)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 kt = ld_tr(Ks, 32 * ks + 4 * g, 16 * mm, li);
          acc[0][mm] = MFMA(kt, dsb[0][ks], acc[0][mm]);
          acc[1][mm] = MFMA(kt, dsb[1][ks], acc[1][mm]);
        }
    }
    if (t + 1 < ntiles) ld.store(sm[buf ^ 1][0], sm[buf ^ 1][1]);
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int q = q0w + 16 * r + li;
    u16* drow = dqkv + ((int64_t)b * T + q) * C3 + h * HD;
#pragma unroll
    for (int mm = 0; mm < 4; ++mm)
      *reinterpret_cast<u32x2*>(drow + 16 * mm + 4 * g) =
          u32x2{pack2(acc[r][mm][0] * sm_scale, acc[r][mm][1] * sm_scale),
                pack2(acc[r][mm][2] * sm_scale, acc[r][mm][3] * sm_scale)};
  }
}

// dK, dV: per key block of 128 (4 waves x 32 keys), sweeping the query tiles at or after it.
// S and dP are computed with the key on the lane, so P and dS are directly the B operands of
// dV^T += dO^T P and dK^T += Q^T dS; dO^T and Q^T come from transposing LDS reads.
__global__ __launch_bounds__(256) void attn_dkdv_k(const u16* __restrict__ qkv, const u16* __restrict__ dout,
                                                   const float* __restrict__ lse, const float* __restrict__ delta,
                                                   u16* __restrict__ dqkv, int T, int H, int BH, float c,
                                                   float sm_scale) {
  __shared__ __align__(16) u16 sm[2][2][KT * LDK];
  __shared__ __align__(16) float rowc[2][2][KT];  // [buf][lse, delta][q]
  const int bh = blockIdx.x % BH, kb = blockIdx.x / BH;  // key block 0 (most query tiles) first
  const int b = bh / H, h = bh - b * H;
  const int C = H * HD;
  const int64_t C3 = 3 * C;
  const u16* base = qkv + (int64_t)b * T * C3 + h * HD;
  const u16* dbase = dout + (int64_t)b * T * C + h * HD;
  const float* lrow = lse + (int64_t)bh * T;
  const float* drow = delta + (int64_t)bh * T;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int k0w = kb * QB + 32 * w;

  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int64_t off = (int64_t)(k0w + 16 * cc + li) * C3 + 8 * g + 32 * ks;
      kf[cc][ks] = ld8(base + C + off);
      vf[cc][ks] = ld8(base + 2 * C + off);
    }
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      dk[cc][mm] = f32x4{0.f, 0.f, 0.f, 0.f};
      dv[cc][mm] = dk[cc][mm];
    }

  const int t0 = kb * QB / KT, ntiles = T / KT;
  TileLoader ld;
  float rc = 0.f;
  auto load_rc = [&](int q0) {
    if (threadIdx.x < 2 * KT) rc = (threadIdx.x < KT ? lrow : drow)[q0 + (threadIdx.x & (KT - 1))];
  };
  auto store_rc = [&](int buf) {
    if (threadIdx.x < 2 * KT) rowc[buf][threadIdx.x >> 6][threadIdx.x & (KT - 1)] = rc;
  };
  {
    const int q0 = t0 * KT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = threadIdx.x + 256 * k, which = idx >> 9, rem = idx & 511, row = rem >> 3, ch = rem & 7;
      ld.r[k] = which ? *reinterpret_cast<const u32x4*>(dbase + (int64_t)(q0 + row) * C + ch * 8)
                      : *reinterpret_cast<const u32x4*>(base + (int64_t)(q0 + row) * C3 + ch * 8);
    }
    load_rc(q0);
  }
  ld.store(sm[0][0], sm[0][1]);
  store_rc(0);
  __syncthreads();
  for (int t = t0; t < ntiles; ++t) {
    const int buf = (t - t0) & 1, q0t = t * KT;
    if (t + 1 < ntiles) {
      const int q1 = q0t + KT;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = threadIdx.x + 256 * k, which = idx >> 9, rem = idx & 511, row = rem >> 3, ch = rem & 7;
        ld.r[k] = which ? *reinterpret_cast<const u32x4*>(dbase + (int64_t)(q1 + row) * C + ch * 8)
                        : *reinterpret_cast<const u32x4*>(base + (int64_t)(q1 + row) * C3 + ch * 8);
      }
      load_rc(q1);
    }
    if (q0t + KT - 1 >= k0w) {
      const u16* Qs = sm[buf][0];
      const u16* Ds = sm[buf][1];
      f32x4 s[2][4], dp[2][4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        s[0][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        s[1][n] = s[0][n];
        dp[0][n] = s[0][n];
        dp[1][n] = s[0][n];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 qa = ld8(Qs + (16 * n + li) * LDK + 8 * g + 32 * ks);
          const bf16x8 da = ld8(Ds + (16 * n + li) * LDK + 8 * g + 32 * ks);
          s[0][n] = MFMA(qa, kf[0][ks], s[0][n]);
          s[1][n] = MFMA(qa, kf[1][ks], s[1][n]);
          dp[0][n] = MFMA(da, vf[0][ks], dp[0][n]);
          dp[1][n] = MFMA(da, vf[1][ks], dp[1][n]);
        }
      }
      const bool diag = q0t < k0w + 31;
      bf16x8 pb[2][2], dsb[2][2];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const f32x4 lq = *reinterpret_cast<const f32x4*>(&rowc[buf][0][16 * n + 4 * g]);
        const f32x4 dq = *reinterpret_cast<const f32x4*>(&rowc[buf][1][16 * n + 4 * g]);
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
          const int key = k0w + 16 * cc + li;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[cc][n][j], c, -lq[j]));
            if (diag && key > q0t + 16 * n + 4 * g + j) p = 0.f;
            s[cc][n][j] = p;
            dp[cc][n][j] = p * (dp[cc][n][j] - dq[j]);
          }
        }
      }
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        pb[cc][0] = pack8(s[cc][0], s[cc][1]);
        pb[cc][1] = pack8(s[cc][2], s[cc][3]);
        dsb[cc][0] = pack8(dp[cc][0], dp[cc][1]);
        dsb[cc][1] = pack8(dp[cc][2], dp[cc][3]);
      }
#pragma unroll
      for (int mm = 0; mm < 4; ++mm)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 dt = ld_tr(Ds, 32 * ks + 4 * g, 16 * mm, li);
          const bf16x8 qt = ld_tr(Qs, 32 * ks + 4 * g, 16 * mm, li);
          dv[0][mm] = MFMA(dt, pb[0][ks], dv[0][mm]);
          dv[1][mm] = MFMA(dt, pb[1][ks], dv[1][mm]);
          dk[0][mm] = MFMA(qt, dsb[0][ks], dk[0][mm]);
          dk[1][mm] = MFMA(qt, dsb[1][ks], dk[1][mm]);
        }
    }
    if (t + 1 < ntiles) {
      ld.store(sm[buf ^ 1][0], sm[buf ^ 1][1]);
      store_rc(buf ^ 1);
    }
    __syncthreads();
  }
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    const int key = k0w + 16 * cc + li;
    u16* krow = dqkv + ((int64_t)b * T + key) * C3 + h * HD;
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      *reinterpret_cast<u32x2*>(krow + C + 16 * mm + 4 * g) =
          u32x2{pack2(dk[cc][mm][0] * sm_scale, dk[cc][mm][1] * sm_scale),
                pack2(dk[cc][mm][2] * sm_scale, dk[cc][mm][3] * sm_scale)};
      *reinterpret_cast<u32x2*>(krow + 2 * C + 16 * mm + 4 * g) =
          u32x2{pack2(dv[cc][mm][0], dv[cc][mm][1]), pack2(dv[cc][mm][2], dv[cc][mm][3])};
    }
  }
}

inline int grid_for(int64_t n, int per_thread) {
  const int64_t b = (n / per_thread + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

}  // namespace

hipError_t ln_fwd(const float* x32, const bf16* r, float* xo, const bf16* gamma, const bf16* beta, bf16* y,
                  float* mean, float* rstd, int M, int D, float eps, hipStream_t st) {
  const dim3 grid((M + 3) / 4), blk(256);
  const u16* rr = reinterpret_cast<const u16*>(r);
  const u16* gg = reinterpret_cast<const u16*>(gamma);
  const u16* bb = reinterpret_cast<const u16*>(beta);
  u16* yy = reinterpret_cast<u16*>(y);
  switch (D / 256) {
#define LN_CASE(V) \
  case V: hipLaunchKernelGGL(ln_fwd_k<V>, grid, blk, 0, st, x32, rr, xo, gg, bb, yy, mean, rstd, M, eps); break;
    LN_CASE(1) LN_CASE(2) LN_CASE(3) LN_CASE(4) LN_CASE(5) LN_CASE(6) LN_CASE(8)
#undef LN_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// (one workgroup per CU: the partial rows stay few for ln_reduce_k; each wave keeps two rows in flight,
// see ln_bwd_k).
int ln_bwd_blocks(int M) { return (M + 3) / 4 < kLnBwdBlocks ? (M + 3) / 4 : kLnBwdBlocks; }

hipError_t ln_bwd(const bf16* dy, const float* xin, const float* mean, const float* rstd, const bf16* gamma,
                  const float* dres, float* dx, bf16* dr, float* part_g, float* part_b, int M, int D,
                  hipStream_t st, float* part_r) {
  const dim3 grid(ln_bwd_blocks(M)), blk(256);
  const u16* d = reinterpret_cast<const u16*>(dy);
  const u16* gg = reinterpret_cast<const u16*>(gamma);
  u16* rr = reinterpret_cast<u16*>(dr);
  switch (D / 256) {
#define LN_CASE(V) \
  case V:          \
    hipLaunchKernelGGL(ln_bwd_k<V>, grid, blk, 0, st, d, xin, mean, rstd, gg, dres, dx, rr, part_g, part_b, part_r, M); \
    break;
    LN_CASE(1) LN_CASE(2) LN_CASE(3) LN_CASE(4) LN_CASE(5) LN_CASE(6) LN_CASE(8)
#undef LN_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t ln_reduce_params(const float* part_g, const float* part_b, int nblk, int D, bf16* dgamma, bf16* dbeta,
                            hipStream_t st, const float* part_r, bf16* dbias) {
  hipLaunchKernelGGL(ln_reduce_k, dim3((D + 63) / 64), dim3(64 * kLnRedGroups), 0, st, part_g, part_b, part_r, nblk, D,
                     reinterpret_cast<u16*>(dgamma), reinterpret_cast<u16*>(dbeta), reinterpret_cast<u16*>(dbias));
  return hipGetLastError();
}

hipError_t gelu_fwd(const bf16* u, bf16* g, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(gelu_fwd_k, dim3(grid_for(n, 8)), dim3(256), 0, st, reinterpret_cast<const u16*>(u),
                     reinterpret_cast<u16*>(g), n / 8);
  return hipGetLastError();
}

hipError_t gelu_bwd(const bf16* u, const bf16* dy, bf16* du, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(gelu_bwd_k, dim3(grid_for(n, 8)), dim3(256), 0, st, reinterpret_cast<const u16*>(u),
                     reinterpret_cast<const u16*>(dy), reinterpret_cast<u16*>(du), n / 8);
  return hipGetLastError();
}

hipError_t xent_fwd(const bf16* logits, const int64_t* tgt, float* loss, float* lse, int N, int V, int Vp,
                    hipStream_t st) {
  hipLaunchKernelGGL(xent_fwd_k, dim3(N), dim3(256), 0, st, reinterpret_cast<const u16*>(logits), tgt, loss, lse, V,
                     Vp);
  return hipGetLastError();
}

hipError_t xent_eval(const bf16* logits, const int64_t* tgt, float* loss, float* hit, int N, int V, int Vp,
                     hipStream_t st) {
  hipLaunchKernelGGL(xent_eval_k, dim3(N), dim3(256), 0, st, reinterpret_cast<const u16*>(logits), tgt, loss, hit, V,
                     Vp);
  return hipGetLastError();
}

hipError_t xent_bwd(bf16* logits, const int64_t* tgt, const float* lse, const float* gscale, float inv_n, int N,
                    int V, int Vp, hipStream_t st) {
  hipLaunchKernelGGL(xent_bwd_k, dim3(N), dim3(256), 0, st, reinterpret_cast<u16*>(logits), tgt, lse, gscale, inv_n,
                     V, Vp);
  return hipGetLastError();
}

hipError_t xent_fused(bf16* logits, const int64_t* tgt, float* loss, float* lse, const float* gscale, float inv_n,
                      int N, int V, int Vp, hipStream_t st) {
  const int nch = Vp / 8;
  u16* L = reinterpret_cast<u16*>(logits);
  if (nch <= 512 * 4)
    hipLaunchKernelGGL(xent_fused_k<4>, dim3(N), dim3(512), 0, st, L, tgt, loss, lse, gscale, inv_n, V, Vp);
  else if (nch <= 512 * 13)
    hipLaunchKernelGGL(xent_fused_k<13>, dim3(N), dim3(512), 0, st, L, tgt, loss, lse, gscale, inv_n, V, Vp);
  else
    return hipErrorInvalidValue;  // wider vocabularies: the two-pass kernels
  return hipGetLastError();
}

hipError_t grad_sumsq(const bf16* g, int64_t n, float* sumsq, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_k, dim3(grid_for(n, 8)), dim3(256), 0, st, reinterpret_cast<const u16*>(g), n / 8, sumsq);
  return hipGetLastError();
}

hipError_t adamw(float* p, const bf16* g, float* m, float* v, bf16* w16, int64_t n, const float* lr,
                 const float* step, float beta1, float beta2, float eps, float wd, const float* sumsq,
                 float max_norm, hipStream_t st) {
  hipLaunchKernelGGL(adamw_k, dim3(grid_for(n, 4)), dim3(256), 0, st, p, reinterpret_cast<const u16*>(g), m, v,
                     reinterpret_cast<u16*>(w16), n / 4, lr, step, beta1, beta2, eps, wd, sumsq, max_norm);
  return hipGetLastError();
}

hipError_t reduce_rows(const float* part, int R, int64_t n, bf16* out, hipStream_t st) {
  hipLaunchKernelGGL(reduce_rows_k, dim3(grid_for(n, 4)), dim3(256), 0, st, part, R, n, reinterpret_cast<u16*>(out));
  return hipGetLastError();
}

int colsum_chunks(int M, int N) {
  const int cb = (N / 8 + 15) / 16;
  int R = 1024 / cb;
  R = R < 1 ? 1 : (R > 64 ? 64 : R);
  const int max_r = (M + 15) / 16;  // >= 16 rows per chunk
  return R > max_r ? max_r : R;
}

hipError_t colsum(const bf16* x, int M, int N, float* part, bf16* out, hipStream_t st) {
  const int R = colsum_chunks(M, N), rows = (M + R - 1) / R;
  hipLaunchKernelGGL(colsum_k, dim3((N / 8 + 15) / 16, R), dim3(256), 0, st, reinterpret_cast<const u16*>(x), M, N,
                     rows, part);
  return reduce_rows(part, R, N, out, st);
}

hipError_t attn_fwd(const bf16* qkv, bf16* o, float* lse, int B, int T, int H, float sm_scale, hipStream_t st) {
  const int BH = B * H;
  hipLaunchKernelGGL(attn_fwd_k, dim3((T / QB) * BH), dim3(256), 0, st, reinterpret_cast<const u16*>(qkv),
                     reinterpret_cast<u16*>(o), lse, T, H, BH, sm_scale * kLog2e);
  return hipGetLastError();
}

hipError_t attn_bwd(const bf16* qkv, const bf16* o, const bf16* dout, const float* lse, float* delta, bf16* dqkv,
                    int B, int T, int H, float sm_scale, hipStream_t st) {
  const int BH = B * H;
  const int64_t n = (int64_t)B * T * H;
  const u16* q = reinterpret_cast<const u16*>(qkv);
  const u16* d = reinterpret_cast<const u16*>(dout);
  u16* dq = reinterpret_cast<u16*>(dqkv);
  hipLaunchKernelGGL(attn_delta_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const u16*>(o), d, delta, T, H, n);
  hipLaunchKernelGGL(attn_dkdv_k, dim3((T / QB) * BH), dim3(256), 0, st, q, d, lse, delta, dq, T, H, BH,
                     sm_scale * kLog2e, sm_scale);
  hipLaunchKernelGGL(attn_dq_k, dim3((T / QB) * BH), dim3(256), 0, st, q, d, lse, delta, dq, T, H, BH,
                     sm_scale * kLog2e, sm_scale);
  return hipGetLastError();
}

}  // namespace tfm
}  // namespace katib_hip
