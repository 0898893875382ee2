// DARTS supernet edge kernels for CDNA4 (gfx950), fp32 NCHW.
//
// One MixedOp edge (reference operations.py:164-180) costs ~100+ tiny kernels
// through PyTorch/MIOpen at C=4..64 channels (per-sample im2col loops, 50-80 us
// BN reductions over 4 channels). Here an edge is ~7 forward / ~12 backward
// launches:
//
//   dwpw_fwd    ReLU (or BN-apply+ReLU of the previous stage) -> depthwise KxK
//               (stride, dilation) -> pointwise 1x1, input tile + halo staged in
//               LDS, depthwise result kept in LDS, pointwise on MFMA
//               (v_mfma_f32_16x16x4_f32) when C % 16 == 0, per-channel BN
//               statistics (sum, sum of squares) reduced in-wave and added with
//               one fp64 atomic per channel per wave.
//   pool_fwd    avg (count_include_pad=False) + max 3x3 in one pass + stats.
//   pw_fwd      ReLU -> 1x1 conv (StdConv / FactorizedReduce halves) + stats.
//   combine_fwd out = sum_k w_k * BN_k(z_k) + w_id * x, running-stat update.
//   *_bwd       BN backward evaluated on the fly from the reductions of
//               combine_bwd_reduce, pointwise-transpose, transposed depthwise,
//               weight gradients accumulated into the flat gradient buffer with
//               float atomics (one per weight per block).
//
// All shapes are checked on the host (darts_bind.cpp) before launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "darts_ops.h"

namespace katib_hip {

// Persistent grids: 2 blocks per CU. Cross-block sums are accumulated per block in LDS
// and flushed as ONE lane-contiguous atomic vector per block - global float atomics
// execute memory-side, and many single-lane adds to the same address serialise
// (MI355X_MICROARCH.md "Global float atomics").
// Cap tunable with KATIB_HIP_MAX_BLOCKS (host side, read once).
static int g_max_blocks = 0;
int max_blocks() {
  if (g_max_blocks <= 0) {
    const char* e = getenv("KATIB_HIP_MAX_BLOCKS");
    g_max_blocks = e ? std::max(1, atoi(e)) : 2048;
  }
  return g_max_blocks;
}
void set_max_blocks(int n) { g_max_blocks = n; }

// 4-pixels-per-thread output paths of the plane kernels, per channel group (KATIB_HIP_VEC_MASK,
// read once): bit 0 dwpw_plane C = 4, bit 1 dwpw_plane C = 8, bit 2 dw_bwd_plane C = 4, bit 3
// dw_bwd_plane C = 8. Default C = 4 only: at C = 8 the four-pixel register arrays cost more than the
// wider stores save (profiles/darts_vec_ab_r04.log).
static int vec_mask() {
  static const int m = getenv("KATIB_HIP_VEC_MASK") ? atoi(getenv("KATIB_HIP_VEC_MASK")) : 0x5;
  return m;
}

// s += p[r*rs], s2 += p[r*rs + off2] over r < rep replicas, 8 replicas (16 loads) in flight per
// step instead of one dependent load-add per replica
__device__ __forceinline__ void sum_replicas(const double* p, int rep, int rs, int off2, double& s, double& s2) {
  s = 0.0;
  s2 = 0.0;
  for (int r0 = 0; r0 < rep; r0 += 8) {
    double a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool ok = r0 + u < rep;
      a[u] = ok ? p[(size_t)(r0 + u) * rs] : 0.0;
      b[u] = ok ? p[(size_t)(r0 + u) * rs + off2] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s += a[u];
      s2 += b[u];
    }
  }
}

// batch mean / biased variance of channel c from the replicated (sum, sum of squares)
__device__ __forceinline__ void bn_moments(const BNRef& b, int c, double& m, double& v) {
  double s, s2;
  sum_replicas(b.sums + c, b.rep, b.rstride, b.C, s, s2);
  m = s * (double)b.inv_count;
  v = s2 * (double)b.inv_count - m * m;
  if (v < 0) v = 0;
}

__device__ __forceinline__ void bn_coeffs(const BNRef& b, int c, float& mean, float& invstd) {
  if (b.eval) {
    mean = b.rmean[c];
    invstd = rsqrtf(b.rvar[c] + b.eps);
  } else {
    double m, v;
    bn_moments(b, c, m, v);
    mean = (float)m;
    invstd = rsqrtf((float)v + b.eps);
  }
}

// per-channel means of the BN-backward reductions: m1 = mean(g), m2 = mean(g * zhat)
__device__ __forceinline__ void gs_means(const GradSrc& gs, int c, float& m1, float& m2) {
  if (gs.eval) {
    m1 = m2 = 0.f;
    return;
  }
  double s1 = 0.0, s2 = 0.0;
  if (gs.rep == 1) {
    s1 = gs.S1[c];
    s2 = gs.S2[c];
  } else {
    sum_replicas(gs.S1 + c, gs.rep, gs.rstride, (int)(gs.S2 - gs.S1), s1, s2);
  }
  m1 = (float)(s1 * (double)gs.bn.inv_count);
  m2 = (float)(s2 * (double)gs.bn.inv_count);
}

// Workgroup-cooperative replica sums for a kernel prologue (called by EVERY thread; the caller
// barriers before reading the outputs): channel ch of [0, n) of the pair (p1, p2) summed over
// `rep` replicas (rs doubles apart) by 16 lanes each - every lane's loads in flight at once and
// a 4-step shuffle tree, instead of one thread walking all replicas. This is what lets a
// consumer read unfolded statistics at the latency of one global round trip, so the separate
// fold launch in front of it can go.
__device__ __forceinline__ void coop_pair_sums(const double* p1, const double* p2, int rep, int rs, int n,
                                               double scale, float* o1, float* o2, bool bn, float eps) {
  const int tid = threadIdx.x, j = tid & 15;
  for (int cb = 0; cb < n; cb += 16) {
    const int ch = cb + (tid >> 4);
    double s = 0.0, s2 = 0.0;
    if (ch < n) {
#pragma unroll 2
      for (int r = j; r < rep; r += 16) {
        s += p1[(size_t)r * rs + ch];
        s2 += p2[(size_t)r * rs + ch];
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      s += __shfl_xor(s, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (ch < n && j == 0) {
      if (bn) {  // (sum, sum of squares) -> (mean, 1 / std) as bn_coeffs
        const double m = s * scale;
        double v = s2 * scale - m * m;
        if (v < 0) v = 0;
        o1[ch] = (float)m;
        o2[ch] = rsqrtf((float)v + eps);
      } else {  // BN-backward sums -> means as gs_means
        o1[ch] = (float)(s * scale);
        o2[ch] = (float)(s2 * scale);
      }
    }
  }
}

// BN coefficients of channels [c0, c0 + n) into mean[0..n), inv[0..n) (every thread calls)
__device__ __forceinline__ void bn_coeffs_coop(const BNRef& b, int c0, int n, float* mean, float* inv) {
  if (b.eval || b.rep == 1) {
    for (int c = threadIdx.x; c < n; c += blockDim.x) bn_coeffs(b, c0 + c, mean[c], inv[c]);
    return;
  }
  coop_pair_sums(b.sums + c0, b.sums + b.C + c0, b.rep, b.rstride, n, (double)b.inv_count, mean, inv, true, b.eps);
}

// BN-backward means of channels [c0, c0 + n) into m1[0..n), m2[0..n) (every thread calls)
__device__ __forceinline__ void gs_means_coop(const GradSrc& gs, int c0, int n, float* m1, float* m2) {
  if (gs.eval || gs.rep == 1) {
    for (int c = threadIdx.x; c < n; c += blockDim.x) gs_means(gs, c0 + c, m1[c], m2[c]);
    return;
  }
  coop_pair_sums(gs.S1 + c0, gs.S2 + c0, gs.rep, gs.rstride, n, (double)gs.bn.inv_count, m1, m2, false, 0.f);
}

__device__ __forceinline__ int rep_slot() { return blockIdx.x % kRep; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Reduce-scatter of M per-lane accumulators across the wave (M a power of two <= 64): at each
// butterfly step a lane keeps half of its values and sends the other half to its partner, so
// after log2(M) steps every lane holds one partial and the remaining 6 - log2(M) steps finish
// the sum: M - 1 + 6 - log2(M) shuffles instead of 6 * M for M separate wave sums. Returns the
// total of accumulator wave_scatter_index<M>(lane) (identical on the 64 / M lanes sharing it).
// (each butterfly level is its own instantiation so every register index is a constant: a
// runtime-bounded level loop made the compiler move the accumulators to scratch)
template <int H, int D>
__device__ __forceinline__ void reduce_scatter_level(float* acc, int lane) {
  if constexpr (H >= 1) {
    const bool up = (lane & D) != 0;  // upper partner keeps the upper half
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float keep = up ? acc[i + H] : acc[i];
      const float send = up ? acc[i] : acc[i + H];
      acc[i] = keep + __shfl_xor(send, D, 64);
    }
    reduce_scatter_level<H / 2, D / 2>(acc, lane);
  }
}

template <int M>
__device__ __forceinline__ float wave_reduce_scatter(float* acc) {
  const int lane = threadIdx.x & 63;
  reduce_scatter_level<M / 2, 32>(acc, lane);
  float v = acc[0];
#pragma unroll
  for (int d = 32 / M; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// accumulator index lane's wave_reduce_scatter<M> result belongs to (lane bits 5, 4, ... select
// the upper / lower halves in turn)
template <int M>
__device__ __forceinline__ int wave_scatter_index(int lane) {
  int idx = 0;
#pragma unroll
  for (int h = M / 2, d = 32; h >= 1; h >>= 1, d >>= 1)
    if (lane & d) idx += h;
  return idx;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// An edge-kernel input that is either a node state (fp32) or the previous stage's z (zt, Z = true):
// one element / four consecutive elements (i a multiple of 4, 16-byte-aligned base) as fp32
template <bool Z>
__device__ __forceinline__ float xval(const void* p, size_t i) {
  if constexpr (Z) return z2f(static_cast<const zt*>(p)[i]);
  else return static_cast<const float*>(p)[i];
}
template <bool Z>
__device__ __forceinline__ float4 xval4(const void* p, size_t i) {
  if constexpr (Z) {
    const zf4 t = zld4(static_cast<const zt*>(p) + i);
    return make_float4(t.x, t.y, t.z, t.w);
  } else {
    return *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
  }
}

// Self-fold epilogue (darts_ops.h FoldTail). Called by EVERY thread of EVERY workgroup of the
// launch, after the workgroup's last replica atomic. The arrival add is relaxed: the payload is
// device-scope atomics (performed memory-side), drained by each wave's vmcnt(0) before the
// workgroup barrier, and the folding workgroup reads it back with returning atomics only, so no
// release / acquire fence (an XCD L2 write-back per workgroup) is needed.
__device__ __forceinline__ void fold_tail(const FoldTail& t) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    // two-level arrival: same-address atomics serialise memory-side (~12 ns each), so ~2000
    // workgroups on one counter cost ~25 us; kFoldShards shard counters (own 128-B lines) cut
    // the chain to total / kFoldShards, and each shard's last arriver adds to the top counter
    const unsigned total = gridDim.x * gridDim.y * gridDim.z;
    const unsigned L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const unsigned sh = L % kFoldShards;
    const unsigned cnt = total / kFoldShards + (sh < total % kFoldShards ? 1u : 0u);
    unsigned* cs = t.ctr + (1 + sh) * kFoldCtrStride;
    int last = 0;
    if (__hip_atomic_fetch_add(cs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == cnt - 1) {
      __hip_atomic_store(cs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm the shard
      const unsigned nsh = total < (unsigned)kFoldShards ? total : (unsigned)kFoldShards;
      last = __hip_atomic_fetch_add(t.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  int tot = 0;
  for (int s = 0; s < t.nseg; ++s) tot += t.n[s];
  for (int g = threadIdx.x; g < tot; g += blockDim.x) {
    int s = 0, i = g;
    while (i >= t.n[s]) i -= t.n[s++];
    double* p = t.p[s] + i;
    const size_t rs = t.rs[s];
    double v[kRep - 1];
#pragma unroll
    for (int r = 1; r < kRep; ++r)  // all exchanges in flight together
      v[r - 1] = __hip_atomic_exchange(p + r * rs, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < kRep - 1; ++r) acc += v[r];
    __hip_atomic_fetch_add(p, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) __hip_atomic_store(t.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// dwpw_fwd: z = pw . dw(act(in)), d = dw(act(in)); act = relu(x) or relu(BN(x))
// grid: N * (Ho / TR) blocks, 256 threads. P = TR * Wo == 64 (host-enforced)
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, bool PREBN>
__global__ void __launch_bounds__(256) dwpw_fwd_kernel(DwPwFwdBatch bt) {
  const DwPwFwdArgs& a = bt.e[blockIdx.y];
  constexpr int P = 64;
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int TR = P / Wo;
  const int tiles = Ho / TR;
  const int ntiles = a.N * tiles;
  const int pad = a.pad;
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (Wo - 1) * S + (K - 1) * DIL + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sD = smem;                       // [C][P]
  float* sIn = smem + C * P;              // [CH][IR][IW]
  float* sMean = sIn + a.chunk * IR * IW;  // [C]
  float* sInv = sMean + C;                 // [C]
  float* sStat = sInv + C;                 // [2C] block-local (sum, sum of squares)
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  for (int c = tid; c < C; c += 256) {
    if (PREBN) bn_coeffs(a.inbn, c, sMean[c], sInv[c]);
    sStat[c] = 0.f;
    sStat[C + c] = 0.f;
  }
  __syncthreads();
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / tiles, oy0 = (t % tiles) * TR;
    const int iy0 = oy0 * S - pad, ix0 = -pad;
    const size_t xin = (size_t)n * C * H * W;
    for (int c0 = 0; c0 < C; c0 += a.chunk) {
      const int cn = min(a.chunk, C - c0);
      const int tot = cn * IR * IW;
      #pragma unroll 4  // keep several global loads of the staging pass in flight
      for (int i = tid; i < tot; i += 256) {
        int cc = i / (IR * IW), r = (i / IW) % IR, q = i % IW;
        int iy = iy0 + r, ix = ix0 + q, c = c0 + cc;
        float v = 0.f;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
          v = xval<PREBN>(a.x, xin + ((size_t)c * H + iy) * W + ix);
          if (PREBN) v = (v - sMean[c]) * sInv[c];
          v = fmaxf(v, 0.f);
        }
        sIn[i] = v;
      }
      __syncthreads();
      for (int i = tid; i < cn * P; i += 256) {
        const int cc = __builtin_amdgcn_readfirstlane(i / P);  // wave-uniform: weights via scalar loads
        const int p = i % P;
        const int c = c0 + cc;
        int ty = p / Wo, tx = p % Wo;
        const float* wk = a.dw + c * K * K;
        const float* src = sIn + (cc * IR + ty * S) * IW + tx * S;
        float acc = 0.f;
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
          for (int kx = 0; kx < K; ++kx) acc += wk[ky * K + kx] * src[ky * DIL * IW + kx * DIL];
        sD[c * P + p] = acc;
        zput(a.d + (((size_t)n * C + c) * Ho + oy0 + ty) * Wo + tx, acc);
      }
      __syncthreads();
    }
    // pointwise: z[co][p] = sum_ci pw[co][ci] * sD[ci][p]
    if (a.use_mfma) {
      // v_mfma_f32_16x16x4_f32: each wave owns 16 output channels per pass, 4 pixel blocks of 16
      typedef float f4 __attribute__((ext_vector_type(4)));
      for (int cob = wave * 16; cob < C; cob += 64) {
        f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
        for (int k0 = 0; k0 < C; k0 += 4) {
          float av = a.pw[(cob + (lane & 15)) * C + k0 + (lane >> 4)];
#pragma unroll
          for (int pb = 0; pb < 4; ++pb) {
            float bv = sD[(k0 + (lane >> 4)) * P + pb * 16 + (lane & 15)];
            acc[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[pb], 0, 0, 0);
          }
        }
        // C/D map: col (pixel) = lane & 15, row (co) = (lane >> 4) * 4 + r
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int co = cob + (lane >> 4) * 4 + r;
          float s = 0.f, s2 = 0.f;
#pragma unroll
          for (int pb = 0; pb < 4; ++pb) {
            int p = pb * 16 + (lane & 15);
            float v = acc[pb][r];
            zput(a.z + (((size_t)n * C + co) * Ho + oy0 + p / Wo) * Wo + p % Wo, v);
            s += v;
            s2 += v * v;
          }
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) {
            s += __shfl_xor(s, o, 64);
            s2 += __shfl_xor(s2, o, 64);
          }
          if ((lane & 15) == 0) {  // unique owner of channel co in this tile
            sStat[co] += s;
            sStat[C + co] += s2;
          }
        }
      }
    } else {
      for (int co = wave; co < C; co += 4) {
        const int cou = __builtin_amdgcn_readfirstlane(co);
        const float* wrow = a.pw + cou * C;
        float v = 0.f;
        for (int ci = 0; ci < C; ++ci) v += wrow[ci] * sD[ci * P + lane];
        zput(a.z + (((size_t)n * C + cou) * Ho + oy0 + lane / Wo) * Wo + lane % Wo, v);
        float s = wave_sum(v), s2 = wave_sum(v * v);
        if (lane == 0) {
          sStat[cou] += s;
          sStat[C + cou] += s2;
        }
      }
    }
    __syncthreads();  // sD / sIn reuse by the next tile
  }
  if (a.stats)  // one contiguous f64 atomic vector per block
    for (int i = tid; i < 2 * C; i += 256) atomicAdd(a.stats + rep_slot() * 2 * C + i, (double)sStat[i]);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// ------------------------------------------------------------------------------------------------
// dwpw_plane: dwpw_fwd for narrow layers (C <= 8). One workgroup per image: the whole input
// plane of every channel (zero-padded, ReLU / BN-apply+ReLU on the way in) is staged in LDS
// with one coalesced burst, then each thread owns output pixels with ALL channels in registers:
// depthwise KxK from LDS, pointwise C x C in registers, BN statistics per thread, one block
// reduction at the end. Against the 64-pixel tiles (halo rows re-read per tile: 5x the input
// for a dilated 5x5 on 2-row tiles, a barrier-separated load/compute chain per tile) this
// reads each input pixel once and has a single barrier before the compute.
// ------------------------------------------------------------------------------------------------
// PW = false (layers wider than 16 channels): depthwise only, d of C-channel group blockIdx.x % (a.C / C);
// the pointwise then runs as its own GEMM (pw_fwd_wave_kernel)
template <int K, int DIL, int S, bool PREBN, int C, bool VEC, bool PW>
__device__ __forceinline__ void dwpw_plane_body(const DwPwFwdArgs& a, const int bx) {
  constexpr int KK = K * K;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo, pad = a.pad;
  // workgroup = (image n, band of BR output rows); the band's input rows + halo are staged
  const int nb = a.chunk, BR = (Ho + nb - 1) / nb;  // chunk carries the band count
  const int G = PW ? 1 : a.C / C, c0 = PW ? 0 : (bx % G) * C, nbx = PW ? bx : bx / G;
  const int n = nbx / nb, band = nbx - n * nb;
  const int oy0 = band * BR, oy1 = min(Ho, oy0 + BR);
  const int HP = (BR - 1) * S + (K - 1) * DIL + 1, WP = W + 2 * pad, PL = HP * WP;
  const int iyb = oy0 * S - pad;  // input row of staged row 0
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sIn = smem;  // [C][HP][WP]
  __shared__ float sMean[C], sInv[C], sStat[2 * C];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (PREBN) bn_coeffs_coop(a.inbn, c0, C, sMean, sInv);  // the input BN may arrive unfolded (rep > 1)
  if (tid < C) {
    sStat[tid] = 0.f;
    sStat[C + tid] = 0.f;
  }
  __syncthreads();
  const size_t xin = ((size_t)n * a.C + c0) * H * W;
  if (VEC) {
    // 16-byte loads over the band's contiguous in-range rows, scattered into the padded plane;
    // the zero border (rows outside [0, H), pad columns) is written separately
    const int va = max(iyb, 0), vb = min(iyb + HP, H), q4 = (vb - va) * W / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4, r = o / W, ix = o - r * W;
      float4 v = xval4<PREBN>(a.x, xin + ((size_t)c * H + va) * W + o);
      if (PREBN) {
        const float m = sMean[c], iv = sInv[c];
        v.x = (v.x - m) * iv;
        v.y = (v.y - m) * iv;
        v.z = (v.z - m) * iv;
        v.w = (v.w - m) * iv;
      }
      float* d = sIn + (c * HP + va - iyb + r) * WP + pad + ix;
      d[0] = fmaxf(v.x, 0.f);
      d[1] = fmaxf(v.y, 0.f);
      d[2] = fmaxf(v.z, 0.f);
      d[3] = fmaxf(v.w, 0.f);
    }
    for (int i = tid; i < C * HP; i += 256) {
      const int iy = iyb + i % HP;
      float* d = sIn + i * WP;
      if (iy < 0 || iy >= H) {
        for (int q = 0; q < WP; ++q) d[q] = 0.f;
      } else {
        for (int q = 0; q < pad; ++q) d[q] = d[pad + W + q] = 0.f;
      }
    }
  } else {
    // one wave per (channel, row); the row index is wave-uniform, lanes sweep columns
#pragma unroll 4
    for (int row = wave; row < C * HP; row += 4) {
      const int c = row / HP, r = row - c * HP, iy = iyb + r;
      const bool rok = iy >= 0 && iy < H;
      const size_t src = xin + ((size_t)c * H + (rok ? iy : 0)) * W;
      for (int q = lane; q < WP; q += 64) {
        const int ix = q - pad;
        float v = 0.f;
        if (rok && ix >= 0 && ix < W) {
          v = xval<PREBN>(a.x, src + ix);
          if (PREBN) v = (v - sMean[c]) * sInv[c];
          v = fmaxf(v, 0.f);
        }
        sIn[row * WP + q] = v;
      }
    }
  }
  __syncthreads();
  float st1[C], st2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) st1[c] = st2[c] = 0.f;
  const int HWo = Ho * Wo;
  zt* dn = a.d + ((size_t)n * a.C + c0) * HWo;
  zt* zn = a.z + (size_t)n * C * HWo;
  const bool vout = VEC && Wo % 4 == 0 && a.vout;
  if (vout) {
    // 4 consecutive output pixels (one row: Wo % 4 == 0) per thread: d and z leave as one 16-byte
    // (bf16: 8-byte) store per channel instead of four 4-byte ones
    for (int p = oy0 * Wo + 4 * tid; p < oy1 * Wo; p += 1024) {
      const int oy = p / Wo, ox0 = p - oy * Wo;
      zf4 d[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float* src = sIn + c * PL + ((oy - oy0) * S) * WP + ox0 * S;
        const float* wk = a.dw + (c0 + c) * KK;  // uniform -> scalar loads
        zf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            const float w = wk[ky * K + kx];
            const float* q = src + ky * DIL * WP + kx * DIL;
            acc.x += w * q[0];
            acc.y += w * q[S];
            acc.z += w * q[2 * S];
            acc.w += w * q[3 * S];
          }
        d[c] = acc;
        zst4(dn + (size_t)c * HWo + p, acc);
      }
      if (!PW) continue;
#pragma unroll
      for (int co = 0; co < C; ++co) {
        zf4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ci = 0; ci < C; ++ci) z += a.pw[co * C + ci] * d[ci];
        zst4(zn + (size_t)co * HWo + p, z);
        st1[co] += (z.x + z.y) + (z.z + z.w);
        st2[co] += (z.x * z.x + z.y * z.y) + (z.z * z.z + z.w * z.w);
      }
    }
  }
  for (int p = oy0 * Wo + tid; p < (vout ? 0 : oy1 * Wo); p += 256) {
    const int oy = p / Wo, ox = p - oy * Wo;
    float d[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* src = sIn + c * PL + ((oy - oy0) * S) * WP + ox * S;
      const float* wk = a.dw + (c0 + c) * KK;  // uniform -> scalar loads
      float acc = 0.f;
#pragma unroll
      for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) acc += wk[ky * K + kx] * src[ky * DIL * WP + kx * DIL];
      d[c] = acc;
      zput(dn + (size_t)c * HWo + p, acc);
    }
    if (!PW) continue;
#pragma unroll
    for (int co = 0; co < C; ++co) {
      float z = 0.f;
#pragma unroll
      for (int ci = 0; ci < C; ++ci) z += a.pw[co * C + ci] * d[ci];
      zput(zn + (size_t)co * HWo + p, z);
      st1[co] += z;
      st2[co] += z * z;
    }
  }
  if (!PW || !a.stats) return;
  {
    float st[2 * C];  // [sum | sum of squares], reduce-scattered over the wave
#pragma unroll
    for (int c = 0; c < C; ++c) st[c] = st1[c], st[C + c] = st2[c];
    const float v = wave_reduce_scatter<2 * C>(st);
    if ((lane & (32 / C - 1)) == 0) atomicAdd(sStat + wave_scatter_index<2 * C>(lane), v);
  }
  __syncthreads();
  if (tid < 2 * C) atomicAdd(a.stats + (bx % kRep) * 2 * C + tid, (double)sStat[tid]);
}
template <int K, int DIL, int S, bool PREBN, int C, bool VEC, bool PW = true>
__global__ void __launch_bounds__(256) dwpw_plane_kernel(DwPwFwdBatch bt) {
  dwpw_plane_body<K, DIL, S, PREBN, C, VEC, PW>(bt.e[blockIdx.y], blockIdx.x);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// One launch for a node's whole separable-stage / dilated-conv forward: every entry (edge x
// primitive) carries its own kernel size, dilation, stride, input-BN flag and band count, and
// each workgroup runs the fully unrolled body of its entry's (K, DIL, S, PREBN, VEC) variant.
// The entries are independent, so their workgroups overlap instead of running as 4-9 serial
// launches that each leave most of the chip waiting on their own tails.
#define DWPW_CASE(KK, DD, SS)                                                                      \
  case ((KK == 5) * 4 + (DD == 2) * 2 + (SS == 2)) * 4 + 0: dwpw_plane_body<KK, DD, SS, false, C, false, PW>(a, bx); break; \
  case ((KK == 5) * 4 + (DD == 2) * 2 + (SS == 2)) * 4 + 1: dwpw_plane_body<KK, DD, SS, false, C, true, PW>(a, bx); break;  \
  case ((KK == 5) * 4 + (DD == 2) * 2 + (SS == 2)) * 4 + 2: dwpw_plane_body<KK, DD, SS, true, C, false, PW>(a, bx); break;  \
  case ((KK == 5) * 4 + (DD == 2) * 2 + (SS == 2)) * 4 + 3: dwpw_plane_body<KK, DD, SS, true, C, true, PW>(a, bx); break;
template <int C, bool PW>
__global__ void __launch_bounds__(256) dwpw_plane_multi_kernel(DwPwMultiBatch bt) {
  // a COPY of the entry: a reference into the by-value batch made hipcc spill the whole 2.3 KB
  // batch to scratch once 32 variant bodies use it (ScratchSize 2320 B/lane, 20x slower)
  const DwPwFwdArgs a = bt.e[blockIdx.y];
  const int bx = blockIdx.x;
  if (bx < a.nblk) {  // entries differ in their band counts (uniform per workgroup)
    switch (a.variant) {
      DWPW_CASE(3, 1, 1) DWPW_CASE(3, 1, 2) DWPW_CASE(5, 1, 1) DWPW_CASE(5, 1, 2)
      DWPW_CASE(3, 2, 1) DWPW_CASE(3, 2, 2) DWPW_CASE(5, 2, 1) DWPW_CASE(5, 2, 2)
      default: break;
    }
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}
#undef DWPW_CASE


// ------------------------------------------------------------------------------------------------
// pw_fwd_wave: z[:, co_off + co] = pw . act(x) for Cin, Cout multiples of 16 (<= 64), plus the BN
// statistics of z. act = relu at (oy*S + off, ox*S + off) (StdConv / FactorizedReduce half) or the
// identity (a.relu == 0: the pointwise half of a wide dw-pw stage, x = the depthwise output d).
// One wave per 64-pixel chunk, no LDS and no barrier in the loop:
//   A[i = co][k = ci] = pw, preloaded in registers for the whole kernel;
//   B[k = ci][j]      lane (c16, q) loads pixels 4*c16 .. 4*c16+3 of channel k0 + q with one 16-byte
//                     load; MFMA t in 0..3 takes pixel 4*j + t as column j, so the D fragment a lane
//                     holds for (co, t = 0..3) is 4 consecutive pixels: one 16-byte store.
// Statistics stay per lane across chunks and are reduced once per workgroup at the end.
// NS > 1 (small planes, too few chunks to fill the chip): work item = (chunk, output-block group
// of CO / NS channels); the grid stride is a multiple of NS, so a wave keeps one group (and its
// weights and statistics) for all its items.
// ------------------------------------------------------------------------------------------------
// relu(x) at output pixels p, p + 1 of a stride-2 FactorizedReduce half (input (2oy + off, 2ox + off)):
// one 16-byte load of x[2oy + off][2ox .. 2ox + 3] holds both (p even and its row inside the plane,
// H = 2 Ho, W = 2 Wo, W % 4 == 0, x 16-byte aligned: the kernels check this as `fr2`)
__device__ __forceinline__ void fr2_pair(const float* plane, int W, int Wo, int off, int p, float& v0, float& v1) {
  const int oy = p / Wo, ox = p - oy * Wo;
  const float4 v = *reinterpret_cast<const float4*>(plane + (size_t)(2 * oy + off) * W + 2 * ox);
  v0 = fmaxf(off ? v.y : v.x, 0.f);
  v1 = fmaxf(off ? v.w : v.z, 0.f);
}

template <int CI, int CO, int NS = 1>
__global__ void __launch_bounds__(256) pw_fwd_wave_kernel(PwFwdBatch bt) {
  static_assert(CI % 16 == 0 && CO % 16 == 0 && CI <= 128 && CO <= 64 && (CO / 16) % NS == 0, "16-channel blocks");
  constexpr int BO = CO / 16 / NS, KS = CI / 4;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const PwFwdArgs& a = bt.e[blockIdx.y];
  const int HWo = a.Ho * a.Wo, Wo = a.Wo;
  const int nchunks = a.N * HWo / 64;  // HWo % 64 == 0 (host-checked)
  __shared__ float sStat[2 * CO];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, c16 = lane & 15, q = lane >> 4;
  for (int i = tid; i < 2 * CO; i += 256) sStat[i] = 0.f;
  __syncthreads();
  const int grp = (blockIdx.x * 4 + wave) % NS, cb0 = grp * BO * 16;  // first output channel of the group
  float wA[BO][KS];
#pragma unroll
  for (int bo = 0; bo < BO; ++bo)
#pragma unroll
    for (int k = 0; k < KS; ++k) wA[bo][k] = a.pw[(cb0 + bo * 16 + c16) * CI + 4 * k + q];
  const bool flat = !a.relu || (a.S == 1 && a.off == 0 && a.H == a.Ho && a.W == a.Wo);
  const bool fr2 = a.S == 2 && a.H == 2 * a.Ho && a.W == 2 * a.Wo && a.W % 4 == 0 && a.off <= 1 &&
                   ((uintptr_t)a.x & 15) == 0;
  f4 s1[BO], s2[BO];  // per-lane partial sums of z, z^2 for channels bo*16 + 4q + r
#pragma unroll
  for (int bo = 0; bo < BO; ++bo) s1[bo] = s2[bo] = f4{0.f, 0.f, 0.f, 0.f};
  for (int w = blockIdx.x * 4 + wave; w < nchunks * NS; w += gridDim.x * 4) {
    const int pix0 = (w / NS) * 64, n = pix0 / HWo, prem = pix0 - n * HWo;
    const int pp = prem + 4 * c16;  // this lane's 4 pixels
    f4 acc[BO][4];
#pragma unroll
    for (int bo = 0; bo < BO; ++bo)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[bo][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int ci = 4 * k + q;
      f4 v;
      if (flat) {
        if (a.relu) {  // node state (fp32), relu on the way in
          const size_t o = plane_off(n, ci, a.N, CI, a.xnodes, HWo) + pp;
          v = *reinterpret_cast<const f4*>(static_cast<const float*>(a.x) + o);
          v = f4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
        } else {  // depthwise output d of a wide dw-pw stage
          v = zld4(static_cast<const zt*>(a.x) + ((size_t)n * CI + ci) * HWo + pp);
        }
      } else if (fr2) {
        const float* plane = static_cast<const float*>(a.x) + plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W);
        float v0, v1, v2, v3;
        fr2_pair(plane, a.W, Wo, a.off, pp, v0, v1);
        fr2_pair(plane, a.W, Wo, a.off, pp + 2, v2, v3);
        v = f4{v0, v1, v2, v3};
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int p = pp + t, oy = p / Wo, ox = p - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
          v[t] = (iy < a.H && ix < a.W)
                     ? fmaxf(static_cast<const float*>(a.x)[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) +
                                                             (size_t)iy * a.W + ix], 0.f)
                     : 0.f;
        }
      }
#pragma unroll
      for (int bo = 0; bo < BO; ++bo)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[bo][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wA[bo][k], v[t], acc[bo][t], 0, 0, 0);
    }
    // D: acc[bo][t][r] = z[co = bo*16 + 4q + r][pixel pp + t]
#pragma unroll
    for (int bo = 0; bo < BO; ++bo)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const f4 z = f4{acc[bo][0][r], acc[bo][1][r], acc[bo][2][r], acc[bo][3][r]};
        zst4(a.z + ((size_t)n * a.CoutTotal + a.co_off + cb0 + bo * 16 + 4 * q + r) * HWo + pp, z);
        s1[bo][r] += (z.x + z.y) + (z.z + z.w);
        s2[bo][r] += (z.x * z.x + z.y * z.y) + (z.z * z.z + z.w * z.w);
      }
  }
  if (a.stats) {
#pragma unroll
  for (int bo = 0; bo < BO; ++bo)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float u = s1[bo][r], w = s2[bo][r];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {  // over the 16 lanes c16 sharing channel bo*16 + 4q + r
        u += __shfl_xor(u, o, 64);
        w += __shfl_xor(w, o, 64);
      }
      if (c16 == 0) {
        atomicAdd(sStat + cb0 + bo * 16 + 4 * q + r, u);
        atomicAdd(sStat + CO + cb0 + bo * 16 + 4 * q + r, w);
      }
    }
  __syncthreads();
  for (int i = tid; i < 2 * CO; i += 256) {
    const int hi = i >= CO;
    atomicAdd(a.stats + rep_slot() * 2 * a.CoutTotal + hi * a.CoutTotal + a.co_off + (i - hi * CO), (double)sStat[i]);
  }
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// ------------------------------------------------------------------------------------------------
// pw_fwd: z[:, co_off + co] = pw . relu(x) at (oy*S + off, ox*S + off); StdConv / FR half
// grid: N*Ho*Wo/64 blocks of 64-pixel tiles; Cin, Cout <= 256
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) pw_fwd_kernel(PwFwdBatch bt) {
  const PwFwdArgs& a = bt.e[blockIdx.y];
  constexpr int P = 64;
  const int Cin = a.Cin, Cout = a.Cout, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int HWo = Ho * Wo;
  const int ntiles = a.N * HWo / P;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sX = smem;              // [Cin][P]
  float* sStat = sX + Cin * P;   // [2*Cout]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int i = tid; i < 2 * Cout; i += 256) sStat[i] = 0.f;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int pix0 = t * P;  // flat over N*Ho*Wo (HWo % 64 == 0)
    const int n = pix0 / HWo, prem = pix0 % HWo;
    #pragma unroll 4  // keep several global loads of the staging pass in flight
    for (int i = tid; i < Cin * P; i += 256) {
      int ci = i / P, p = i % P;
      int pp = prem + p, oy = pp / Wo, ox = pp % Wo;
      int iy = oy * a.S + a.off, ix = ox * a.S + a.off;
      float v = 0.f;
      if (iy < H && ix < W) {
        const size_t xi = a.relu ? plane_off(n, ci, a.N, Cin, a.xnodes, (size_t)H * W) + (size_t)iy * W + ix
                                 : (((size_t)n * Cin + ci) * H + iy) * W + ix;
        v = a.relu ? fmaxf(static_cast<const float*>(a.x)[xi], 0.f) : z2f(static_cast<const zt*>(a.x)[xi]);
      }
      sX[i] = v;
    }
    __syncthreads();
    for (int co = wave; co < Cout; co += 4) {
      const int cou = __builtin_amdgcn_readfirstlane(co);
      const float* wrow = a.pw + cou * Cin;
      float v = 0.f;
      for (int ci = 0; ci < Cin; ++ci) v += wrow[ci] * sX[ci * P + lane];
      zput(a.z + ((size_t)n * a.CoutTotal + a.co_off + cou) * HWo + prem + lane, v);
      float s = wave_sum(v), s2 = wave_sum(v * v);
      if (lane == 0) {
        sStat[cou] += s;
        sStat[Cout + cou] += s2;
      }
    }
    __syncthreads();
  }
  if (a.stats)
    for (int i = tid; i < 2 * Cout; i += 256) {
      int hi = i >= Cout;
      atomicAdd(a.stats + rep_slot() * 2 * a.CoutTotal + hi * a.CoutTotal + a.co_off + (i - hi * Cout),
                (double)sStat[i]);
    }
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// ------------------------------------------------------------------------------------------------
// pool_fwd: avg (count_include_pad=False) and max 3x3/pad 1, stride S. One block per (n, c) plane.
// ------------------------------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void pool_fwd_body(const PoolFwdArgs& a, const int bx, const int gx) {
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int c = bx % C, g0 = bx / C, G = gx / C;
  float sa = 0, sa2 = 0, sm = 0, sm2 = 0;
  for (int n = g0; n < a.N; n += G) {
    const int nc = n * C + c;
    const float* xp = a.x + (size_t)nc * H * W;
    for (int o = threadIdx.x; o < Ho * Wo; o += 256) {
      int oy = o / Wo, ox = o % Wo;
      float sum = 0.f, mx = -INFINITY;
      int cnt = 0, arg = 0;
      for (int ky = 0; ky < 3; ++ky) {
        int iy = oy * S - 1 + ky;
        if (iy < 0 || iy >= H) continue;
        for (int kx = 0; kx < 3; ++kx) {
          int ix = ox * S - 1 + kx;
          if (ix < 0 || ix >= W) continue;
          float v = xp[iy * W + ix];
          sum += v;
          cnt++;
          if (v > mx || v != v) {  // first maximal element in row-major order (max_pool2d)
            mx = v;
            arg = ky * 3 + kx;
          }
        }
      }
      float av = sum / (float)cnt;
      zput(a.zavg + (size_t)nc * Ho * Wo + o, av);
      zput(a.zmax + (size_t)nc * Ho * Wo + o, mx);
      if (a.amax) a.amax[(size_t)nc * Ho * Wo + o] = (unsigned char)arg;
      sa += av;
      sa2 += av * av;
      sm += mx;
      sm2 += mx * mx;
    }
  }
  if (!a.stats_avg && !a.stats_max) return;
  __shared__ float red[4][4];
  int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  {
    float v[4] = {sa, sa2, sm, sm2};
    const float t = wave_reduce_scatter<4>(v);
    if ((lane & 15) == 0) red[wave][wave_scatter_index<4>(lane)] = t;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    double* dst = threadIdx.x < 2 ? a.stats_avg : a.stats_max;
    if (dst) atomicAdd(dst + (bx % kRep) * 2 * C + (threadIdx.x & 1) * C + c, (double)t);
  }
}
template <int S>
__global__ void __launch_bounds__(256) pool_fwd_kernel(PoolFwdBatch bt) {
  pool_fwd_body<S>(bt.e[blockIdx.y], blockIdx.x, gridDim.x);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// stride-1 and stride-2 pooling of a node in one launch (entry a.S; a.nblk workgroups, a multiple of C)
__global__ void __launch_bounds__(256) pool_fwd_multi_kernel(PoolFwdBatch bt) {
  const PoolFwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x < a.nblk) {
    if (a.S == 1) pool_fwd_body<1>(a, blockIdx.x, a.nblk);
    else pool_fwd_body<2>(a, blockIdx.x, a.nblk);
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}


// ------------------------------------------------------------------------------------------------
// combine_fwd: out = sum_k w[k] * BN_k(z_k) + wid * x  (elementwise), running stats in block 0
// ------------------------------------------------------------------------------------------------
template <bool V4>
__global__ void __launch_bounds__(256) combine_fwd_kernel(CombineFwdBatch bt) {
  // All edges of a node in one pass: out = sum_e [ sum_k w_e[k] * BN_ek(z_ek) + w_e[id] * x_e ].
  const CombineFwdArgs& a0 = bt.e[0];
  const int C = a0.C, HW = a0.HW, ne = bt.n;
  const size_t total = (size_t)a0.N * C * HW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sMean = smem;                                 // [ne][kMaxOps][C]
  float* sInv = sMean + ne * kMaxOps * C;              // [ne][kMaxOps][C]
  float* sW = sInv + ne * kMaxOps * C;                 // [ne][kMaxOps + 1]
  // every (edge, op, channel) coefficient in one pass: one round of statistic loads per block
  if (ne == 1 && a0.nops == 1 && !a0.bn[0].eval && a0.bn[0].rep > 1) {
    // a preprocess BN whose statistics arrive unfolded (their fold joins the cell's first node's)
    bn_coeffs_coop(a0.bn[0], 0, C, sMean, sInv);
  } else {
    for (int i = threadIdx.x; i < ne * kMaxOps * C; i += 256) {
      const int e = i / (kMaxOps * C), k = (i / C) % kMaxOps, c = i % C;
      const CombineFwdArgs& a = bt.e[e];
      if (k < a.nops) bn_coeffs(a.bn[k], c, sMean[i], sInv[i]);
    }
  }
  for (int i = threadIdx.x; i < ne * (kMaxOps + 1); i += 256) {
    const int e = i / (kMaxOps + 1), k = i % (kMaxOps + 1);
    const CombineFwdArgs& a = bt.e[e];
    if (k < a.nops) sW[i] = a.w ? a.w[a.widx[k]] : 1.f;
    else if (k == kMaxOps) sW[i] = (a.w && a.id_idx >= 0) ? a.w[a.id_idx] : 0.f;
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    for (int e = 0; e < ne; ++e) {
      const CombineFwdArgs& a = bt.e[e];
      if (!a.update_running) continue;
      for (int i = threadIdx.x; i < (a.nops + a.nupd) * C; i += 256) {
        int k = i / C, c = i % C;
        const BNRef& b = k < a.nops ? a.bn[k] : a.upd[k - a.nops];
        if (!b.rmean || b.eval) continue;
        double m, v;
        bn_moments(b, c, m, v);
        double cnt = 1.0 / (double)b.inv_count;
        double vu = cnt > 1 ? v * cnt / (cnt - 1) : v;
        b.rmean[c] = (1.f - a.momentum) * b.rmean[c] + a.momentum * (float)m;
        b.rvar[c] = (1.f - a.momentum) * b.rvar[c] + a.momentum * (float)vu;
      }
    }
  }
  if (V4) {
    // 4 consecutive elements per thread (HW % 4 == 0: one channel), 16-byte loads/stores;
    // the host picks this path only when every operand pointer is 16-byte aligned
    typedef float f4 __attribute__((ext_vector_type(4)));
    const size_t total4 = total / 4;
    constexpr int EM = CombineFwdBatch::kCap;
    for (size_t i4 = (size_t)blockIdx.x * 256 + threadIdx.x; i4 < total4; i4 += (size_t)gridDim.x * 256) {
      const int c = (int)((i4 * 4 / HW) % C);
      // issue every operand load first (up to EM * (kMaxOps + 1) in flight), then accumulate in
      // the scalar path's order: a runtime-bounded load-then-add loop waited on each load in turn
      f4 zv[EM][kMaxOps], xv[EM];
#pragma unroll
      for (int e = 0; e < EM; ++e) {
        const CombineFwdArgs& a = bt.e[e < ne ? e : 0];
#pragma unroll
        for (int k = 0; k < kMaxOps; ++k)
          if (e < ne && k < a.nops) zv[e][k] = zld4(a.z[k] + 4 * i4);
        if (e < ne && a.xid) xv[e] = reinterpret_cast<const f4*>(a.xid)[i4];
      }
      f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < EM; ++e) {
        if (e >= ne) break;
        const CombineFwdArgs& a = bt.e[e];
        const float* sw = sW + e * (kMaxOps + 1);
#pragma unroll
        for (int k = 0; k < kMaxOps; ++k) {
          if (k >= a.nops) break;
          const int j = (e * kMaxOps + k) * C + c;
          // same rounding as the scalar path: w * ((z - mean) * inv)
          const float m = sMean[j], inv = sInv[j];
          acc += sw[k] * ((zv[e][k] - m) * inv);
        }
        if (a.xid) acc += sw[kMaxOps] * xv[e];
      }
      if (a0.gamma) acc = acc * a0.gamma[c] + a0.beta[c];
      f4* o = reinterpret_cast<f4*>(a0.out) + i4;
      *o = a0.accumulate ? *o + acc : acc;
    }
    return;
  }
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    int c = (int)((i / HW) % C);
    float acc = 0.f;
    for (int e = 0; e < ne; ++e) {
      const CombineFwdArgs& a = bt.e[e];
      const float* sw = sW + e * (kMaxOps + 1);
      for (int k = 0; k < a.nops; ++k) {
        const int j = (e * kMaxOps + k) * C + c;
        acc += sw[k] * ((z2f(a.z[k][i]) - sMean[j]) * sInv[j]);
      }
      if (a.xid) acc += sw[kMaxOps] * a.xid[i];
    }
    if (a0.gamma) acc = acc * a0.gamma[c] + a0.beta[c];
    a0.out[i] = a0.accumulate ? a0.out[i] + acc : acc;
  }
}

// ------------------------------------------------------------------------------------------------
// combine_bwd_reduce: S1[c] = sum dout, S2[k][c] = sum dout * zhat_k, Sid = sum dout * x
// One block per (n, c) plane.
// ------------------------------------------------------------------------------------------------
template <bool V4>
__global__ void __launch_bounds__(256) combine_bwd_reduce_kernel(CombineBwdBatch bt) {
  const CombineBwdArgs& a = bt.e[blockIdx.y];
  const int C = a.C, HW = a.HW;
  const int c = blockIdx.x % C, g0 = blockIdx.x / C, G = gridDim.x / C;
  __shared__ float sMean[kMaxOps], sInv[kMaxOps];
  __shared__ float part[4][kMaxOps + 2];
  if (threadIdx.x < a.nops) bn_coeffs(a.bn[threadIdx.x], c, sMean[threadIdx.x], sInv[threadIdx.x]);
  __syncthreads();
  float s1 = 0.f, sid = 0.f;
  float s2[kMaxOps];
#pragma unroll
  for (int k = 0; k < kMaxOps; ++k) s2[k] = 0.f;
  if (V4) {
    // the block's (image, float4) pairs flattened so every thread has work at small HW;
    // 16-byte loads, all operands of an element issued before use
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int q4 = HW / 4, cnt = (a.N - g0 + G - 1) / G;
    for (int t = threadIdx.x; t < cnt * q4; t += 256) {
      const int n = g0 + (t / q4) * G, i4 = t - (t / q4) * q4;
      const size_t b4 = ((size_t)n * C + c) * q4 + i4;
      const f4 g = reinterpret_cast<const f4*>(a.dout)[b4];
      f4 zv[kMaxOps];
#pragma unroll
      for (int k = 0; k < kMaxOps; ++k)
        if (k < a.nops) zv[k] = zld4(a.z[k] + 4 * b4);
      f4 xv = {0.f, 0.f, 0.f, 0.f};
      if (a.xid) xv = reinterpret_cast<const f4*>(a.xid)[b4];
      s1 += (g.x + g.y) + (g.z + g.w);
#pragma unroll
      for (int k = 0; k < kMaxOps; ++k)
        if (k < a.nops) {
          const f4 t2 = g * (zv[k] - sMean[k]) * sInv[k];
          s2[k] += (t2.x + t2.y) + (t2.z + t2.w);
        }
      if (a.xid) {
        const f4 t3 = g * xv;
        sid += (t3.x + t3.y) + (t3.z + t3.w);
      }
    }
  } else {
    for (int n = g0; n < a.N; n += G) {
      const size_t base = ((size_t)n * C + c) * HW;
      for (int i = threadIdx.x; i < HW; i += 256) {
        float g = a.dout[base + i];
        s1 += g;
#pragma unroll
        for (int k = 0; k < kMaxOps; ++k)
          if (k < a.nops) s2[k] += g * (z2f(a.z[k][base + i]) - sMean[k]) * sInv[k];
        if (a.xid) sid += g * a.xid[base + i];
      }
    }
  }
  int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  {
    // [s1, sid, s2[0..kMaxOps)] reduce-scattered over the wave (padded to 16 accumulators)
    static_assert(kMaxOps + 2 <= 16, "combine_bwd_reduce: accumulators exceed the 16-slot scatter");
    float v[16];
    v[0] = s1;
    v[1] = sid;
#pragma unroll
    for (int k = 0; k < 14; ++k) v[2 + k] = k < kMaxOps ? s2[k] : 0.f;
    const float t = wave_reduce_scatter<16>(v);
    const int j = wave_scatter_index<16>(lane);
    if ((lane & 3) == 0 && j < kMaxOps + 2) part[wave][j] = t;
  }
  __syncthreads();
  double* red = a.red + (size_t)rep_slot() * a.rstride;
  double* gw = a.gw ? a.gw + (size_t)rep_slot() * a.gwstride : nullptr;
  if (threadIdx.x < a.nops + 2) {
    int j = threadIdx.x;
    float t = part[0][j] + part[1][j] + part[2][j] + part[3][j];
    if (j == 0) {
      atomicAdd(red + c, (double)t);
    } else if (j == 1) {
      if (a.xid) {
        atomicAdd(red + (size_t)(1 + a.nops) * C, (double)t);
        if (gw && a.id_idx >= 0) atomicAdd(gw + a.id_idx, (double)t);
      }
    } else {
      atomicAdd(red + (size_t)(j - 1) * C + c, (double)t);
      if (gw) atomicAdd(gw + a.widx[j - 2], (double)t);
    }
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// on-the-fly BN backward: dz = wk * invstd * (g - S1/cnt - zhat * S2/cnt)
__device__ __forceinline__ float bn_bwd_val(const GradSrc& gs, size_t i, float mean, float inv, float wk, float m1,
                                           float m2) {
  float zh = (z2f(gs.z[i]) - mean) * inv;
  float g = gs.g[i];
  return wk * inv * (g - m1 - zh * m2);  // eval: m1 = m2 = 0
}

// ------------------------------------------------------------------------------------------------
// pw_bwd: dz (on the fly) -> dd = pw^T dz ; dW_pw += dz (x) a_in.
// mode 0 (dw-pw stage): a_in = stored depthwise output d; writes dd [N,Cin,Ho,Wo].
// mode 1 (StdConv / FR half): a_in = relu(x) at strided positions; gx += dd * (x > 0).
// grid: persistent over 64-pixel tiles; weight grads accumulated in registers across tiles.
// ------------------------------------------------------------------------------------------------
template <bool MFMA, int MBLK = 4>
__global__ void __launch_bounds__(256) pw_bwd_kernel(PwBwdBatch bt) {
  const PwBwdArgs& a = bt.e[blockIdx.y];
  constexpr int P = 64, PS = P + 1;  // padded LDS rows: per-channel row reads hit distinct banks
  const int Cin = a.Cin, Cout = a.Cout, Ho = a.Ho, Wo = a.Wo, HWo = Ho * Wo;
  const int ntiles = a.N * HWo / P;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sDz = smem;             // [Cout][PS]
  float* sA = sDz + Cout * PS;   // [Cin][PS]
  float* sMean = sA + Cin * PS;  // [Cout]
  float* sInv = sMean + Cout;
  float* sM1 = sInv + Cout;      // [Cout]
  float* sM2 = sM1 + Cout;
  float* sW = sM2 + Cout;        // [1]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int c = tid; c < Cout; c += 256) bn_coeffs(a.gs.bn, a.co_off + c, sMean[c], sInv[c]);
  gs_means_coop(a.gs, a.co_off, Cout, sM1, sM2);
  if (tid == 0) sW[0] = a.gs.w ? a.gs.w[a.gs.widx] : 1.f;
  __syncthreads();
  const float wk = sW[0];
  typedef float f4 __attribute__((ext_vector_type(4)));
  // weight-grad accumulators live in registers across tiles.
  // scalar path: pairs (co, ci) = tid + 256*j; MFMA path: 16x16 blocks b = wave + 4*j
  // Cout*Cin <= 8192 (the 128 -> 64 preprocess of darts-gpu.yaml's last cell); MFMA: MBLK 16x16
  // blocks per wave (4 waves x MBLK x 256), 8 only where needed (more accumulators, fewer waves)
  constexpr int MAXJ = 32;
  float gacc[MFMA ? 1 : MAXJ];
  f4 macc[MFMA ? MBLK : 1];
#pragma unroll
  for (int j = 0; j < (MFMA ? 1 : MAXJ); ++j) gacc[j] = 0.f;
#pragma unroll
  for (int j = 0; j < (MFMA ? MBLK : 1); ++j) macc[j] = f4{0, 0, 0, 0};
  const int npairs = Cout * Cin;
  const int nbi = Cin / 16, nblk = (Cout / 16) * nbi;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int pix0 = t * P, n = pix0 / HWo, prem = pix0 % HWo;
    #pragma unroll 4  // keep several global loads of the staging pass in flight
    for (int i = tid; i < Cout * P; i += 256) {
      int co = i / P, p = i % P;
      size_t gi = ((size_t)n * a.CoutTotal + a.co_off + co) * HWo + prem + p;
      sDz[co * PS + p] = bn_bwd_val(a.gs, gi, sMean[co], sInv[co], wk, sM1[co], sM2[co]);
    }
    #pragma unroll 4  // keep several global loads of the staging pass in flight
    for (int i = tid; i < Cin * P; i += 256) {
      int ci = i / P, p = i % P;
      int pp = prem + p;
      float v;
      if (a.mode == 0) {
        v = z2f(a.ain[((size_t)n * Cin + ci) * HWo + pp]);
      } else {
        int oy = pp / Wo, ox = pp % Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
        v = (iy < a.H && ix < a.W)
                ? fmaxf(a.x[plane_off(n, ci, a.N, Cin, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix], 0.f)
                : 0.f;
      }
      sA[ci * PS + p] = v;
    }
    __syncthreads();
    if (a.gW) {
      if (MFMA) {
        // gW[co][ci] += sum_p dz[co][p] * a[ci][p]  (M = co, N = ci, K = pixels)
#pragma unroll
        for (int j = 0; j < MBLK; ++j) {
          int b = wave + 4 * j;
          if (b < nblk) {
            int cob = (b / nbi) * 16, cib = (b % nbi) * 16;
            for (int p0 = 0; p0 < P; p0 += 4) {
              float av = sDz[(cob + (lane & 15)) * PS + p0 + (lane >> 4)];
              float bv = sA[(cib + (lane & 15)) * PS + p0 + (lane >> 4)];
              macc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, macc[j], 0, 0, 0);
            }
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
          int pr = tid + 256 * j;
          if (pr < npairs) {
            int co = pr / Cin, ci = pr % Cin;
            float s = 0.f;
            for (int p = 0; p < P; ++p) s += sDz[co * PS + p] * sA[ci * PS + p];
            gacc[j] += s;
          }
        }
      }
    }
    // dd[ci][p] = sum_co pw[co][ci] dz[co][p]
    if (a.need_dx) {
      if (MFMA) {
        for (int cib = wave * 16; cib < Cin; cib += 64) {
          f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
          for (int k0 = 0; k0 < Cout; k0 += 4) {
            float av = a.pw[(k0 + (lane >> 4)) * Cin + cib + (lane & 15)];
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) {
              float bv = sDz[(k0 + (lane >> 4)) * PS + pb * 16 + (lane & 15)];
              acc[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[pb], 0, 0, 0);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            int ci = cib + (lane >> 4) * 4 + r;
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) {
              int pp = prem + pb * 16 + (lane & 15);
              float v = acc[pb][r];
              if (a.mode == 0) {
                a.dd[((size_t)n * Cin + ci) * HWo + pp] = v;
              } else {
                int oy = pp / Wo, ox = pp % Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
                if (iy < a.H && ix < a.W) {
                  size_t xi = plane_off(n, ci, a.N, Cin, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix;
                  if (a.overwrite) a.gx[xi] = a.x[xi] > 0.f ? v : 0.f;
                  else if (a.x[xi] > 0.f) a.gx[xi] += v;
                }
              }
            }
          }
        }
      } else {
        for (int ci = wave; ci < Cin; ci += 4) {
          const int ciu = __builtin_amdgcn_readfirstlane(ci);
          float v = 0.f;
          for (int co = 0; co < Cout; ++co) v += a.pw[co * Cin + ciu] * sDz[co * PS + lane];
          int pp = prem + lane;
          if (a.mode == 0) {
            a.dd[((size_t)n * Cin + ciu) * HWo + pp] = v;
          } else {
            int oy = pp / Wo, ox = pp % Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
            if (iy < a.H && ix < a.W) {
              size_t xi = plane_off(n, ciu, a.N, Cin, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix;
              if (a.overwrite) a.gx[xi] = a.x[xi] > 0.f ? v : 0.f;
              else if (a.x[xi] > 0.f) a.gx[xi] += v;
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (a.gW) {
    float* gW = a.gW + (size_t)rep_slot() * a.gstride;
    if (MFMA) {
#pragma unroll
      for (int j = 0; j < MBLK; ++j) {
        int b = wave + 4 * j;
        if (b < nblk) {
          int cob = (b / nbi) * 16, cib = (b % nbi) * 16;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            atomicAdd(gW + (cob + (lane >> 4) * 4 + r) * Cin + cib + (lane & 15), macc[j][r]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        int pr = tid + 256 * j;
        if (pr < npairs) atomicAdd(gW + pr, gacc[j]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// pw_bwd_px: pw_bwd for narrow layers (Cin * Cout <= 96, the C = 4..12 channels of small
// supernets). The tiled kernel above spends most of its time in the weight-gradient sum, where
// Cin * Cout threads (16 of 256 at C = 4) each walk the tile's 64 pixels through LDS. Here
// every thread owns whole pixels with ALL channels in registers: dz (BN backward on the fly),
// the layer input, dd = pw^T dz, and a private Cin x Cout weight-gradient accumulator; loads
// and stores are coalesced across the wave (consecutive pixels), there is no LDS staging and
// no barrier until the block's single reduction of its accumulators (wave shuffles, then one
// LDS add per wave and one global atomic vector per block into the block's replica).
// ------------------------------------------------------------------------------------------------
template <int CI, int CO, bool V4>
__global__ void __launch_bounds__(256) pw_bwd_px_kernel(PwBwdBatch bt) {
  const PwBwdArgs& a = bt.e[blockIdx.y];
  const int HWo = a.Ho * a.Wo, Wo = a.Wo;
  const int total = a.N * HWo;
  __shared__ float sC[4 * CO + 1];
  __shared__ float sGW[CI * CO];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int c = tid; c < CO; c += 256) bn_coeffs(a.gs.bn, a.co_off + c, sC[c], sC[CO + c]);
  gs_means_coop(a.gs, a.co_off, CO, sC + 2 * CO, sC + 3 * CO);  // the BN-backward sums may arrive unfolded
  if (tid == 0) sC[4 * CO] = a.gs.w ? a.gs.w[a.gs.widx] : 1.f;
  for (int i = tid; i < CI * CO; i += 256) sGW[i] = 0.f;
  __syncthreads();
  float mean[CO], inv[CO], m1[CO], m2[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    mean[c] = sC[c];
    inv[c] = sC[CO + c];
    m1[c] = sC[2 * CO + c];
    m2[c] = sC[3 * CO + c];
  }
  const float wk = sC[4 * CO];
  float wpw[CI * CO];  // pointwise weights in registers (the loop's stores could alias them)
#pragma unroll
  for (int i = 0; i < CI * CO; ++i) wpw[i] = a.pw[i];
  float gacc[CI * CO];
#pragma unroll
  for (int i = 0; i < CI * CO; ++i) gacc[i] = 0.f;
  const bool want_w = a.gW != nullptr;
  if (V4) {
    // 4 consecutive pixels per thread with 16-byte loads/stores (HWo % 4 == 0; mode 0, or
    // mode 1 at stride 1 / offset 0 where the input plane is the output plane)
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int t = blockIdx.x * 256 + tid; t < total / 4; t += gridDim.x * 256) {
      const int p = t * 4, n = p / HWo, pp = p - n * HWo;
      f4 dz[CO], av[CI];
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        const size_t gi = ((size_t)n * a.CoutTotal + a.co_off + c) * HWo + pp;
        const f4 zz = zld4(a.gs.z + gi), gg = *reinterpret_cast<const f4*>(a.gs.g + gi);
        dz[c] = wk * inv[c] * (gg - m1[c] - ((zz - mean[c]) * inv[c]) * m2[c]);
      }
#pragma unroll
      for (int c = 0; c < CI; ++c) {
        const size_t o = a.mode == 0 ? ((size_t)n * CI + c) * HWo + pp : plane_off(n, c, a.N, CI, a.xnodes, HWo) + pp;
        av[c] = a.mode == 0 ? zld4(a.ain + o) : *reinterpret_cast<const f4*>(a.x + o);
        if (a.mode != 0) {
          av[c].x = fmaxf(av[c].x, 0.f);
          av[c].y = fmaxf(av[c].y, 0.f);
          av[c].z = fmaxf(av[c].z, 0.f);
          av[c].w = fmaxf(av[c].w, 0.f);
        }
      }
      if (want_w) {
#pragma unroll
        for (int co = 0; co < CO; ++co)
#pragma unroll
          for (int ci = 0; ci < CI; ++ci) {
            const f4 t2 = dz[co] * av[ci];
            gacc[co * CI + ci] += (t2.x + t2.y) + (t2.z + t2.w);
          }
      }
      if (a.need_dx) {
#pragma unroll
        for (int ci = 0; ci < CI; ++ci) {
          f4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int co = 0; co < CO; ++co) v += wpw[co * CI + ci] * dz[co];
          const size_t o = a.mode == 0 ? ((size_t)n * CI + ci) * HWo + pp : plane_off(n, ci, a.N, CI, a.xnodes, HWo) + pp;
          if (a.mode == 0) {
            *reinterpret_cast<f4*>(a.dd + o) = v;
          } else {
            f4 m;
            m.x = av[ci].x > 0.f ? v.x : 0.f;
            m.y = av[ci].y > 0.f ? v.y : 0.f;
            m.z = av[ci].z > 0.f ? v.z : 0.f;
            m.w = av[ci].w > 0.f ? v.w : 0.f;
            f4* g = reinterpret_cast<f4*>(a.gx + o);
            *g = a.overwrite ? m : *g + m;
          }
        }
      }
    }
  }
  for (int p = blockIdx.x * 256 + tid; p < (V4 ? 0 : total); p += gridDim.x * 256) {
    const int n = p / HWo, pp = p - n * HWo;
    float dz[CO], av[CI];
#pragma unroll
    for (int c = 0; c < CO; ++c)
      dz[c] = bn_bwd_val(a.gs, ((size_t)n * a.CoutTotal + a.co_off + c) * HWo + pp, mean[c], inv[c], wk, m1[c], m2[c]);
    size_t xi0 = 0;
    bool inb = true;
    if (a.mode == 0) {
#pragma unroll
      for (int c = 0; c < CI; ++c) av[c] = z2f(a.ain[((size_t)n * CI + c) * HWo + pp]);
    } else {
      const int oy = pp / Wo, ox = pp - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
      inb = iy < a.H && ix < a.W;
      xi0 = (size_t)iy * a.W + ix;  // pixel inside the channel plane (plane_off below)
#pragma unroll
      for (int c = 0; c < CI; ++c)
        av[c] = inb ? fmaxf(a.x[plane_off(n, c, a.N, CI, a.xnodes, (size_t)a.H * a.W) + xi0], 0.f) : 0.f;
    }
    if (want_w) {
#pragma unroll
      for (int co = 0; co < CO; ++co)
#pragma unroll
        for (int ci = 0; ci < CI; ++ci) gacc[co * CI + ci] += dz[co] * av[ci];
    }
    if (a.need_dx) {
#pragma unroll
      for (int ci = 0; ci < CI; ++ci) {
        float v = 0.f;
#pragma unroll
        for (int co = 0; co < CO; ++co) v += wpw[co * CI + ci] * dz[co];
        if (a.mode == 0) {
          a.dd[((size_t)n * CI + ci) * HWo + pp] = v;
        } else if (a.overwrite) {  // stride 1: every input pixel is some thread's own
          a.gx[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + xi0] = av[ci] > 0.f ? v : 0.f;
        } else if (inb && av[ci] > 0.f) {  // relu'(x): x > 0  <=>  relu(x) > 0
          a.gx[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + xi0] += v;
        }
      }
    }
  }
  if (!want_w) return;
  constexpr int M = CI * CO;
  if (M <= 64 && (M & (M - 1)) == 0) {
    const float s = wave_reduce_scatter<(M <= 64 ? M : 64)>(gacc);
    if ((lane & (64 / M - 1)) == 0) atomicAdd(sGW + wave_scatter_index<(M <= 64 ? M : 64)>(lane), s);
  } else {
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const float s = wave_sum(gacc[i]);
      if (lane == 0) atomicAdd(sGW + i, s);
    }
  }
  __syncthreads();
  float* gW = a.gW + (size_t)rep_slot() * a.gstride;
  for (int i = tid; i < CI * CO; i += 256) atomicAdd(gW + i, sGW[i]);
}

// orders a wave's LDS writes before its later LDS reads of other lanes' data (LDS executes one
// wave's instructions in order, so only the compiler has to be kept from reordering them)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------------------------------------------
// pw_bwd_wave: pw_bwd for the 16..64-channel layers of darts-gpu.yaml-sized supernets (Cin, Cout
// multiples of 16). The tiled kernel above stages a 64-pixel tile per workgroup between two
// barriers and runs its MFMA chains on one wave when Cin = Cout = 16, so each workgroup walks a
// serial load -> barrier -> compute chain per tile. Here every WAVE owns whole 64-pixel chunks
// and never waits for the others until the final weight-gradient reduction:
//   loads   lane (c = lane & 15, q = lane >> 4) reads 16 consecutive pixels q*16 .. q*16+15 of
//           channel c of every 16-channel block with 16-byte loads: dz (BN backward on the fly)
//           and the layer input, straight into MFMA operand registers;
//   dW      v_mfma_f32_16x16x4f32 with K = pixels: step j feeds pixel q*16 + j of lane group q
//           as k-index q, so the 16 steps cover the chunk with no data movement;
//   dd      pw^T dz needs dz with channels on the K axis: the wave writes its dz chunk to a
//           wave-private LDS tile (no workgroup barrier) and reads it back in B-operand order.
// ------------------------------------------------------------------------------------------------
// NS > 1 (small planes): work item = (chunk, group of CI / NS input channels): the wave forms dz for
// every output channel but the weight gradients and dd of its input-channel group only.
template <int CI, int CO, int NS = 1>
__global__ void __launch_bounds__(256) pw_bwd_wave_kernel(PwBwdBatch bt) {
  static_assert(CI % 16 == 0 && CO % 16 == 0 && CI <= 128 && CO <= 64 && (CI / 16) % NS == 0, "16-channel blocks");
  constexpr int BO = CO / 16, BI = CI / 16 / NS, RS = 64 + 4;  // LDS tile row stride (floats)
  typedef float f4 __attribute__((ext_vector_type(4)));
  const PwBwdArgs& a = bt.e[blockIdx.y];
  const int HWo = a.Ho * a.Wo, Wo = a.Wo;
  const int nchunks = a.N * HWo / 64;  // HWo % 64 == 0 (host-checked)
  extern __shared__ __attribute__((aligned(16))) float smem[];  // [4 waves][CO][RS]
  __shared__ float sC[4 * CO + 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int c16 = lane & 15, q = lane >> 4;
  for (int c = tid; c < CO; c += 256) bn_coeffs(a.gs.bn, a.co_off + c, sC[c], sC[CO + c]);
  gs_means_coop(a.gs, a.co_off, CO, sC + 2 * CO, sC + 3 * CO);
  if (tid == 0) sC[4 * CO] = a.gs.w ? a.gs.w[a.gs.widx] : 1.f;
  __syncthreads();
  const float wk = sC[4 * CO];
  float mean[BO], inv[BO], m1[BO], m2[BO];
#pragma unroll
  for (int bo = 0; bo < BO; ++bo) {
    const int c = bo * 16 + c16;
    mean[bo] = sC[c];
    inv[bo] = sC[CO + c];
    m1[bo] = sC[2 * CO + c];
    m2[bo] = sC[3 * CO + c];
  }
  const bool want_w = a.gW != nullptr;
  // contiguous input rows: the dw-pw stage, or a stride-1 StdConv whose input plane is the output plane
  const bool flat = a.mode == 0 || (a.S == 1 && a.off == 0 && a.H == a.Ho && a.W == a.Wo);
  const bool fr2 = a.mode != 0 && a.S == 2 && a.H == 2 * a.Ho && a.W == 2 * a.Wo && a.W % 4 == 0 && a.off <= 1 &&
                   ((uintptr_t)a.x & 15) == 0;
  float* sT = smem + wave * CO * RS;
  const int ci0 = ((blockIdx.x * 4 + wave) % NS) * BI * 16;  // the wave's input-channel group (fixed: stride % NS == 0)
  f4 macc[BO][BI];
#pragma unroll
  for (int bo = 0; bo < BO; ++bo)
#pragma unroll
    for (int bi = 0; bi < BI; ++bi) macc[bo][bi] = f4{0.f, 0.f, 0.f, 0.f};
  for (int w = blockIdx.x * 4 + wave; w < nchunks * NS; w += gridDim.x * 4) {
    const int pix0 = (w / NS) * 64, n = pix0 / HWo, prem = pix0 - n * HWo;
    const int pq = prem + q * 16;  // this lane's pixels pq .. pq + 15
    float dz[BO][16];
#pragma unroll
    for (int bo = 0; bo < BO; ++bo) {
      const size_t gi = ((size_t)n * a.CoutTotal + a.co_off + bo * 16 + c16) * HWo + pq;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4 zz = zld4(a.gs.z + gi + 4 * t);
        const f4 gg = *reinterpret_cast<const f4*>(a.gs.g + gi + 4 * t);
        const f4 v = wk * inv[bo] * (gg - m1[bo] - ((zz - mean[bo]) * inv[bo]) * m2[bo]);
        dz[bo][4 * t] = v.x;
        dz[bo][4 * t + 1] = v.y;
        dz[bo][4 * t + 2] = v.z;
        dz[bo][4 * t + 3] = v.w;
      }
    }
    if (want_w) {
      float av[BI][16];
#pragma unroll
      for (int bi = 0; bi < BI; ++bi) {
        const int ci = ci0 + bi * 16 + c16;
        if (flat) {
          const size_t so = a.mode == 0 ? ((size_t)n * CI + ci) * HWo + pq : plane_off(n, ci, a.N, CI, a.xnodes, HWo) + pq;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            f4 v = a.mode == 0 ? zld4(a.ain + so + 4 * t) : *reinterpret_cast<const f4*>(a.x + so + 4 * t);
            if (a.mode != 0) v = f4{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f)};
            av[bi][4 * t] = v.x;
            av[bi][4 * t + 1] = v.y;
            av[bi][4 * t + 2] = v.z;
            av[bi][4 * t + 3] = v.w;
          }
        } else if (fr2) {
          const float* plane = a.x + plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W);
#pragma unroll
          for (int j = 0; j < 16; j += 2) fr2_pair(plane, a.W, Wo, a.off, pq + j, av[bi][j], av[bi][j + 1]);
        } else {  // FactorizedReduce half: relu(x) at (oy*S + off, ox*S + off)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int pp = pq + j, oy = pp / Wo, ox = pp - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
            av[bi][j] = (iy < a.H && ix < a.W)
                            ? fmaxf(a.x[plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix], 0.f)
                            : 0.f;
          }
        }
      }
      // gW[co][ci] += sum_p dz[co][p] a[ci][p]: A[i = co][k = p], B[k = p][j = ci]
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int bo = 0; bo < BO; ++bo)
#pragma unroll
          for (int bi = 0; bi < BI; ++bi)
            macc[bo][bi] = __builtin_amdgcn_mfma_f32_16x16x4f32(dz[bo][j], av[bi][j], macc[bo][bi], 0, 0, 0);
    }
    if (!a.need_dx) continue;
    // dz chunk -> wave-private LDS tile [co][p]
    wave_lds_sync();  // the previous chunk's tile reads are done
#pragma unroll
    for (int bo = 0; bo < BO; ++bo)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        *reinterpret_cast<f4*>(sT + (bo * 16 + c16) * RS + q * 16 + 4 * t) =
            f4{dz[bo][4 * t], dz[bo][4 * t + 1], dz[bo][4 * t + 2], dz[bo][4 * t + 3]};
    wave_lds_sync();
    // dd[ci][p] = sum_co pw[co][ci] dz[co][p]: A[i = ci][k = co] = pw[co][ci], B[k = co][j = p]
#pragma unroll
    for (int bi = 0; bi < BI; ++bi) {
      f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
      for (int k0 = 0; k0 < CO; k0 += 4) {
        const float av = a.pw[(k0 + q) * CI + ci0 + bi * 16 + c16];
#pragma unroll
        for (int pb = 0; pb < 4; ++pb)
          acc[pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sT[(k0 + q) * RS + pb * 16 + c16], acc[pb], 0, 0, 0);
      }
      // D map: row (ci) = bi*16 + q*4 + r, col (pixel) = pb*16 + c16
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ci = ci0 + bi * 16 + q * 4 + r;
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          const int pp = prem + pb * 16 + c16;
          const float v = acc[pb][r];
          if (a.mode == 0) {
            a.dd[((size_t)n * CI + ci) * HWo + pp] = v;
          } else {
            const int oy = pp / Wo, ox = pp - oy * Wo, iy = oy * a.S + a.off, ix = ox * a.S + a.off;
            if (iy < a.H && ix < a.W) {
              const size_t xi = plane_off(n, ci, a.N, CI, a.xnodes, (size_t)a.H * a.W) + (size_t)iy * a.W + ix;
              if (a.overwrite) a.gx[xi] = a.x[xi] > 0.f ? v : 0.f;
              else if (a.x[xi] > 0.f) a.gx[xi] += v;
            }
          }
        }
      }
    }
  }
  if (!want_w) return;
  // the 4 waves' partial 16x16 blocks -> one LDS sum -> one atomic vector per workgroup
  __syncthreads();
  float* sG = smem;  // [CO][CI]
  for (int i = tid; i < CO * CI; i += 256) sG[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int bo = 0; bo < BO; ++bo)
#pragma unroll
    for (int bi = 0; bi < BI; ++bi)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(sG + (bo * 16 + q * 4 + r) * CI + ci0 + bi * 16 + c16, macc[bo][bi][r]);
  __syncthreads();
  float* gW = a.gW + (size_t)rep_slot() * a.gstride;
  for (int i = tid; i < CO * CI; i += 256) atomicAdd(gW + i, sG[i]);
}

// ------------------------------------------------------------------------------------------------
// dw_bwd: transposed depthwise. For own output rows [oy0, oy0+TR): dW_dw += dd * act(in);
// for own input rows [oy0*S, (oy0+TR)*S): ga = sum_taps dw * dd, masked by act'(in).
// PREBN: input = z_prev (pre-BN), act = relu(BN(.)) -> writes g_prev and reductions for BN bwd.
// else  : input = x, act = relu -> gx += ga * (x > 0).
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, bool PREBN>
__global__ void __launch_bounds__(256) dw_bwd_kernel(DwBwdBatch bt) {
  const DwBwdArgs& a = bt.e[blockIdx.y];
  constexpr int P = 64, KK = K * K;
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int TR = P / Wo;
  const int tiles = Ho / TR;
  const int ntiles = a.N * tiles;
  const int pad = a.pad;
  const int r = (K - 1) / 2 * DIL;         // == pad for these ops
  const int h = (r + S - 1) / S;           // halo output rows
  const int OR = TR + 2 * h;               // staged dd rows
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (Wo - 1) * S + (K - 1) * DIL + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sDD = smem;                        // [CH][OR][Wo]
  float* sIn = sDD + a.chunk * OR * Wo;     // [CH][IR][IW]
  float* sMean = sIn + a.chunk * IR * IW;   // [C]
  float* sInv = sMean + C;
  float* sRed = sInv + C;                   // [2C] block-local BN-bwd partials (PREBN)
  float* sGW = sRed + 2 * C;                // [C*K*K] block-local depthwise weight grads
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int c = tid; c < C; c += 256) {
    if (PREBN) bn_coeffs(a.inbn, c, sMean[c], sInv[c]);
    sRed[c] = 0.f;
    sRed[C + c] = 0.f;
  }
  if (a.gW)
    for (int i = tid; i < C * KK; i += 256) sGW[i] = 0.f;
  __syncthreads();
  const int own_in = TR * S;  // own input rows [oy0*S, oy0*S + own_in)
  const int nq = own_in * W;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / tiles, oy0 = (t % tiles) * TR;
    const int iy0 = oy0 * S - pad;
    const size_t xin = (size_t)n * C * H * W;
    const float* ddn = a.dd + (size_t)n * C * Ho * Wo;
    for (int c0 = 0; c0 < C; c0 += a.chunk) {
      const int cn = min(a.chunk, C - c0);
      #pragma unroll 4  // keep several global loads of the staging pass in flight
      for (int i = tid; i < cn * OR * Wo; i += 256) {
        int cc = i / (OR * Wo), rr = (i / Wo) % OR, q = i % Wo;
        int oy = oy0 - h + rr;
        sDD[i] = (oy >= 0 && oy < Ho) ? ddn[((size_t)(c0 + cc) * Ho + oy) * Wo + q] : 0.f;
      }
      if (a.gW) {
        #pragma unroll 4  // keep several global loads of the staging pass in flight
        for (int i = tid; i < cn * IR * IW; i += 256) {
          int cc = i / (IR * IW), rr = (i / IW) % IR, q = i % IW;
          int iy = iy0 + rr, ix = -pad + q, c = c0 + cc;
          float v = 0.f;
          if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
            v = xval<PREBN>(a.x, xin + ((size_t)c * H + iy) * W + ix);
            if (PREBN) v = (v - sMean[c]) * sInv[c];
            v = fmaxf(v, 0.f);
          }
          sIn[i] = v;
        }
      }
      __syncthreads();
      // weight grads: thread per (channel, tap), summed over the tile's 64 output pixels
      if (a.gW) {
        for (int job = tid; job < cn * KK; job += 256) {
          const int cc = job / KK, tap = job % KK, ky = tap / K, kx = tap % K;
          const float* dd = sDD + (cc * OR + h) * Wo;
          const float* in = sIn + (cc * IR + ky * DIL) * IW + kx * DIL;
          float s = 0.f;
          for (int ty = 0; ty < TR; ++ty)
            for (int tx = 0; tx < Wo; ++tx) s += dd[ty * Wo + tx] * in[ty * S * IW + tx * S];
          sGW[(c0 + cc) * KK + tap] += s;  // unique owner
        }
      }
      // input grads for own input rows: the tap geometry depends only on the pixel q, so it
      // is computed once per pixel (branch-free masks) and reused for every channel. A tile
      // owns nq = 64*S*S input pixels: at stride 1 the block's 4 waves take 4 channel groups
      // of the same 64 pixels (wave-uniform channel -> scalar weight loads, wave-level sums).
      const int qspan = (nq < 256 && 256 % nq == 0) ? nq : 256;
      const int G = 256 / qspan;
      for (int q0 = 0; q0 < nq; q0 += qspan) {
        const int q = q0 + tid % qspan;
        const int cg = __builtin_amdgcn_readfirstlane(tid / qspan);
        const int rr = q / W, ix = q - rr * W;
        const int iy = oy0 * S + rr;
        const bool ok = q < nq && iy < H;
        int srow[K], ocol[K];
        float mrow[K], mcol[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          int ty = iy + pad - k * DIL;  // = oy * S when valid
          int oy = ty >= 0 ? ty / S : -1;
          bool v = ok && ty >= 0 && (ty % S) == 0 && oy < Ho;
          srow[k] = v ? oy - (oy0 - h) : 0;
          mrow[k] = v ? 1.f : 0.f;
          int tx = ix + pad - k * DIL;
          int ox = tx >= 0 ? tx / S : -1;
          bool u = ok && tx >= 0 && (tx % S) == 0 && ox < Wo;
          ocol[k] = u ? ox : 0;
          mcol[k] = u ? 1.f : 0.f;
        }
        for (int cc = cg; cc < cn; cc += G) {
          const int c = c0 + cc;
          const float* wk = a.dw + c * KK;  // wave-uniform -> scalar loads
          const float* dd = sDD + cc * OR * Wo;
          float ga = 0.f;
#pragma unroll
          for (int ky = 0; ky < K; ++ky) {
            float rowacc = 0.f;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) rowacc += mcol[kx] * wk[ky * K + kx] * dd[srow[ky] * Wo + ocol[kx]];
            ga += mrow[ky] * rowacc;
          }
          const size_t xi = ((size_t)(n * C + c) * H + iy) * W + ix;
          if (PREBN) {
            float g = 0.f, gy = 0.f;
            if (ok) {
              float y = (xval<true>(a.x, xi) - sMean[c]) * sInv[c];
              g = y > 0.f ? ga : 0.f;
              gy = g * y;
              a.gout[xi] = g;
            }
            if (a.red) {
              g = wave_sum(g);
              gy = wave_sum(gy);
              if (lane == 0) {
                atomicAdd(sRed + c, g);  // one LDS atomic per wave per channel
                atomicAdd(sRed + C + c, gy);
              }
            }
          } else if (ok) {
            const float gm = xval<false>(a.x, xi) > 0.f ? ga : 0.f;
            if (a.overwrite) a.gout[xi] = gm;
            else if (gm != 0.f) a.gout[xi] += gm;
          }
        }
      }
      __syncthreads();
    }
  }
  if (PREBN && a.red)
    for (int i = tid; i < 2 * C; i += 256) atomicAdd(a.red + rep_slot() * 2 * C + i, (double)sRed[i]);
  if (a.gW)
    for (int i = tid; i < C * KK; i += 256) atomicAdd(a.gW + (size_t)rep_slot() * a.gstride + i, sGW[i]);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// ------------------------------------------------------------------------------------------------
// pool_bwd: gx += avg^T(dz_avg) + max^T(dz_max) + wid * dout (identity skip), per (n,c) plane
// ------------------------------------------------------------------------------------------------
template <int S, bool V4 = false>
__device__ __forceinline__ void pool_bwd_body(const PoolBwdArgs& a, const int bx) {
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo, HWo = Ho * Wo;
  const int nc = bx, c = nc % C;
  const size_t ob = (size_t)nc * HWo;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sGa = smem;                                          // [HWo] dz_avg / window count
  float* sGm = smem + HWo;                                    // [HWo] dz_max
  unsigned char* sArg = (unsigned char*)(smem + 2 * HWo);     // [HWo] argmax tap
  // the plane's BN coefficients: four threads each sum one pair over the replicas
  __shared__ float sCo[8];
  if (threadIdx.x < 8) sCo[threadIdx.x] = (threadIdx.x & 1) ? 1.f : 0.f;
  __syncthreads();
  if (threadIdx.x == 0 && a.ga.z) bn_coeffs(a.ga.bn, c, sCo[0], sCo[1]);
  if (threadIdx.x == 128 && a.gm.z) bn_coeffs(a.gm.bn, c, sCo[4], sCo[5]);
  // BN-backward means: the reductions may arrive unfolded (workgroup-cooperative replica sums)
  if (a.ga.z) gs_means_coop(a.ga, c, 1, sCo + 2, sCo + 3);
  if (a.gm.z) gs_means_coop(a.gm, c, 1, sCo + 6, sCo + 7);
  __syncthreads();
  const float ma = sCo[0], ia = sCo[1], a1 = a.ga.z ? sCo[2] : 0.f, a2 = a.ga.z ? sCo[3] : 0.f;
  const float mm = sCo[4], im = sCo[5], m1 = a.gm.z ? sCo[6] : 0.f, m2 = a.gm.z ? sCo[7] : 0.f;
  const float wa = a.ga.w ? a.ga.w[a.ga.widx] : 0.f;
  const float wm = a.gm.w ? a.gm.w[a.gm.widx] : 0.f;
  const float wid = (a.w && a.id_idx >= 0) ? a.w[a.id_idx] : 0.f;
  if constexpr (V4) {
    // 4 consecutive outputs / input pixels per thread: every operand one 16-byte (amax: 4-byte)
    // access instead of four 4-byte ones - a quarter of the memory requests in flight for the
    // same bytes (HWo, H*W % 4 == 0 and every operand 16-byte aligned: host-checked)
    typedef float f4 __attribute__((ext_vector_type(4)));
    const float* gsrc = a.ga.z ? a.ga.g : a.gm.g;  // both pools read the edge's dout
    for (int o4 = threadIdx.x * 4; o4 < HWo; o4 += 1024) {
      const f4 g = *reinterpret_cast<const f4*>(gsrc + ob + o4);
      if (a.ga.z) {
        const f4 z = zld4(a.ga.z + ob + o4);
        const f4 d = wa * ia * (g - a1 - ((z - ma) * ia) * a2);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int o = o4 + t, oy = o / Wo, ox = o - oy * Wo;
          const int y0 = max(oy * S - 1, 0), y1 = min(oy * S + 1, H - 1);
          const int x0 = max(ox * S - 1, 0), x1 = min(ox * S + 1, W - 1);
          sGa[o] = d[t] / (float)((y1 - y0 + 1) * (x1 - x0 + 1));
        }
      } else {
        *reinterpret_cast<f4*>(sGa + o4) = f4{0.f, 0.f, 0.f, 0.f};
      }
      if (a.gm.z) {
        const f4 z = zld4(a.gm.z + ob + o4);
        *reinterpret_cast<f4*>(sGm + o4) = wm * im * (g - m1 - ((z - mm) * im) * m2);
        *reinterpret_cast<unsigned*>(sArg + o4) = *reinterpret_cast<const unsigned*>(a.amax + ob + o4);
      } else {
        *reinterpret_cast<f4*>(sGm + o4) = f4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<unsigned*>(sArg + o4) = 0xffffffffu;
      }
    }
    __syncthreads();
    const size_t pb = (size_t)nc * H * W;
    for (int q4 = threadIdx.x * 4; q4 < H * W; q4 += 1024) {
      f4 g = {0.f, 0.f, 0.f, 0.f};
      if (a.dout_id) g = wid * *reinterpret_cast<const f4*>(a.dout_id + pb + q4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < a.nextra) g += *reinterpret_cast<const f4*>(a.extra[j] + pb + q4);
      const int iy = q4 / W, ix0 = q4 - iy * W;  // 4 pixels of one row (W % 4 == 0)
      const int oy_lo = iy - 1 < 0 ? 0 : (iy - 1 + S - 1) / S, oy_hi = min((iy + 1) / S, Ho - 1);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int ix = ix0 + t;
        const int ox_lo = ix - 1 < 0 ? 0 : (ix - 1 + S - 1) / S, ox_hi = min((ix + 1) / S, Wo - 1);
        float v = 0.f;
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
          for (int ox = ox_lo; ox <= ox_hi; ++ox) {
            const int o = oy * Wo + ox;
            v += sGa[o];
            if (sArg[o] == (iy - oy * S + 1) * 3 + (ix - ox * S + 1)) v += sGm[o];
          }
        g[t] += v;
      }
      f4* dst = reinterpret_cast<f4*>(a.gx + pb + q4);
      *dst = a.overwrite ? g : *dst + g;
    }
    return;
  }
  for (int o = threadIdx.x; o < HWo; o += 256) {
    int oy = o / Wo, ox = o % Wo;
    if (a.ga.z) {
      int y0 = max(oy * S - 1, 0), y1 = min(oy * S + 1, H - 1);
      int x0 = max(ox * S - 1, 0), x1 = min(ox * S + 1, W - 1);
      sGa[o] = bn_bwd_val(a.ga, ob + o, ma, ia, wa, a1, a2) / (float)((y1 - y0 + 1) * (x1 - x0 + 1));
    } else {
      sGa[o] = 0.f;
    }
    if (a.gm.z) {
      sGm[o] = bn_bwd_val(a.gm, ob + o, mm, im, wm, m1, m2);
      sArg[o] = a.amax[ob + o];
    } else {
      sGm[o] = 0.f;
      sArg[o] = 255;
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < H * W; q += 256) {
    int iy = q / W, ix = q % W;
    float g = 0.f;
    // outputs whose 3x3 window (pad 1) covers (iy, ix): oy*S - 1 <= iy <= oy*S + 1
    int oy_lo = iy - 1 < 0 ? 0 : (iy - 1 + S - 1) / S, oy_hi = min((iy + 1) / S, Ho - 1);
    int ox_lo = ix - 1 < 0 ? 0 : (ix - 1 + S - 1) / S, ox_hi = min((ix + 1) / S, Wo - 1);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        int o = oy * Wo + ox;
        g += sGa[o];
        int tap = (iy - oy * S + 1) * 3 + (ix - ox * S + 1);
        if (sArg[o] == tap) g += sGm[o];
      }
    }
    if (a.dout_id) g += wid * a.dout_id[(size_t)nc * H * W + q];
#pragma unroll
    for (int j = 0; j < 4; ++j)  // the node's conv input grads (constant indices: a dynamic index into
      if (j < a.nextra) g += a.extra[j][(size_t)nc * H * W + q];  // the argument copy sends it to scratch)
    if (a.overwrite) a.gx[(size_t)nc * H * W + q] = g;
    else a.gx[(size_t)nc * H * W + q] += g;
  }
}
template <int S>
__global__ void __launch_bounds__(256) pool_bwd_kernel(PoolBwdBatch bt) {
  pool_bwd_body<S>(bt.e[blockIdx.y], blockIdx.x);
}

// stride-1 and stride-2 pool backward of a node in one launch (different edges: different gx)
template <bool V4>
__global__ void __launch_bounds__(256) pool_bwd_multi_kernel(PoolBwdBatch bt) {
  const PoolBwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x >= a.N * a.C) return;
  if (a.S == 1) pool_bwd_body<1, V4>(a, blockIdx.x);
  else pool_bwd_body<2, V4>(a, blockIdx.x);
}


// ------------------------------------------------------------------------------------------------
// dw_bwd_plane: dw_bwd for narrow layers (C <= 16), the backward twin of dwpw_plane. One
// workgroup per (image, band of input rows): the dd rows the band's input pixels reach (plus a
// zero border of PO = ceil(pad/S), so every tap lands inside the staged grid) and act(in) of the
// band are staged with one coalesced burst (and, when accumulating, the current input gradient),
// then
//   input grads : thread per own input pixel, all channels: ga = sum_taps w * dd (transposed
//                 depthwise gather from LDS), masked by act'(in); PREBN keeps the BN-backward
//                 sums per thread and reduces once per block;
//   weight grads: thread per (channel, tap[, pixel part]) summing act(in) * dd over the band.
// Every input pixel belongs to exactly one band, so both sums are complete without overlap.
// Replaces the 64-pixel tiles whose halo rows were re-staged per tile behind two barriers.
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, bool PREBN, int C>
__device__ __forceinline__ void dw_bwd_plane_body(const DwBwdArgs& a, const int bx, const int nb, const int dbg) {
  constexpr int KK = K * K, PAD = (K - 1) / 2 * DIL, PO = (PAD + S - 1) / S, SH = S == 2 ? 1 : 0;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  // channel groups: depthwise backward never mixes channels, so wider layers run as a.C / C
  // independent C-channel groups (blockIdx.x = (image * nb + band) * G + group)
  const int G = a.C / C, grp = bx % G, nbx = bx / G, c0 = grp * C;
  const int n = nbx / nb, band = nbx - n * nb;
  const int BRi = H / nb, iy0 = band * BRi, nrow = BRi;
  const int oyA = (iy0 - PAD) >> SH;                 // floor division (S in {1, 2})
  const int oyB = (iy0 + nrow - 1 + PAD) >> SH;
  const int ODR = oyB - oyA + 1, ODW = Wo + 2 * PO, NP = nrow * W;
  const bool accum = !PREBN && !a.overwrite;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sDD = smem;                    // [C][ODR][ODW]
  float* sIn = sDD + C * ODR * ODW;     // [C][nrow][W] act(in)
  float* sOld = sIn + C * NP;           // [C][nrow][W] current gradient (accumulate mode)
  __shared__ float sMean[C], sInv[C], sRed[2 * C], sGW[C * KK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < C) {
    if (PREBN) bn_coeffs(a.inbn, c0 + tid, sMean[tid], sInv[tid]);
    sRed[tid] = 0.f;
    sRed[C + tid] = 0.f;
  }
  for (int i = tid; i < C * KK; i += 256) sGW[i] = 0.f;
  __syncthreads();
  // staging with 16-byte loads (the band's rows are contiguous per channel; W, Wo % 4 == 0):
  // many wide loads in flight per wave, which the one-row-per-wave scalar loop lacked
  const float* ddn = a.dd + ((size_t)n * a.C + c0) * Ho * Wo;
  const size_t xn = ((size_t)n * a.C + c0) * H * W;
  const int va = max(oyA, 0), vb = min(oyB, Ho - 1), vrows = vb - va + 1;  // staged dd rows inside [0, Ho)
  {
    const int q4 = vrows * Wo / 4;  // float4s per channel
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4, r = o / Wo, ox = o - r * Wo;
      const float4 v = *reinterpret_cast<const float4*>(ddn + ((size_t)c * Ho + va) * Wo + o);
      float* d = sDD + (c * ODR + va - oyA + r) * ODW + PO + ox;
      d[0] = v.x;
      d[1] = v.y;
      d[2] = v.z;
      d[3] = v.w;
    }
    // zero border: rows outside [0, Ho) and the PO columns on each side
    for (int i = tid; i < C * ODR; i += 256) {
      const int c = i / ODR, oy = oyA + i - c * ODR;
      float* d = sDD + i * ODW;
      if (oy < 0 || oy >= Ho) {
        for (int q = 0; q < ODW; ++q) d[q] = 0.f;
      } else {
        for (int q = 0; q < PO; ++q) d[q] = d[PO + Wo + q] = 0.f;
      }
    }
  }
  {
    const int q4 = NP / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4;
      float4 v = xval4<PREBN>(a.x, xn + ((size_t)c * H + iy0) * W + o);
      if (PREBN) {
        const float m = sMean[c], iv = sInv[c];
        v.x = (v.x - m) * iv;
        v.y = (v.y - m) * iv;
        v.z = (v.z - m) * iv;
        v.w = (v.w - m) * iv;
      }
      v.x = fmaxf(v.x, 0.f);
      v.y = fmaxf(v.y, 0.f);
      v.z = fmaxf(v.z, 0.f);
      v.w = fmaxf(v.w, 0.f);
      *reinterpret_cast<float4*>(sIn + c * NP + o) = v;
    }
    if (accum) {
      const float* gsrc = a.gout + ((size_t)n * a.C + c0) * H * W;
#pragma unroll 4
      for (int i = tid; i < C * q4; i += 256) {
        const int c = i / q4, o = (i - c * q4) * 4;
        *reinterpret_cast<float4*>(sOld + c * NP + o) =
            *reinterpret_cast<const float4*>(gsrc + ((size_t)c * H + iy0) * W + o);
      }
    }
  }
  __syncthreads();
  // input gradients of the band's own pixels
  float st1[C], st2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) st1[c] = st2[c] = 0.f;
  float* gn = a.gout + ((size_t)n * a.C + c0) * H * W;
  if (S == 1 && a.vin) {
    // stride 1: 4 consecutive input pixels of one row per thread (W % 4 == 0, as the staging
    // assumes): the taps' column offsets are shared, and the gradient leaves as one 16-byte store
    // per channel instead of four 4-byte ones
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int p = 4 * tid; p < ((dbg & 1) ? 0 : NP); p += 1024) {
      const int r = p / W, ix = p - r * W, iy = iy0 + r;
      int srow[K], scol[K];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        srow[k] = (iy + PAD - k * DIL - oyA) * ODW;
        scol[k] = ix + PAD - k * DIL + PO;
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float* wk = a.dw + (c0 + c) * KK;  // uniform -> scalar loads
        const float* dd = sDD + c * ODR * ODW;
        f4 ga = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < K; ++ky)
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            const float w = wk[ky * K + kx];
            const float* q = dd + srow[ky] + scol[kx];
            ga.x += w * q[0];
            ga.y += w * q[1];
            ga.z += w * q[2];
            ga.w += w * q[3];
          }
        const int li = (c * nrow + r) * W + ix;
        const f4 act = *reinterpret_cast<const f4*>(sIn + li);
        const f4 g = {act.x > 0.f ? ga.x : 0.f, act.y > 0.f ? ga.y : 0.f, act.z > 0.f ? ga.z : 0.f,
                      act.w > 0.f ? ga.w : 0.f};
        f4* dst = reinterpret_cast<f4*>(gn + ((size_t)c * H + iy) * W + ix);
        if (PREBN) {
          *dst = g;
          st1[c] += (g.x + g.y) + (g.z + g.w);
          st2[c] += (g.x * act.x + g.y * act.y) + (g.z * act.z + g.w * act.w);
        } else {
          *dst = accum ? *reinterpret_cast<const f4*>(sOld + li) + g : g;
        }
      }
    }
  }
  for (int p = tid; p < ((dbg & 1) || (S == 1 && a.vin) ? 0 : NP); p += 256) {
    const int r = p / W, ix = p - r * W, iy = iy0 + r;
    int srow[K], scol[K];
    float mrow[K], mcol[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int t = iy + PAD - k * DIL, u = ix + PAD - k * DIL;
      srow[k] = ((t >> SH) - oyA) * ODW;
      scol[k] = (u >> SH) + PO;
      mrow[k] = (S == 1 || (t & 1) == 0) ? 1.f : 0.f;
      mcol[k] = (S == 1 || (u & 1) == 0) ? 1.f : 0.f;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* wk = a.dw + (c0 + c) * KK;  // uniform -> scalar loads
      const float* dd = sDD + c * ODR * ODW;
      float ga = 0.f;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        float rowacc = 0.f;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float v = wk[ky * K + kx] * dd[srow[ky] + scol[kx]];
          rowacc += S == 1 ? v : mcol[kx] * v;
        }
        ga += S == 1 ? rowacc : mrow[ky] * rowacc;
      }
      const int li = (c * nrow + r) * W + ix;
      const float act = sIn[li];
      const size_t gi = ((size_t)c * H + iy) * W + ix;
      const float g = act > 0.f ? ga : 0.f;
      if (PREBN) {
        gn[gi] = g;
        st1[c] += g;
        st2[c] += g * act;  // g * y == g * relu(y)
      } else {
        gn[gi] = accum ? sOld[li] + g : g;
      }
    }
  }
  if (PREBN && a.red) {
    float st[2 * C];  // [sum g | sum g*y], reduce-scattered over the wave
#pragma unroll
    for (int c = 0; c < C; ++c) st[c] = st1[c], st[C + c] = st2[c];
    const float v = wave_reduce_scatter<2 * C>(st);
    if ((lane & (32 / C - 1)) == 0) atomicAdd(sRed + wave_scatter_index<2 * C>(lane), v);
  }
  // depthwise weight gradients over the band: thread per (channel, tap, pixel part)
  if (a.gW && !(dbg & 2) && S == 1) {
    // stride 1: job = (channel, ky, own row). A 4-pixel quad of the input row (one 16-byte LDS
    // read) and the 4 + 2*PAD dd values it meets across all K column taps (registers) feed
    // 4*K multiply-adds: ~1.5 per LDS read against 0.5 for a pixel-by-pixel walk per tap
    const int JB = C * K * nrow;
    for (int j = tid; j < JB; j += 256) {
      const int c = j / (K * nrow), rem = j - c * K * nrow, ky = rem / nrow, r = rem - ky * nrow;
      const float* ddr = sDD + (c * ODR + iy0 + r + PAD - ky * DIL - oyA) * ODW + PO;
      const float* inr = sIn + c * NP + r * W;
      float acc[K];
#pragma unroll
      for (int kx = 0; kx < K; ++kx) acc[kx] = 0.f;
      for (int ix = 0; ix < W; ix += 4) {
        const float4 v = *reinterpret_cast<const float4*>(inr + ix);
        float dseg[4 + 2 * PAD];  // dseg[m] = dd[ix - PAD + m]
#pragma unroll
        for (int m = 0; m < 4 + 2 * PAD; ++m) dseg[m] = ddr[ix - PAD + m];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const int o = 2 * PAD - kx * DIL;  // in[ix + q] meets dd[ix + q + PAD - kx*DIL]
          acc[kx] += v.x * dseg[o] + v.y * dseg[o + 1] + v.z * dseg[o + 2] + v.w * dseg[o + 3];
        }
      }
#pragma unroll
      for (int kx = 0; kx < K; ++kx) atomicAdd(sGW + c * KK + ky * K + kx, acc[kx]);
    }
  } else if (a.gW && !(dbg & 2)) {
    constexpr int JOBS = C * KK, T = JOBS >= 256 ? 1 : 256 / JOBS;
    for (int j = tid; j < JOBS * T; j += 256) {
      const int job = j / T, part = j - job * T;
      const int c = job / KK, tap = job - c * KK, ky = tap / K, kx = tap - ky * K;
      const float* dd = sDD + c * ODR * ODW;
      const float* in = sIn + c * NP;
      float acc = 0.f;
      for (int r = 0; r < nrow; ++r) {
        const int t = iy0 + r + PAD - ky * DIL;
        if (S == 2 && (t & 1)) continue;
        const float* ddr = dd + ((t >> SH) - oyA) * ODW + PO;
        const float* inr = in + r * W;
        for (int ix = part * S + ((S == 2) ? ((PAD - kx * DIL) & 1) : 0); ix < W; ix += T * S)
          acc += inr[ix] * ddr[(ix + PAD - kx * DIL) >> SH];
      }
      atomicAdd(sGW + job, acc);
    }
  }
  __syncthreads();
  if (PREBN && a.red && tid < 2 * C)  // red replica layout [sum g: a.C | sum g*y: a.C]
    atomicAdd(a.red + rep_slot() * 2 * a.C + (tid < C ? c0 + tid : a.C + c0 + tid - C), (double)sRed[tid]);
  if (a.gW)
    for (int i = tid; i < C * KK; i += 256) atomicAdd(a.gW + (size_t)rep_slot() * a.gstride + c0 * KK + i, sGW[i]);
}

template <int K, int DIL, int S, bool PREBN, int C>
__global__ void __launch_bounds__(256) dw_bwd_plane_kernel(DwBwdBatch bt, int nb, int dbg) {
  dw_bwd_plane_body<K, DIL, S, PREBN, C>(bt.e[blockIdx.y], blockIdx.x, nb, dbg);
  if (bt.tail.ctr) fold_tail(bt.tail);
}

// Mixed-variant depthwise backward: one launch for entries of different kernel size / dilation /
// stride / input BN that write DISTINCT outputs - a node's separable second stages (3x3 and 5x5,
// input BN), or a node's stage-1 separable and dilated convolutions each writing its own
// (masked) input-gradient buffer that the pool backward then sums into gx. Each entry carries
// its variant (dw_bwd_variant), band count and workgroup count.
#define DWB_CASE(KK, DD, SS, PB) \
  case dw_bwd_variant(KK, DD, SS, PB): dw_bwd_plane_body<KK, DD, SS, PB, C>(a, blockIdx.x, a.nbands, 0); break;
template <int C>
__global__ void __launch_bounds__(256) dw_bwd_plane_multi_kernel(DwBwdBatch bt) {
  const DwBwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x < a.nblk) {
    switch (a.variant) {
      DWB_CASE(3, 1, 1, true) DWB_CASE(5, 1, 1, true)
      DWB_CASE(3, 1, 1, false) DWB_CASE(3, 1, 2, false) DWB_CASE(5, 1, 1, false) DWB_CASE(5, 1, 2, false)
      DWB_CASE(3, 2, 1, false) DWB_CASE(3, 2, 2, false) DWB_CASE(5, 2, 1, false) DWB_CASE(5, 2, 2, false)
      default: break;
    }
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}
#undef DWB_CASE

// ------------------------------------------------------------------------------------------------
// edge_bwd: the whole input gradient of one edge in one pass (cf. dw_bwd_plane_kernel, whose band
// layout it shares). Workgroup = (image, band of input rows, C-channel group); act = relu(x) of
// the band is staged once and the gradient is accumulated in LDS:
//   conv slots (sep 3x3 / 5x5 stage 1, dil 3x3 / 5x5): dd of the slot staged with its halo, the
//     transposed depthwise gather added to sGX, the slot's depthwise weight gradient reduced in
//     LDS and flushed with one atomic per weight (replica rep_slot());
//   pools: dz_avg / window count and dz_max (BN backward on the fly from the combine reductions)
//     of the output rows the band reaches, plus the argmax taps, staged and gathered;
//   identity: w_id * dout.
// gx = relu'(x) * conv + pool + identity, written (or added) once per element. Replaces the
// per-(K, S) dw_bwd launches, the pool backward and the identity add of a node: 4-10 launches
// that each re-read and re-wrote gx.
// ------------------------------------------------------------------------------------------------
template <int K, int DIL, int S, int C>
__device__ __forceinline__ void edge_conv_part(const EdgeBwdArgs& a, const int v, const int n, const int c0,
                                               const int iy0, const int nrow, float* sDD, const float* sAct,
                                               float* sGX, float* sGW) {
  constexpr int KK = K * K, PAD = (K - 1) / 2 * DIL, PO = (PAD + S - 1) / S, SH = S == 2 ? 1 : 0;
  const int W = a.W, Ho = a.Ho, Wo = a.Wo, NP = nrow * W;
  const int oyA = (iy0 - PAD) >> SH, oyB = (iy0 + nrow - 1 + PAD) >> SH;
  const int ODR = oyB - oyA + 1, ODW = Wo + 2 * PO;
  const int tid = threadIdx.x;
  const float* ddn = a.dd[v] + ((size_t)n * a.C + c0) * Ho * Wo;
  const int va = max(oyA, 0), vb = min(oyB, Ho - 1), vrows = vb - va + 1;
  {
    const int q4 = vrows * Wo / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4, r = o / Wo, ox = o - r * Wo;
      const float4 f = *reinterpret_cast<const float4*>(ddn + ((size_t)c * Ho + va) * Wo + o);
      float* d = sDD + (c * ODR + va - oyA + r) * ODW + PO + ox;
      d[0] = f.x;
      d[1] = f.y;
      d[2] = f.z;
      d[3] = f.w;
    }
    for (int i = tid; i < C * ODR; i += 256) {
      const int c = i / ODR, oy = oyA + i - c * ODR;
      float* d = sDD + i * ODW;
      if (oy < 0 || oy >= Ho) {
        for (int q = 0; q < ODW; ++q) d[q] = 0.f;
      } else {
        for (int q = 0; q < PO; ++q) d[q] = d[PO + Wo + q] = 0.f;
      }
    }
    for (int i = tid; i < C * KK; i += 256) sGW[i] = 0.f;
  }
  __syncthreads();
  for (int p = tid; p < NP; p += 256) {
    const int r = p / W, ix = p - r * W, iy = iy0 + r;
    int srow[K], scol[K];
    float mrow[K], mcol[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int t = iy + PAD - k * DIL, u = ix + PAD - k * DIL;
      srow[k] = ((t >> SH) - oyA) * ODW;
      scol[k] = (u >> SH) + PO;
      mrow[k] = (S == 1 || (t & 1) == 0) ? 1.f : 0.f;
      mcol[k] = (S == 1 || (u & 1) == 0) ? 1.f : 0.f;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float* wk = a.dw[v] + (c0 + c) * KK;  // uniform -> scalar loads
      const float* dd = sDD + c * ODR * ODW;
      float ga = 0.f;
#pragma unroll
      for (int ky = 0; ky < K; ++ky) {
        float rowacc = 0.f;
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
          const float t = wk[ky * K + kx] * dd[srow[ky] + scol[kx]];
          rowacc += S == 1 ? t : mcol[kx] * t;
        }
        ga += S == 1 ? rowacc : mrow[ky] * rowacc;
      }
      sGX[c * NP + p] += ga;  // own pixel: no other thread touches it
    }
  }
  if (a.gW[v]) {
    if (S == 1) {
      // job = (channel, ky, own row): 4-pixel input quads against the dd row segment they meet
      const int JB = C * K * nrow;
      for (int j = tid; j < JB; j += 256) {
        const int c = j / (K * nrow), rem = j - c * K * nrow, ky = rem / nrow, r = rem - ky * nrow;
        const float* ddr = sDD + (c * ODR + iy0 + r + PAD - ky * DIL - oyA) * ODW + PO;
        const float* inr = sAct + c * NP + r * W;
        float acc[K];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) acc[kx] = 0.f;
        for (int ix = 0; ix < W; ix += 4) {
          const float4 f = *reinterpret_cast<const float4*>(inr + ix);
          float dseg[4 + 2 * PAD];
#pragma unroll
          for (int m = 0; m < 4 + 2 * PAD; ++m) dseg[m] = ddr[ix - PAD + m];
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            const int o = 2 * PAD - kx * DIL;
            acc[kx] += f.x * dseg[o] + f.y * dseg[o + 1] + f.z * dseg[o + 2] + f.w * dseg[o + 3];
          }
        }
#pragma unroll
        for (int kx = 0; kx < K; ++kx) atomicAdd(sGW + c * KK + ky * K + kx, acc[kx]);
      }
    } else {
      constexpr int JOBS = C * KK, T = JOBS >= 256 ? 1 : 256 / JOBS;
      for (int j = tid; j < JOBS * T; j += 256) {
        const int job = j / T, part = j - job * T;
        const int c = job / KK, tap = job - c * KK, ky = tap / K, kx = tap - ky * K;
        const float* dd = sDD + c * ODR * ODW;
        const float* in = sAct + c * NP;
        float acc = 0.f;
        for (int r = 0; r < nrow; ++r) {
          const int t = iy0 + r + PAD - ky * DIL;
          if (t & 1) continue;
          const float* ddr = dd + ((t >> SH) - oyA) * ODW + PO;
          const float* inr = in + r * W;
          for (int ix = part * S + ((PAD - kx * DIL) & 1); ix < W; ix += T * S)
            acc += inr[ix] * ddr[(ix + PAD - kx * DIL) >> SH];
        }
        atomicAdd(sGW + job, acc);
      }
    }
  }
  __syncthreads();
  if (a.gW[v])
    for (int i = tid; i < C * KK; i += 256) atomicAdd(a.gW[v] + (size_t)rep_slot() * a.gstride[v] + c0 * KK + i, sGW[i]);
  __syncthreads();  // sDD / sGW are restaged by the next slot
}

template <int S, int C>
__device__ __forceinline__ void edge_bwd_body(const EdgeBwdArgs& a, const int bx) {
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int G = a.C / C, grp = bx % G, nbx = bx / G, c0 = grp * C;
  const int n = nbx / a.nb, band = nbx - n * a.nb;
  const int nrow = H / a.nb, iy0 = band * nrow, NP = nrow * W;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sAct = smem;           // [C][NP] relu(x)
  float* sGX = sAct + C * NP;   // [C][NP] conv gradient (pre-mask)
  float* sDD = sGX + C * NP;    // staging: one conv slot's dd band, or the pool gradients
  __shared__ float sGW[C * 25];
  __shared__ float sCo[C][10];
  const int tid = threadIdx.x;
  const float* xn = a.x + ((size_t)n * a.C + c0) * H * W;
  {
    const int q4 = NP / 4;
#pragma unroll 4
    for (int i = tid; i < C * q4; i += 256) {
      const int c = i / q4, o = (i - c * q4) * 4;
      float4 f = *reinterpret_cast<const float4*>(xn + ((size_t)c * H + iy0) * W + o);
      f.x = fmaxf(f.x, 0.f);
      f.y = fmaxf(f.y, 0.f);
      f.z = fmaxf(f.z, 0.f);
      f.w = fmaxf(f.w, 0.f);
      *reinterpret_cast<float4*>(sAct + c * NP + o) = f;
      *reinterpret_cast<float4*>(sGX + c * NP + o) = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  const bool pa = a.ga.z != nullptr, pm = a.gm.z != nullptr;
  if (tid < C) {  // pool BN coefficients and softmax weights per channel
    float* co = sCo[tid];
    co[0] = 0.f; co[1] = 1.f; co[2] = 0.f; co[3] = 0.f; co[4] = 0.f; co[5] = 1.f; co[6] = 0.f; co[7] = 0.f;
    if (pa) {
      bn_coeffs(a.ga.bn, c0 + tid, co[0], co[1]);
      gs_means(a.ga, c0 + tid, co[2], co[3]);
    }
    if (pm) {
      bn_coeffs(a.gm.bn, c0 + tid, co[4], co[5]);
      gs_means(a.gm, c0 + tid, co[6], co[7]);
    }
    co[8] = pa && a.ga.w ? a.ga.w[a.ga.widx] : 1.f;
    co[9] = pm && a.gm.w ? a.gm.w[a.gm.widx] : 1.f;
  }
  __syncthreads();
  if (a.conv_mask & 1) edge_conv_part<3, 1, S, C>(a, 0, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  if (a.conv_mask & 2) edge_conv_part<5, 1, S, C>(a, 1, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  if (a.conv_mask & 4) edge_conv_part<3, 2, S, C>(a, 2, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  if (a.conv_mask & 8) edge_conv_part<5, 2, S, C>(a, 3, n, c0, iy0, nrow, sDD, sAct, sGX, sGW);
  // pools: output rows whose 3x3 window (pad 1) touches the band's input rows
  const int poA = max(0, (iy0 - 1 + S - 1) / S), poB = min(Ho - 1, (iy0 + nrow) / S);
  const int PR = poB - poA + 1, PP = PR * Wo;
  float* sGa = sDD;
  float* sGm = sDD + C * PP;
  unsigned char* sArg = reinterpret_cast<unsigned char*>(sDD + 2 * C * PP);
  if (pa || pm) {
    for (int i = tid; i < C * PP; i += 256) {
      const int c = i / PP, o = poA * Wo + (i - c * PP), oy = o / Wo, ox = o - oy * Wo;
      const size_t idx = ((size_t)n * a.C + c0 + c) * Ho * Wo + o;
      const float* co = sCo[c];
      float gav = 0.f, gmv = 0.f;
      unsigned char arg = 255;
      if (pa) {
        const int y0 = max(oy * S - 1, 0), y1 = min(oy * S + 1, H - 1);
        const int x0 = max(ox * S - 1, 0), x1 = min(ox * S + 1, W - 1);
        gav = bn_bwd_val(a.ga, idx, co[0], co[1], co[8], co[2], co[3]) / (float)((y1 - y0 + 1) * (x1 - x0 + 1));
      }
      if (pm) {
        gmv = bn_bwd_val(a.gm, idx, co[4], co[5], co[9], co[6], co[7]);
        arg = a.amax[idx];
      }
      sGa[i] = gav;
      sGm[i] = gmv;
      sArg[i] = arg;
    }
    __syncthreads();
  }
  const float wid = (a.dout_id && a.w && a.id_idx >= 0) ? a.w[a.id_idx] : 0.f;
  for (int p = tid; p < NP; p += 256) {
    const int r = p / W, ix = p - r * W, iy = iy0 + r;
    const int oy_lo = iy - 1 < 0 ? 0 : (iy - 1 + S - 1) / S, oy_hi = min((iy + 1) / S, Ho - 1);
    const int ox_lo = ix - 1 < 0 ? 0 : (ix - 1 + S - 1) / S, ox_hi = min((ix + 1) / S, Wo - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float g = sAct[c * NP + p] > 0.f ? sGX[c * NP + p] : 0.f;
      if (pa || pm) {
        for (int oy = oy_lo; oy <= oy_hi; ++oy)
          for (int ox = ox_lo; ox <= ox_hi; ++ox) {
            const int o = c * PP + (oy - poA) * Wo + ox;
            g += sGa[o];
            if (sArg[o] == (iy - oy * S + 1) * 3 + (ix - ox * S + 1)) g += sGm[o];
          }
      }
      const size_t gi = ((size_t)n * a.C + c0 + c) * H * W + (size_t)iy * W + ix;
      if (a.dout_id) g += wid * a.dout_id[gi];
      a.gx[gi] = a.overwrite ? g : a.gx[gi] + g;
    }
  }
}

template <int C>
__global__ void __launch_bounds__(256) edge_bwd_kernel(EdgeBwdBatch bt) {
  const EdgeBwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x >= a.nblk) return;
  if (a.S == 1) edge_bwd_body<1, C>(a, blockIdx.x);
  else edge_bwd_body<2, C>(a, blockIdx.x);
}

// LDS floats of one edge_bwd band: act + gradient planes, then the larger of the widest conv
// slot's staged dd band and the pool staging
static size_t edge_bwd_floats(const EdgeBwdArgs& a, int nb, int CG) {
  const int nrow = a.H / nb, S = a.S, sh = S == 2 ? 1 : 0;
  auto fdiv = [sh](int v) { return v >= 0 ? v >> sh : -((-v + (1 << sh) - 1) >> sh); };
  size_t stage = 0;
  const int pads[4] = {1, 2, 2, 4};
  for (int v = 0; v < 4; ++v) {
    if (!(a.conv_mask & (1 << v))) continue;
    const int PAD = pads[v], PO = (PAD + S - 1) / S;
    const int ODR = fdiv(nrow - 1 + PAD) - fdiv(-PAD) + 2;
    stage = std::max(stage, (size_t)CG * ODR * (a.Wo + 2 * PO));
  }
  if (a.ga.z || a.gm.z) {
    const size_t PP = (size_t)(nrow / S + 3) * a.Wo;
    stage = std::max(stage, 2 * CG * PP + (CG * PP + 3) / 4);
  }
  return 2 * (size_t)CG * nrow * a.W + stage;
}

bool launch_edge_bwd(EdgeBwdBatch b, hipStream_t st) {
  if (b.n < 1) return true;
  const int C = b.e[0].C, N = b.e[0].N;
  if (!(C == 4 || (C % 8 == 0 && C <= kMaxC))) return false;
  const int CG = C == 4 ? 4 : 8, G = C / CG;
  int maxblk = 0;
  size_t lds = 0;
  for (int i = 0; i < b.n; ++i) {
    EdgeBwdArgs& a = b.e[i];
    if (a.C != C || a.N != N || a.H != a.Ho * a.S || a.W != a.Wo * a.S || a.W % 4 || a.Wo % 4) return false;
    uintptr_t bits = (uintptr_t)a.x;
    for (int v = 0; v < 4; ++v)
      if (a.conv_mask & (1 << v)) bits |= (uintptr_t)a.dd[v];
    if (bits & 15) return false;
    // bands: LDS per workgroup <= KATIB_HIP_EDGE_LDS_KB and >= KATIB_HIP_EDGE_WG workgroups per launch
    static const int lds_kb = getenv("KATIB_HIP_EDGE_LDS_KB") ? atoi(getenv("KATIB_HIP_EDGE_LDS_KB")) : 48;
    static const int min_wg = getenv("KATIB_HIP_EDGE_WG") ? atoi(getenv("KATIB_HIP_EDGE_WG")) : 1024;
    int nb = 1;
    while (nb < 32 && a.H % (2 * nb) == 0 &&
           (edge_bwd_floats(a, nb, CG) * 4 > (size_t)lds_kb * 1024 || N * nb * G * b.n < min_wg))
      nb *= 2;
    if (edge_bwd_floats(a, nb, CG) * 4 > 64 * 1024) return false;
    a.nb = nb;
    a.nblk = N * nb * G;
    maxblk = std::max(maxblk, a.nblk);
    lds = std::max(lds, edge_bwd_floats(a, nb, CG) * sizeof(float));
  }
  const dim3 grid(maxblk, b.n);
  if (CG == 4) hipLaunchKernelGGL(edge_bwd_kernel<4>, grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL(edge_bwd_kernel<8>, grid, dim3(256), lds, st, b);
  return true;
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
static int per_edge_blocks(int tiles, int n) { return std::max(1, std::min(tiles, max_blocks() / std::max(n, 1))); }

template <int K, int DIL, int S, int C>
static void launch_dwpw_plane_t(const DwPwFwdBatch& b, bool prebn, hipStream_t st) {
  const DwPwFwdArgs& a = b.e[0];
  const int nb = a.chunk, BR = (a.Ho + nb - 1) / nb;
  const size_t lds = sizeof(float) * C * ((BR - 1) * S + (K - 1) * DIL + 1) * (a.W + 2 * a.pad);
  dim3 grid(a.N * nb, b.n);
  // 16-byte staging when every row is whole float4s and every input is 16-byte aligned
  bool vec = a.W % 4 == 0;
  for (int i = 0; i < b.n; ++i) vec &= ((uintptr_t)b.e[i].x & 15) == 0;
  if (vec) {
    if (prebn) hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, true, C, true>), grid, dim3(256), lds, st, b);
    else hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, false, C, true>), grid, dim3(256), lds, st, b);
  } else {
    if (prebn) hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, true, C, false>), grid, dim3(256), lds, st, b);
    else hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, false, C, false>), grid, dim3(256), lds, st, b);
  }
}

// row-band kernel for C = 4 / 8 / 16 (the staged band fits 64 KB of LDS by construction)
static bool plane_ok(const DwPwFwdArgs& a) { return a.C == 4 || a.C == 8 || a.C == 16; }

template <int CI, int CO>
static bool try_pw_fwd_wave(const PwFwdBatch& b, hipStream_t st);

template <int K, int DIL, int S, int CG>
static bool try_dwpw_split_g(const DwPwFwdBatch& b, bool prebn, hipStream_t st, bool split16);

// layers of 16..64 channels: depthwise on channel groups (dwpw_plane_kernel<..., PW = false>), then
// the pointwise + BN statistics as an MFMA GEMM over d (pw_fwd_wave_kernel). At C = 16 this measured
// faster than the fused plane kernel (50.7 vs 52.5 ms per darts-gpu.yaml step); KATIB_HIP_DWPW_SPLIT=0
// keeps the fused kernel there.
template <int K, int DIL, int S>
static bool try_dwpw_split(const DwPwFwdBatch& b, bool prebn, hipStream_t st) {
  const DwPwFwdArgs& a = b.e[0];
  static const bool split16 = !getenv("KATIB_HIP_DWPW_SPLIT") || atoi(getenv("KATIB_HIP_DWPW_SPLIT")) > 0;
  static const int grp = getenv("KATIB_HIP_DW_GROUP") ? atoi(getenv("KATIB_HIP_DW_GROUP")) : 8;
  if (grp == 4) return try_dwpw_split_g<K, DIL, S, 4>(b, prebn, st, split16);
  if (grp == 8) return try_dwpw_split_g<K, DIL, S, 8>(b, prebn, st, split16);
  return try_dwpw_split_g<K, DIL, S, 16>(b, prebn, st, split16);
}

template <int K, int DIL, int S, int CG>
static bool try_dwpw_split_g(const DwPwFwdBatch& b, bool prebn, hipStream_t st, bool split16) {
  const DwPwFwdArgs& a = b.e[0];
  if (getenv("KATIB_HIP_DWPW_TILED") || a.C % 16 != 0 || a.C > 64 || (a.C == 16 && !split16) ||
      (a.Ho * a.Wo) % 64 != 0 || a.W % 4 != 0)
    return false;
  for (int i = 0; i < b.n; ++i)
    if (((uintptr_t)b.e[i].x | (uintptr_t)b.e[i].d | (uintptr_t)b.e[i].z) & 15) return false;
  const int G = a.C / CG;
  int nb = std::max(1, std::min(a.Ho / 4, 2048 / std::max(a.N * b.n * G, 1)));
  auto band_bytes = [&](int v) {
    const int BR = (a.Ho + v - 1) / v;
    return (size_t)CG * ((BR - 1) * S + (K - 1) * DIL + 1) * (a.W + 2 * a.pad) * sizeof(float);
  };
  while (band_bytes(nb) > 65536 && nb < a.Ho) ++nb;
  DwPwFwdBatch db = b;
  db.tail.ctr = nullptr;  // the statistics come from the pointwise launch below, which folds them
  for (int i = 0; i < b.n; ++i) db.e[i].chunk = nb;
  dim3 grid(a.N * nb * G, b.n);
  const size_t lds = band_bytes(nb);
  if (prebn) hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, true, CG, true, false>), grid, dim3(256), lds, st, db);
  else hipLaunchKernelGGL((dwpw_plane_kernel<K, DIL, S, false, CG, true, false>), grid, dim3(256), lds, st, db);
  PwFwdBatch pb{};
  pb.n = b.n;
  pb.tail = b.tail;
  for (int i = 0; i < b.n; ++i) {
    const DwPwFwdArgs& e = b.e[i];
    PwFwdArgs& p = pb.e[i];
    p.x = e.d; p.pw = e.pw; p.z = e.z; p.stats = e.stats;
    p.N = e.N; p.Cin = e.C; p.Cout = e.C; p.CoutTotal = e.C; p.co_off = 0;
    p.H = e.Ho; p.W = e.Wo; p.Ho = e.Ho; p.Wo = e.Wo; p.S = 1; p.off = 0; p.relu = 0;
  }
  if (try_pw_fwd_wave<16, 16>(pb, st) || try_pw_fwd_wave<32, 32>(pb, st) || try_pw_fwd_wave<64, 64>(pb, st))
    return true;
  launch_pw_fwd(pb, st);  // C = 48: the generic dispatch
  return true;
}

template <int K, int DIL, int S>
static void launch_dwpw_fwd_t(const DwPwFwdBatch& b, bool prebn, hipStream_t st) {
  const DwPwFwdArgs& a = b.e[0];
  if (try_dwpw_split<K, DIL, S>(b, prebn, st)) return;
  if (plane_ok(a)) {
    if (a.C == 4) return launch_dwpw_plane_t<K, DIL, S, 4>(b, prebn, st);
    if (a.C == 8) return launch_dwpw_plane_t<K, DIL, S, 8>(b, prebn, st);
    return launch_dwpw_plane_t<K, DIL, S, 16>(b, prebn, st);
  }
  const int TR = 64 / a.Wo;
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (a.Wo - 1) * S + (K - 1) * DIL + 1;
  size_t lds = sizeof(float) * (a.C * 64 + a.chunk * IR * IW + 4 * a.C);
  dim3 grid(per_edge_blocks(a.N * (a.Ho / TR), b.n), b.n);
  if (prebn) hipLaunchKernelGGL((dwpw_fwd_kernel<K, DIL, S, true>), grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL((dwpw_fwd_kernel<K, DIL, S, false>), grid, dim3(256), lds, st, b);
}

void launch_dwpw_fwd(const DwPwFwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st) {
#define DISPATCH(KK, DD, SS) \
  if (K == KK && dil == DD && S == SS) return launch_dwpw_fwd_t<KK, DD, SS>(b, prebn, st);
  DISPATCH(3, 1, 1) DISPATCH(3, 1, 2) DISPATCH(5, 1, 1) DISPATCH(5, 1, 2)
  DISPATCH(3, 2, 1) DISPATCH(3, 2, 2) DISPATCH(5, 2, 1) DISPATCH(5, 2, 2)
#undef DISPATCH
}

// ------------------------------------------------------------------------------------------------
// Mixed-variant launches (one per node stage instead of one per (K, dil, S) group). The entries
// must share the channel count; returns false (nothing launched) when they do not fit the plane
// kernels, and the caller falls back to the per-group launches.
// ------------------------------------------------------------------------------------------------
static int channel_groups(int N, int C, int n);

bool launch_dwpw_multi(DwPwMultiBatch b, hipStream_t st) {
  if (b.n < 1) return true;
  const int C = b.e[0].C, N = b.e[0].N;
  static const bool split16 = !getenv("KATIB_HIP_DWPW_SPLIT") || atoi(getenv("KATIB_HIP_DWPW_SPLIT")) > 0;
  const bool fused = C == 4 || C == 8 || (C == 16 && !split16);
  const bool split = !fused && C % 16 == 0 && C <= 64;
  if (!fused && !split) return false;
  const int CG = fused ? C : 8, G = C / CG;
  int maxblk = 0;
  size_t lds = 0;
  for (int i = 0; i < b.n; ++i) {
    DwPwFwdArgs& a = b.e[i];
    if (a.C != C || a.N != N) return false;
    const int code = a.variant >> 2;
    const int K = (code & 4) ? 5 : 3, DIL = (code & 2) ? 2 : 1, S = (code & 1) ? 2 : 1;
    const bool aligned = ((((uintptr_t)a.x) | (uintptr_t)a.d | (uintptr_t)a.z) & 15) == 0;
    if (split && (!aligned || (a.Ho * a.Wo) % 64 != 0 || a.W % 4 != 0)) return false;
    int nb = std::max(1, std::min(a.Ho / 4, 2048 / std::max(N * b.n * G, 1)));
    auto band_bytes = [&](int v) {
      const int BR = (a.Ho + v - 1) / v;
      return (size_t)CG * ((BR - 1) * S + (K - 1) * DIL + 1) * (a.W + 2 * a.pad) * sizeof(float);
    };
    while (band_bytes(nb) > 65536 && nb < a.Ho) ++nb;
    a.chunk = nb;
    a.nblk = N * nb * G;
    const bool vec = a.W % 4 == 0 && (((uintptr_t)a.x) & 15) == 0;
    a.variant = (a.variant & ~1) | (vec ? 1 : 0);
    a.vout = (vec_mask() >> (CG == 4 ? 0 : 1)) & 1;
    maxblk = std::max(maxblk, a.nblk);
    lds = std::max(lds, band_bytes(nb));
  }
  const dim3 grid(maxblk, b.n);
  if (fused) {
    if (C == 4) hipLaunchKernelGGL((dwpw_plane_multi_kernel<4, true>), grid, dim3(256), lds, st, b);
    else if (C == 8) hipLaunchKernelGGL((dwpw_plane_multi_kernel<8, true>), grid, dim3(256), lds, st, b);
    else hipLaunchKernelGGL((dwpw_plane_multi_kernel<16, true>), grid, dim3(256), lds, st, b);
    return true;
  }
  {
    DwPwMultiBatch db = b;
    db.tail.ctr = nullptr;  // statistics (and their fold) come from the pointwise launch
    hipLaunchKernelGGL((dwpw_plane_multi_kernel<8, false>), grid, dim3(256), lds, st, db);
  }
  // the pointwise halves + BN statistics of every entry: one MFMA wave launch
  PwFwdBatch pb{};
  pb.n = b.n;
  pb.tail = b.tail;  // per-entry launches below share the counter: they run one after another
  for (int i = 0; i < b.n; ++i) {
    const DwPwFwdArgs& e = b.e[i];
    PwFwdArgs& p = pb.e[i];
    p.x = e.d; p.pw = e.pw; p.z = e.z; p.stats = e.stats;
    p.N = e.N; p.Cin = e.C; p.Cout = e.C; p.CoutTotal = e.C; p.co_off = 0;
    p.H = e.Ho; p.W = e.Wo; p.Ho = e.Ho; p.Wo = e.Wo; p.S = 1; p.off = 0; p.relu = 0;
  }
  bool same_hw = true;
  for (int i = 1; i < b.n; ++i) same_hw &= b.e[i].Ho == b.e[0].Ho && b.e[i].Wo == b.e[0].Wo;
  if (same_hw && (try_pw_fwd_wave<16, 16>(pb, st) || try_pw_fwd_wave<32, 32>(pb, st) || try_pw_fwd_wave<64, 64>(pb, st)))
    return true;
  for (int i = 0; i < b.n; ++i) {  // mixed output sizes (stride-1 and stride-2 entries): per entry
    PwFwdBatch one{};
    one.n = 1;
    one.tail = pb.tail;
    one.e[0] = pb.e[i];
    if (!(try_pw_fwd_wave<16, 16>(one, st) || try_pw_fwd_wave<32, 32>(one, st) || try_pw_fwd_wave<64, 64>(one, st)))
      launch_pw_fwd(one, st);
  }
  return true;
}

void launch_pool_fwd_multi(PoolFwdBatch b, hipStream_t st) {
  int maxblk = 0;
  for (int i = 0; i < b.n; ++i) {
    PoolFwdArgs& a = b.e[i];
    a.nblk = a.C * channel_groups(a.N, a.C, b.n);
    maxblk = std::max(maxblk, a.nblk);
  }
  hipLaunchKernelGGL(pool_fwd_multi_kernel, dim3(maxblk, b.n), dim3(256), 0, st, b);
}

void launch_pool_bwd_multi(const PoolBwdBatch& b, hipStream_t st) {
  int maxblk = 0;
  size_t lds = 0;
  bool v4 = !getenv("KATIB_HIP_POOL_BWD_SCALAR");
  auto al = [](const void* p, uintptr_t m) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & (m - 1)) == 0; };
  for (int i = 0; i < b.n; ++i) {
    const PoolBwdArgs& a = b.e[i];
    maxblk = std::max(maxblk, a.N * a.C);
    lds = std::max(lds, sizeof(float) * 2 * a.Ho * a.Wo + a.Ho * a.Wo + 16);
    v4 = v4 && (a.Ho * a.Wo) % 4 == 0 && (a.H * a.W) % 4 == 0 && a.W % 4 == 0 && al(a.ga.g, 16) && al(a.gm.g, 16) &&
         al(a.ga.z, 4 * sizeof(zt)) && al(a.gm.z, 4 * sizeof(zt)) && al(a.amax, 4) && al(a.dout_id, 16) &&
         al(a.gx, 16) && (!a.ga.z || !a.gm.z || a.ga.g == a.gm.g);
    for (int j = 0; j < a.nextra; ++j) v4 = v4 && al(a.extra[j], 16);
  }
  if (v4) hipLaunchKernelGGL(pool_bwd_multi_kernel<true>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  else hipLaunchKernelGGL(pool_bwd_multi_kernel<false>, dim3(maxblk, b.n), dim3(256), lds, st, b);
}

// LDS floats of one dw_bwd_plane band (nb bands per image)
static size_t dw_plane_floats(const DwBwdArgs& a, int K, int DIL, int S, int nb, bool accum, int C) {
  const int PAD = (K - 1) / 2 * DIL, PO = (PAD + S - 1) / S, sh = S == 2 ? 1 : 0, BRi = a.H / nb;
  auto fdiv = [sh](int v) { return v >= 0 ? v >> sh : -((-v + (1 << sh) - 1) >> sh); };
  const int ODR = fdiv(BRi - 1 + PAD) - fdiv(-PAD) + 2;  // +1: odd bands start at odd rows
  return (size_t)C * ODR * (a.Wo + 2 * PO) + (size_t)C * BRi * a.W * (accum ? 2 : 1);
}

template <int K, int DIL, int S, int C>
static void launch_dw_bwd_plane_t(const DwBwdBatch& b, bool prebn, hipStream_t st) {
  const DwBwdArgs& a = b.e[0];
  bool accum = false;
  for (int i = 0; i < b.n; ++i) accum |= !prebn && !b.e[i].overwrite;
  // bands: as few as possible (less halo) while the launch still has ~4 workgroups per CU and a
  // band stays within 40 KB of LDS
  int nb = 1;
  const int G = a.C / C;  // channel groups per image
  while (nb < 8 && a.H % (2 * nb) == 0 &&
         (dw_plane_floats(a, K, DIL, S, nb, accum, C) * 4 > 40 * 1024 || a.N * nb * G * b.n < 1024))
    nb *= 2;
  const size_t lds = sizeof(float) * dw_plane_floats(a, K, DIL, S, nb, accum, C);
  dim3 grid(a.N * nb * G, b.n);
  static const int dbg = getenv("KATIB_HIP_DWB_DBG") ? atoi(getenv("KATIB_HIP_DWB_DBG")) : 0;  // timing probes
  if (prebn) hipLaunchKernelGGL((dw_bwd_plane_kernel<K, DIL, S, true, C>), grid, dim3(256), lds, st, b, nb, dbg);
  else hipLaunchKernelGGL((dw_bwd_plane_kernel<K, DIL, S, false, C>), grid, dim3(256), lds, st, b, nb, dbg);
}

static bool aligned16(const DwBwdBatch& b) {
  for (int i = 0; i < b.n; ++i)
    if (((uintptr_t)b.e[i].x | (uintptr_t)b.e[i].dd | (uintptr_t)b.e[i].gout) & 15) return false;
  return true;
}

// plane path: narrow layers whose spatial sizes divide exactly by the stride
static bool dw_plane_ok(const DwBwdBatch& b, int K, int DIL, int S) {
  if (getenv("KATIB_HIP_DW_BWD_TILED")) return false;
  const DwBwdArgs& a = b.e[0];
  return (a.C == 4 || a.C == 8 || (a.C % 16 == 0 && a.C <= kMaxC)) && a.H == a.Ho * S && a.W == a.Wo * S &&
         a.pad == (K - 1) / 2 * DIL && a.Wo % 4 == 0 && aligned16(b);
}

template <int K, int DIL, int S>
static void launch_dw_bwd_t(const DwBwdBatch& b, bool prebn, hipStream_t st) {
  const DwBwdArgs& a = b.e[0];
  if (dw_plane_ok(b, K, DIL, S)) {
    // wide layers run in channel groups of KATIB_HIP_DWB_GROUP (4, 8 or 16) channels: 8 measured
    // 48.2 vs 50.8 ms per darts-gpu.yaml step against 16 (half the LDS per band: fewer, taller bands)
    static const int grp = getenv("KATIB_HIP_DWB_GROUP") ? atoi(getenv("KATIB_HIP_DWB_GROUP")) : 8;
    if (a.C == 4 || grp == 4) return launch_dw_bwd_plane_t<K, DIL, S, 4>(b, prebn, st);
    if (a.C == 8 || grp == 8) return launch_dw_bwd_plane_t<K, DIL, S, 8>(b, prebn, st);
    return launch_dw_bwd_plane_t<K, DIL, S, 16>(b, prebn, st);
  }
  const int TR = 64 / a.Wo;
  const int r = (K - 1) / 2 * DIL, h = (r + S - 1) / S, OR = TR + 2 * h;
  const int IR = (TR - 1) * S + (K - 1) * DIL + 1;
  const int IW = (a.Wo - 1) * S + (K - 1) * DIL + 1;
  size_t lds = sizeof(float) * (a.chunk * OR * a.Wo + a.chunk * IR * IW + 4 * a.C + (a.gW ? a.C * K * K : 0));
  dim3 grid(per_edge_blocks(a.N * (a.Ho / TR), b.n), b.n);
  if (prebn) hipLaunchKernelGGL((dw_bwd_kernel<K, DIL, S, true>), grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL((dw_bwd_kernel<K, DIL, S, false>), grid, dim3(256), lds, st, b);
}

bool launch_dw_bwd_multi(DwBwdBatch b, hipStream_t st) {
  if (b.n < 1) return true;
  const DwBwdArgs& a0 = b.e[0];
  if (!(a0.C == 4 || a0.C == 8 || (a0.C % 16 == 0 && a0.C <= kMaxC)) || !aligned16(b)) return false;
  static const int grp = getenv("KATIB_HIP_DWB_GROUP") ? atoi(getenv("KATIB_HIP_DWB_GROUP")) : 8;
  const int C = (a0.C == 4 || grp == 4) ? 4 : 8;  // wide layers: 8-channel groups (launch_dw_bwd_t)
  if (a0.C % C) return false;
  int maxblk = 0;
  size_t lds = 0;
  for (int i = 0; i < b.n; ++i) {
    DwBwdArgs& a = b.e[i];
    const int K = dw_variant_k(a.variant), DIL = dw_variant_dil(a.variant), S = dw_variant_s(a.variant);
    const bool prebn = dw_variant_prebn(a.variant);
    // the plane kernel's layout (dw_plane_ok) and an overwriting (never accumulating) input BN-free entry
    if (a.C != a0.C || a.H != a.Ho * S || a.W != a.Wo * S || a.pad != (K - 1) / 2 * DIL || a.Wo % 4 ||
        (prebn && (DIL != 1 || S != 1)) || (!prebn && !a.overwrite))
      return false;
    int nb = 1;
    const int G = a.C / C;
    while (nb < 8 && a.H % (2 * nb) == 0 &&
           (dw_plane_floats(a, K, DIL, S, nb, false, C) * 4 > 40 * 1024 || a.N * nb * G * b.n < 1024))
      nb *= 2;
    a.nbands = nb;
    a.nblk = a.N * nb * G;
    a.vin = (vec_mask() >> (C == 4 ? 2 : 3)) & 1;
    maxblk = std::max(maxblk, a.nblk);
    lds = std::max(lds, sizeof(float) * dw_plane_floats(a, K, DIL, S, nb, false, C));
  }
  if (C == 4) hipLaunchKernelGGL(dw_bwd_plane_multi_kernel<4>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  else hipLaunchKernelGGL(dw_bwd_plane_multi_kernel<8>, dim3(maxblk, b.n), dim3(256), lds, st, b);
  return true;
}

void launch_dw_bwd(const DwBwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st) {
#define DISPATCH(KK, DD, SS) \
  if (K == KK && dil == DD && S == SS) return launch_dw_bwd_t<KK, DD, SS>(b, prebn, st);
  DISPATCH(3, 1, 1) DISPATCH(3, 1, 2) DISPATCH(5, 1, 1) DISPATCH(5, 1, 2)
  DISPATCH(3, 2, 1) DISPATCH(3, 2, 2) DISPATCH(5, 2, 1) DISPATCH(5, 2, 2)
#undef DISPATCH
}

template <int CI, int CO>
static bool try_pw_fwd_wave(const PwFwdBatch& b, hipStream_t st) {
  const PwFwdArgs& a = b.e[0];
  constexpr int BO = CO / 16;
  if (a.Cin != CI || a.Cout != CO || (a.Ho * a.Wo) % 64 != 0 || getenv("KATIB_HIP_PW_FWD_TILED")) return false;
  for (int e = 0; e < b.n; ++e) {  // 16-byte loads (flat input) and stores
    const PwFwdArgs& x = b.e[e];
    const bool flat = !x.relu || (x.S == 1 && x.off == 0 && x.H == x.Ho && x.W == x.Wo);
    if ((((uintptr_t)x.z) | (flat ? (uintptr_t)x.x : 0)) & 15) return false;
  }
  const int chunks = a.N * a.Ho * a.Wo / 64;
  // split the output channels over waves while the launch has fewer than ~4 waves per SIMD
  int ns = 1;
  while (BO % (2 * ns) == 0 && chunks * ns * b.n < 4096) ns *= 2;
  const int per_edge = std::max(1, std::min((chunks * ns + 3) / 4, max_blocks() / std::max(b.n, 1)));
  const dim3 grid(per_edge, b.n);
  if (ns == 1) hipLaunchKernelGGL((pw_fwd_wave_kernel<CI, CO, 1>), grid, dim3(256), 0, st, b);
  else if constexpr (BO % 2 == 0) {
    if (ns == 2) hipLaunchKernelGGL((pw_fwd_wave_kernel<CI, CO, 2>), grid, dim3(256), 0, st, b);
    else if constexpr (BO % 4 == 0) hipLaunchKernelGGL((pw_fwd_wave_kernel<CI, CO, 4>), grid, dim3(256), 0, st, b);
  }
  return true;
}

void launch_pw_fwd(const PwFwdBatch& b, hipStream_t st) {
  const PwFwdArgs& a = b.e[0];
  if (try_pw_fwd_wave<48, 16>(b, st) || try_pw_fwd_wave<48, 32>(b, st) || try_pw_fwd_wave<64, 32>(b, st) ||
      try_pw_fwd_wave<32, 16>(b, st) || try_pw_fwd_wave<16, 16>(b, st) || try_pw_fwd_wave<32, 32>(b, st) ||
      try_pw_fwd_wave<64, 64>(b, st) || try_pw_fwd_wave<128, 64>(b, st))  // 128 -> 64: last-cell preprocess
    return;
  size_t lds = sizeof(float) * (a.Cin * 64 + 2 * a.Cout);
  dim3 grid(per_edge_blocks(a.N * a.Ho * a.Wo / 64, b.n), b.n);
  hipLaunchKernelGGL(pw_fwd_kernel, grid, dim3(256), lds, st, b);
}

static int channel_groups(int N, int C, int n) { return std::max(1, std::min(N, max_blocks() / (C * std::max(n, 1)))); }

void launch_pool_fwd(const PoolFwdBatch& b, int S, hipStream_t st) {
  const PoolFwdArgs& a = b.e[0];
  dim3 grid(a.C * channel_groups(a.N, a.C, b.n), b.n);
  if (S == 1) hipLaunchKernelGGL(pool_fwd_kernel<1>, grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL(pool_fwd_kernel<2>, grid, dim3(256), 0, st, b);
}

void launch_pool_bwd(const PoolBwdBatch& b, int S, hipStream_t st) {
  const PoolBwdArgs& a = b.e[0];
  size_t lds = sizeof(float) * 2 * a.Ho * a.Wo + a.Ho * a.Wo + 16;
  dim3 grid(a.N * a.C, b.n);
  if (S == 1) hipLaunchKernelGGL(pool_bwd_kernel<1>, grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL(pool_bwd_kernel<2>, grid, dim3(256), lds, st, b);
}

void launch_combine_fwd(const CombineFwdBatch& b, hipStream_t st) {
  const CombineFwdArgs& a = b.e[0];
  size_t total = (size_t)a.N * a.C * a.HW;
  auto al16 = [](const void* p) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  bool v4 = a.HW % 4 == 0 && al16(a.out);
  for (int e = 0; e < b.n && v4; ++e) {
    v4 = al16(b.e[e].xid);
    for (int k = 0; k < b.e[e].nops && v4; ++k) v4 = al16(b.e[e].z[k]);
  }
  int blocks = (int)std::min<size_t>(((v4 ? total / 4 : total) + 255) / 256, (size_t)max_blocks());
  size_t lds = sizeof(float) * (2 * b.n * kMaxOps * a.C + b.n * (kMaxOps + 1));
  if (v4) hipLaunchKernelGGL(combine_fwd_kernel<true>, dim3(blocks), dim3(256), lds, st, b);
  else hipLaunchKernelGGL(combine_fwd_kernel<false>, dim3(blocks), dim3(256), lds, st, b);
}

void launch_combine_bwd_reduce(const CombineBwdBatch& b, hipStream_t st) {
  const CombineBwdArgs& a = b.e[0];
  bool v4 = a.HW % 4 == 0;
  for (int e = 0; e < b.n; ++e) {
    const CombineBwdArgs& x = b.e[e];
    uintptr_t bits = (uintptr_t)x.dout | (uintptr_t)x.xid;
    for (int k = 0; k < x.nops; ++k) bits |= (uintptr_t)x.z[k];
    v4 &= (bits & 15) == 0;
  }
  const dim3 grid(a.C * channel_groups(a.N, a.C, b.n), b.n);
  if (v4) hipLaunchKernelGGL(combine_bwd_reduce_kernel<true>, grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL(combine_bwd_reduce_kernel<false>, grid, dim3(256), 0, st, b);
}

template <int CI, int CO>
static bool try_pw_bwd_px(const PwBwdBatch& b, hipStream_t st) {
  const PwBwdArgs& a = b.e[0];
  if (a.Cin != CI || a.Cout != CO) return false;
  const int total = a.N * a.Ho * a.Wo;
  // the 4-pixel vector path measured slower at C = 8 (register pressure: 21.7 vs 17.6 us) and
  // neutral at C = 4 on MI355X; it stays selectable for experiments (KATIB_HIP_PW_PX_V4=1)
  bool v4 = CI * CO <= 64 && (a.Ho * a.Wo) % 4 == 0 && getenv("KATIB_HIP_PW_PX_V4");
  for (int e = 0; e < b.n && v4; ++e) {
    const PwBwdArgs& x = b.e[e];
    const bool m1ok = x.mode == 0 || (x.S == 1 && x.off == 0 && x.H == x.Ho && x.W == x.Wo);
    const uintptr_t bits = (uintptr_t)x.gs.z | (uintptr_t)x.gs.g | (x.mode == 0 ? (uintptr_t)x.ain : (uintptr_t)x.x) |
                           (uintptr_t)(x.mode == 0 ? x.dd : x.gx);
    v4 = m1ok && (bits & 15) == 0 && x.co_off % 4 == 0;
  }
  const int per_edge = std::max(1, std::min(((v4 ? total / 4 : total) + 255) / 256, max_blocks() / std::max(b.n, 1)));
  if (v4) hipLaunchKernelGGL((pw_bwd_px_kernel<CI, CO, true>), dim3(per_edge, b.n), dim3(256), 0, st, b);
  else hipLaunchKernelGGL((pw_bwd_px_kernel<CI, CO, false>), dim3(per_edge, b.n), dim3(256), 0, st, b);
  return true;
}

template <int CI, int CO>
static bool try_pw_bwd_wave(const PwBwdBatch& b, hipStream_t st) {
  const PwBwdArgs& a = b.e[0];
  if (a.Cin != CI || a.Cout != CO || (a.Ho * a.Wo) % 64 != 0 || getenv("KATIB_HIP_PW_BWD_TILED")) return false;
  for (int e = 0; e < b.n; ++e) {  // 16-byte operand loads
    const PwBwdArgs& x = b.e[e];
    const bool flat = x.mode == 0 || (x.S == 1 && x.off == 0 && x.H == x.Ho && x.W == x.Wo);
    const uintptr_t bits = (uintptr_t)x.gs.z | (uintptr_t)x.gs.g | (flat ? (x.mode == 0 ? (uintptr_t)x.ain : (uintptr_t)x.x) : (uintptr_t)0);
    if (bits & 15) return false;
  }
  constexpr int BI = CI / 16;
  const int chunks = a.N * a.Ho * a.Wo / 64;
  // split the input channels over waves while the launch has fewer than ~4 waves per SIMD
  int ns = 1;
  while (BI % (2 * ns) == 0 && chunks * ns * b.n < 4096) ns *= 2;
  const int per_edge = std::max(1, std::min((chunks * ns + 3) / 4, max_blocks() / std::max(b.n, 1)));
  const size_t lds = sizeof(float) * 4 * CO * (64 + 4);
  const dim3 grid(per_edge, b.n);
  if (ns == 1) hipLaunchKernelGGL((pw_bwd_wave_kernel<CI, CO, 1>), grid, dim3(256), lds, st, b);
  else if constexpr (BI % 2 == 0) {
    if (ns == 2) hipLaunchKernelGGL((pw_bwd_wave_kernel<CI, CO, 2>), grid, dim3(256), lds, st, b);
    else if constexpr (BI % 4 == 0) hipLaunchKernelGGL((pw_bwd_wave_kernel<CI, CO, 4>), grid, dim3(256), lds, st, b);
  }
  return true;
}

void launch_pw_bwd(const PwBwdBatch& b, hipStream_t st) {
  const PwBwdArgs& a = b.e[0];
  // narrow layers: pixel-per-thread kernel (see pw_bwd_px_kernel)
  if (try_pw_bwd_px<4, 4>(b, st) || try_pw_bwd_px<8, 8>(b, st) || try_pw_bwd_px<4, 8>(b, st) ||
      try_pw_bwd_px<8, 4>(b, st) || try_pw_bwd_px<12, 8>(b, st) || try_pw_bwd_px<2, 2>(b, st) ||
      try_pw_bwd_px<4, 2>(b, st) || try_pw_bwd_px<2, 4>(b, st))
    return;
  // 16..64-channel layers: wave-per-chunk MFMA kernel (see pw_bwd_wave_kernel)
  if (try_pw_bwd_wave<16, 16>(b, st) || try_pw_bwd_wave<32, 32>(b, st) || try_pw_bwd_wave<64, 64>(b, st) ||
      try_pw_bwd_wave<48, 16>(b, st) || try_pw_bwd_wave<48, 32>(b, st) || try_pw_bwd_wave<64, 32>(b, st) ||
      try_pw_bwd_wave<32, 16>(b, st) || try_pw_bwd_wave<128, 64>(b, st))
    return;
  int ntiles = a.N * a.Ho * a.Wo / 64;
  dim3 grid(per_edge_blocks(ntiles, b.n), b.n);
  size_t lds = sizeof(float) * (a.Cout * 65 + a.Cin * 65 + 4 * a.Cout + 4);
  const int nblk = (a.Cin % 16 == 0 && a.Cout % 16 == 0) ? (a.Cin / 16) * (a.Cout / 16) : 1 << 30;
  if (nblk <= 16) hipLaunchKernelGGL((pw_bwd_kernel<true, 4>), grid, dim3(256), lds, st, b);
  else if (nblk <= 32) hipLaunchKernelGGL((pw_bwd_kernel<true, 8>), grid, dim3(256), lds, st, b);
  else hipLaunchKernelGGL((pw_bwd_kernel<false>), grid, dim3(256), lds, st, b);
}


__global__ void __launch_bounds__(256) fold_rows_kernel(FoldArgs a) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < a.n; i += gridDim.x * 256) {
    float acc = a.buf[i];
    for (int r = 1; r < a.rows; ++r) {
      float* q = a.buf + (size_t)r * a.n + i;
      acc += *q;
      *q = 0.f;
    }
    a.buf[i] = acc;
  }
}

// Replica fold for the f64 reductions (BN statistics, BN-backward sums, d alpha): run between a
// producer and its consumers so that every consumer reads ONE value per channel (rep = 1).
__global__ void __launch_bounds__(256) fold_f64_kernel(FoldF64Args a) {
  for (int g = blockIdx.x * 256 + threadIdx.x; g < a.total; g += gridDim.x * 256) {
    int seg = 0, i = g;
    while (seg < a.nseg - 1 && i >= a.n[seg]) i -= a.n[seg++];
    double* p = a.p[seg] + i;
    const int rs = a.rstride[seg];
    double v[kRep];
#pragma unroll
    for (int r = 0; r < kRep; ++r) v[r] = p[(size_t)r * rs];  // all loads in flight together
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < kRep; ++r) acc += v[r];
    p[0] = acc;
#pragma unroll
    for (int r = 1; r < kRep; ++r) p[(size_t)r * rs] = 0.0;
  }
}

void launch_fold_f64(const FoldF64Args& a, hipStream_t st) {
  int blocks = std::max(1, std::min((a.total + 255) / 256, 1024));
  hipLaunchKernelGGL(fold_f64_kernel, dim3(blocks), dim3(256), 0, st, a);
}

void launch_fold_rows(const FoldArgs& a, hipStream_t st) {
  int blocks = std::max(1, std::min((a.n + 255) / 256, 2048));
  hipLaunchKernelGGL(fold_rows_kernel, dim3(blocks), dim3(256), 0, st, a);
}

}  // namespace katib_hip
