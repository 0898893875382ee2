// Internal: device helpers and host launch heuristics shared by the DARTS kernel translation
// units (darts_ops.hip core + combine + folds, darts_ops_fwd.hip, darts_ops_pwb.hip,
// darts_ops_dwb.hip). Split so the four compile in parallel; not a public header.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "darts_ops.h"

namespace katib_hip {

int max_blocks();

// Diagnostic build only (-DKATIB_HIP_STAMPS, _build.build_hip_stamps): phase timestamps of every
// workgroup of ONE armed launch (s_memrealtime, 100 MHz, device-wide clock), written by lane 0 of
// the workgroup to stamps[wg * 8 + phase] (a vector store). The per-TU device pointer is set by
// the host launcher right before the armed launch and cleared after it; the production build
// compiles every KSTAMP to nothing.
#ifdef KATIB_HIP_STAMPS
static __device__ unsigned long long* g_stamps = nullptr;
#define KSTAMP(k)                                                                          \
  do {                                                                                     \
    unsigned long long* _sp = g_stamps;                                                    \
    if (_sp != nullptr && threadIdx.x == 0) {                                              \
      const unsigned _wg = blockIdx.y * gridDim.x + blockIdx.x;                            \
      if (_wg < 65536u) _sp[(size_t)_wg * 8 + (k)] = __builtin_amdgcn_s_memrealtime();     \
    }                                                                                      \
  } while (0)
bool stamp_take(int kind);  // host: is this launch of `kind` the armed one (darts_ops.hip)
unsigned long long* stamp_buffer();
#define KSTAMP_ARM(kind, st)                                                               \
  const bool _stamp_armed = stamp_take(kind);                                              \
  if (_stamp_armed) {                                                                      \
    static unsigned long long* _on;                                                        \
    _on = stamp_buffer();                                                                  \
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stamps), &_on, sizeof(_on), 0, hipMemcpyHostToDevice, st); \
  }
#define KSTAMP_DISARM(st)                                                                  \
  if (_stamp_armed) {                                                                      \
    static unsigned long long* _off = nullptr;                                             \
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stamps), &_off, sizeof(_off), 0, hipMemcpyHostToDevice, st); \
  }
#else
#define KSTAMP(k)
#define KSTAMP_ARM(kind, st)
#define KSTAMP_DISARM(st)
#endif
enum StampKind { kStampDwBwd = 1, kStampDwPw = 2, kStampPoolBwd = 3, kStampPoolFwd = 4, kStampCombineFwd = 5,
                 kStampCombineBwd = 6, kStampPwBwd = 7 };
// Compiler fence at the top of a per-channel loop body that reads LDS-resident weights: keeps
// those reads inside the iteration. Without it hipcc hoists every weight of every channel out of
// the pixel loop into registers (C * K^2 live values: 256 VGPRs + AGPRs, one wave per SIMD).
#define KEEP_WEIGHT_READS_LOCAL() asm volatile("" ::: "memory")
// Dynamic-LDS head of the plane kernels (floats, a multiple of 4): the group's depthwise weights
// (up to 5x5 taps) and pointwise weights (dwpw) / depthwise weight-gradient sums (dw_bwd). In the
// dynamic region, one allocation serves every variant body of a mixed-variant kernel; as static
// __shared__ arrays each of the 10-32 inlined variants held its own copy, and the extra static
// LDS cost a workgroup per CU.
__host__ __device__ constexpr int plane_head_floats(int C) { return (C * 25 + C * C + 3) & ~3; }
__host__ __device__ constexpr int dwb_head_floats(int C) { return (2 * C * 25 + 3) & ~3; }
// Row pitch (floats) of the LDS planes the plane kernels stage (dwpw_plane, dw_bwd_plane): a
// multiple of 4 floats, so the 4-pixel paths read every tap row as whole 16-byte ds_read_b128
// quads from an aligned base (a lane's 4 outputs at stride 4 floats hit 8 of 32 banks as
// 4-byte reads: 4-way conflicts), and an odd number of quads, so the lanes of one b128 lane
// group that sit on consecutive rows start on different 16-byte bank slots.
__host__ __device__ constexpr int lds_pitch(int w) {
  return (((w + 3) & ~3) >> 2) & 1 ? ((w + 3) & ~3) : ((w + 3) & ~3) + 4;
}
// 4-pixels-per-thread output paths of the plane kernels (darts_ops.hip vec_mask())
int vec_mask();

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

// Split form of bn_coeffs for prologues that overlap the statistic loads with operand loads:
// bn_raw issues the loads (a folded or eval BN: two loads; unfolded: the replica walk), bn_finish
// turns them into (mean, 1 / std) after the caller has issued its other loads - s_waitcnt vmcnt is
// in order, so loads issued AFTER the statistic loads do not delay them.
struct BnRaw {
  double s, s2;
  float rm, rv;
};
__device__ __forceinline__ BnRaw bn_raw(const BNRef& b, int c) {
  BnRaw r{0.0, 0.0, 0.f, 1.f};
  if (b.eval) {
    r.rm = b.rmean[c];
    r.rv = b.rvar[c];
  } else if (b.rep == 1) {
    r.s = b.sums[c];
    r.s2 = b.sums[b.C + c];
  } else {
    sum_replicas(b.sums + c, b.rep, b.rstride, b.C, r.s, r.s2);
  }
  return r;
}
__device__ __forceinline__ void bn_finish(const BNRef& b, const BnRaw& r, float& mean, float& invstd) {
  if (b.eval) {
    mean = r.rm;
    invstd = rsqrtf(r.rv + b.eps);
  } else {  // as bn_moments / bn_coeffs
    const double m = r.s * (double)b.inv_count;
    double v = r.s2 * (double)b.inv_count - m * m;
    if (v < 0) v = 0;
    mean = (float)m;
    invstd = rsqrtf((float)v + b.eps);
  }
}

// A backward kernel's BN coefficients (mean, 1 / std) AND BN-backward means (m1, m2) of channels
// [c0, c0 + n) in ONE memory round trip: 16-lane groups, the first n on the statistics, the next n
// on the BN-backward sums, each folded (rep 1) or not (kRep replicas: a few loads per lane). The
// per-channel bn_coeffs threads followed by a cooperative gs_means_coop were two dependent trips
// (plus kRep / 8 more when the statistics arrived unfolded). Every thread calls; the caller
// barriers before reading. Needs 32 n <= blockDim.x (falls back to the two-step form otherwise).
__device__ __forceinline__ void bn_gs_coop(const GradSrc& gs, int c0, int n, float* mean, float* inv, float* m1,
                                           float* m2) {
  const BNRef& b = gs.bn;
  if (32 * n > (int)blockDim.x) {
    for (int c = threadIdx.x; c < n; c += blockDim.x) bn_coeffs(b, c0 + c, mean[c], inv[c]);
    gs_means_coop(gs, c0, n, m1, m2);
    return;
  }
  const int grp = threadIdx.x >> 4, j = threadIdx.x & 15;
  const bool stats = grp < n, act = grp < 2 * n;
  const int ch = c0 + (stats ? grp : grp - n);
  double s = 0.0, s2 = 0.0;
  if (act && stats && !b.eval) {
    for (int r = j; r < b.rep; r += 16) {
      s += b.sums[(size_t)r * b.rstride + ch];
      s2 += b.sums[(size_t)r * b.rstride + b.C + ch];
    }
  } else if (act && !stats && !gs.eval) {
    const int rs = gs.rep == 1 ? 0 : gs.rstride;
    const size_t off2 = gs.S2 - gs.S1;
    for (int r = j; r < gs.rep; r += 16) {
      s += gs.S1[(size_t)r * rs + ch];
      s2 += gs.S1[(size_t)r * rs + off2 + ch];
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if (act && j == 0) {
    const int k = ch - c0;
    if (stats) {
      if (b.eval) {
        mean[k] = b.rmean[ch];
        inv[k] = rsqrtf(b.rvar[ch] + b.eps);
      } else {  // as bn_moments / bn_coeffs
        const double m = s * (double)b.inv_count;
        double v = s2 * (double)b.inv_count - m * m;
        if (v < 0) v = 0;
        mean[k] = (float)m;
        inv[k] = rsqrtf((float)v + b.eps);
      }
    } else {  // as gs_means
      m1[k] = gs.eval ? 0.f : (float)(s * (double)b.inv_count);
      m2[k] = gs.eval ? 0.f : (float)(s2 * (double)b.inv_count);
    }
  }
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

// wave sums of M accumulators (any M) added into dst[0 .. M): power-of-two chunks of at most 64
// through the reduce-scatter (a 96-entry weight-gradient tile is 64 + 32, not 96 separate
// 6-step wave sums)
template <int M>
__device__ __forceinline__ void wave_sums_to_lds(float* acc, float* dst, int lane) {
  if constexpr (M > 0) {
    constexpr int P = M >= 64 ? 64 : (M >= 32 ? 32 : (M >= 16 ? 16 : (M >= 8 ? 8 : (M >= 4 ? 4 : (M >= 2 ? 2 : 1)))));
    const float s = wave_reduce_scatter<P>(acc);
    if ((lane & (64 / P - 1)) == 0) atomicAdd(dst + wave_scatter_index<P>(lane), s);
    wave_sums_to_lds<M - P>(acc + P, dst + P, lane);
  }
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

// on-the-fly BN backward: dz = wk * invstd * (g - S1/cnt - zhat * S2/cnt)
__device__ __forceinline__ float bn_bwd_val(const GradSrc& gs, size_t i, float mean, float inv, float wk, float m1,
                                           float m2) {
  float zh = (z2f(gs.z[i]) - mean) * inv;
  float g = gs.g[i];
  return wk * inv * (g - m1 - zh * m2);  // eval: m1 = m2 = 0
}

// orders a wave's LDS writes before its later LDS reads of other lanes' data (LDS executes one
// wave's instructions in order, so only the compiler has to be kept from reordering them)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

static inline int per_edge_blocks(int tiles, int n) { return std::max(1, std::min(tiles, max_blocks() / std::max(n, 1))); }
static inline int channel_groups(int N, int C, int n) { return std::max(1, std::min(N, max_blocks() / (C * std::max(n, 1)))); }

}  // namespace katib_hip
