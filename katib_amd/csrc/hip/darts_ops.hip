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
#include "darts_ops_dev.h"

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

// 4-pixels-per-thread output paths of the plane kernels, per channel group: bit 0 dwpw_plane C = 4, bit 1 dwpw_plane C = 8, bit 2 dw_bwd_plane C = 4, bit 3
// dw_bwd_plane C = 8 (stride 1), bit 4 dw_bwd_plane stride-2 parity classes (any C). Default C = 4
// only: at C = 8 the four-pixel register arrays cost more than the wider stores save, and the
// stride-2 classes (a quarter of the multiply-adds) measured slower, B5 6.98 vs 6.80 ms
// (profiles/darts_vec_ab_r04.log).
int vec_mask() { return 0x5; }

// phase-stamp arming (diagnostic build): the `call`-th launch of `kind` after stamps_arm()
static int g_stamp_kind = 0, g_stamp_call = -1, g_stamp_seen = 0;
static unsigned long long* g_stamp_buf = nullptr;
void stamps_arm(int kind, int call, unsigned long long* buf) {
  g_stamp_kind = kind;
  g_stamp_call = call;
  g_stamp_seen = 0;
  g_stamp_buf = buf;
}
bool stamp_take(int kind) {
  if (kind != g_stamp_kind || g_stamp_buf == nullptr) return false;
  return g_stamp_seen++ == g_stamp_call;
}
unsigned long long* stamp_buffer() { return g_stamp_buf; }
bool stamps_compiled() {
#ifdef KATIB_HIP_STAMPS
  return true;
#else
  return false;
#endif
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
  // V4: the statistic loads go out first, then the first element's operands (which do not depend
  // on them), then the coefficient math: the two memory round trips of a block overlap
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int EM = CombineFwdBatch::kCap;
  const size_t total4 = total / 4;
  f4 zv[EM][kMaxOps], xv[EM];
  auto load4 = [&](size_t i4) {
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      const CombineFwdArgs& a = bt.e[e < ne ? e : 0];
#pragma unroll
      for (int k = 0; k < kMaxOps; ++k)
        if (e < ne && k < a.nops) zv[e][k] = zld4(a.z[k] + 4 * i4);
      if (e < ne && a.xid) xv[e] = reinterpret_cast<const f4*>(a.xid)[i4];
    }
  };
  size_t i4 = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int NE = ne * kMaxOps * C;
  const bool coop = ne == 1 && a0.nops == 1 && !a0.bn[0].eval && a0.bn[0].rep > 1;
  const bool split = !coop && NE <= 256;  // one (edge, op, channel) coefficient per thread
  BnRaw raw{0.0, 0.0, 0.f, 1.f};
  bool has_raw = false;
  if (split && (int)threadIdx.x < NE) {
    const int i = threadIdx.x, e = i / (kMaxOps * C), k = (i / C) % kMaxOps, c = i % C;
    const CombineFwdArgs& a = bt.e[e];
    if (k < a.nops) {
      raw = bn_raw(a.bn[k], c);
      has_raw = true;
    }
  }
  // the softmax weights of every (edge, op) and identity, issued with the statistics
  float wv = 0.f;
  if ((int)threadIdx.x < ne * (kMaxOps + 1)) {
    const int e = threadIdx.x / (kMaxOps + 1), k = threadIdx.x % (kMaxOps + 1);
    const CombineFwdArgs& a = bt.e[e];
    if (k < a.nops) wv = a.w ? a.w[a.widx[k]] : 1.f;
    else if (k == kMaxOps) wv = (a.w && a.id_idx >= 0) ? a.w[a.id_idx] : 0.f;
  }
  if (V4 && i4 < total4) load4(i4);
  // every (edge, op, channel) coefficient in one pass: one round of statistic loads per block
  if (split) {
    if (has_raw) {
      const int i = threadIdx.x, e = i / (kMaxOps * C), k = (i / C) % kMaxOps;
      bn_finish(bt.e[e].bn[k], raw, sMean[i], sInv[i]);
    }
  } else if (coop) {
    // a preprocess BN whose statistics arrive unfolded (their fold joins the cell's first node's)
    bn_coeffs_coop(a0.bn[0], 0, C, sMean, sInv);
  } else {
    for (int i = threadIdx.x; i < ne * kMaxOps * C; i += 256) {
      const int e = i / (kMaxOps * C), k = (i / C) % kMaxOps, c = i % C;
      const CombineFwdArgs& a = bt.e[e];
      if (k < a.nops) bn_coeffs(a.bn[k], c, sMean[i], sInv[i]);
    }
  }
  if ((int)threadIdx.x < ne * (kMaxOps + 1)) sW[threadIdx.x] = wv;  // ne * (kMaxOps + 1) <= 36 < 256
  __syncthreads();
  // running-statistic updates spread over the grid's threads (one (edge, op, channel) each), not
  // looped by block 0: its fp64 moments then delayed that one block's elementwise work - the tail
  // of every launch
  {
    int base = 0;
    const int gt = blockIdx.x * 256 + threadIdx.x;
    for (int e = 0; e < ne; ++e) {
      const CombineFwdArgs& a = bt.e[e];
      if (!a.update_running) continue;
      const int n_e = (a.nops + a.nupd) * C, S = gridDim.x * 256;
      int i0 = (gt - base) % S;  // global entry base + i goes to thread (base + i) mod S
      if (i0 < 0) i0 += S;
      for (int i = i0; i < n_e; i += S) {
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
      base += n_e;
    }
  }
  if (V4) {
    // 4 consecutive elements per thread (HW % 4 == 0: one channel), 16-byte loads/stores;
    // the host picks this path only when every operand pointer is 16-byte aligned
    // every operand load of an element is issued first (up to EM * (kMaxOps + 1) in flight), then
    // accumulated in the scalar path's order: a runtime-bounded load-then-add loop waited on each
    // load in turn. The first element's loads went out before the prologue.
    for (bool first = true; i4 < total4; i4 += (size_t)gridDim.x * 256, first = false) {
      const int c = (int)((i4 * 4 / HW) % C);
      if (!first) load4(i4);
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
  // half the persistent-grid budget: two images per workgroup at B5 sizes, so each thread keeps two
  // elements' operands in flight and the coefficient prologue / reduction tail are paid half as often
  const dim3 grid(a.C * channel_groups(a.N, a.C, 2 * b.n), b.n);
  if (v4) hipLaunchKernelGGL(combine_bwd_reduce_kernel<true>, grid, dim3(256), 0, st, b);
  else hipLaunchKernelGGL(combine_bwd_reduce_kernel<false>, grid, dim3(256), 0, st, b);
}

__global__ void __launch_bounds__(256) fold_rows_kernel(FoldArgs a) {
  // every replica loaded before any is zeroed (16 in flight per step): interleaving each row's
  // load with its zeroing store kept the compiler from hoisting the next load past the store to
  // the same buffer - one memory round trip per replica (14 us per launch at REP = 32). The sum
  // keeps the row order, so the result is bit-identical.
  for (int i = blockIdx.x * 256 + threadIdx.x; i < a.n; i += gridDim.x * 256) {
    float acc = 0.f;
    for (int r0 = 0; r0 < a.rows; r0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = r0 + u < a.rows ? a.buf[(size_t)(r0 + u) * a.n + i] : 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (r0 + u < a.rows) acc = (r0 + u == 0) ? v[u] : acc + v[u];
    }
    for (int r = 1; r < a.rows; ++r) a.buf[(size_t)r * a.n + i] = 0.f;
    a.buf[i] = acc;
  }
}

// Replica fold for the f64 reductions (BN statistics, BN-backward sums, d alpha): run between a
// producer and its consumers so that every consumer reads ONE value per channel (rep = 1).
__global__ void __launch_bounds__(256) fold_f64_kernel(FoldF64Args a) {
  // one grid row per segment: its pointer / length / stride are wave-uniform kernarg reads. A flat
  // element index walked the segment table per thread (a dependent, divergent load per segment
  // passed) before its first replica load could issue
  const int seg = blockIdx.y;
  const int n = a.n[seg], rs = a.rstride[seg];
  double* base = a.p[seg];
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    double* p = base + i;
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
  if (a.nseg < 1) return;
  int maxn = 1;
  for (int s = 0; s < a.nseg; ++s) maxn = std::max(maxn, a.n[s]);
  const int bx = std::max(1, std::min((maxn + 255) / 256, std::max(1, 1024 / a.nseg)));
  hipLaunchKernelGGL(fold_f64_kernel, dim3(bx, a.nseg), dim3(256), 0, st, a);
}

void launch_fold_rows(const FoldArgs& a, hipStream_t st) {
  int blocks = std::max(1, std::min((a.n + 255) / 256, 2048));
  hipLaunchKernelGGL(fold_rows_kernel, dim3(blocks), dim3(256), 0, st, a);
}

}  // namespace katib_hip
