// Internal: the DARTS forward kernel templates, included by darts_ops_fwd.hip (launchers, single-variant
// instantiations) and darts_ops_fwd_m{4,8,16}.hip (the mixed-variant multi / joint kernels of one channel
// count each, so the heaviest instantiations compile in parallel).
#pragma once
#include "darts_ops_dev.h"

namespace katib_hip {

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
  const int HP = (BR - 1) * S + (K - 1) * DIL + 1, WP = lds_pitch(W + 2 * pad), PL = HP * WP;
  const int iyb = oy0 * S - pad;  // input row of staged row 0
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sWt = smem;                            // [C][KK] depthwise weights (plane_head_floats)
  float* sPw = smem + C * 25;                   // [C][C] pointwise weights
  float* sIn = smem + plane_head_floats(C);     // [C][HP][WP]
  __shared__ float sMean[C], sInv[C], sStat[2 * C];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  KSTAMP(0);
  // depthwise and pointwise weights in LDS, loaded with the prologue: read from global memory in
  // the compute loops, each weight was a separate load + s_waitcnt vmcnt(0) (not hoistable above
  // the d / z stores, which could alias) - a serial chain of C (K^2 + C) round trips per thread
  for (int i = tid; i < C * KK; i += 256) sWt[i] = a.dw[c0 * KK + i];
  if (PW)
    for (int i = tid; i < C * C; i += 256) sPw[i] = a.pw[i];
  if (PREBN) bn_coeffs_coop(a.inbn, c0, C, sMean, sInv);  // the input BN may arrive unfolded (rep > 1)
  if (tid < C) {
    sStat[tid] = 0.f;
    sStat[C + tid] = 0.f;
  }
  // only the input-BN staging reads the prologue's LDS (sMean / sInv) before the staging barrier:
  // without an input BN the weight loads and the staging loads share one round trip
  if (PREBN) __syncthreads();
  KSTAMP(1);
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
  KSTAMP(2);
  float st1[C], st2[C];
#pragma unroll
  for (int c = 0; c < C; ++c) st1[c] = st2[c] = 0.f;
  const int HWo = Ho * Wo;
  zt* dn = a.d + ((size_t)n * a.C + c0) * HWo;
  zt* zn = a.z + (size_t)n * C * HWo;
  const bool vout = VEC && Wo % 4 == 0 && a.vout;
  if (vout) {
    // 4 consecutive output pixels (one row: Wo % 4 == 0) per thread: d and z leave as one 16-byte
    // (bf16: 8-byte) store per channel instead of four 4-byte ones. Each tap row the 4 outputs
    // reach (SPAN staged columns from ox0 * S, a multiple of 4) is read as NQ aligned 16-byte
    // quads (WP = lds_pitch: a multiple of 4 floats, wide enough for the last quad): 2-4
    // ds_read_b128 per row instead of 4 K ds_read_b32 whose lanes, 4 S floats apart, sat on 8 (S = 1)
    // or 4 (S = 2) of the 32 banks
    constexpr int SPAN = 3 * S + (K - 1) * DIL + 1, NQ = (SPAN + 3) / 4;
    for (int p = oy0 * Wo + 4 * tid; p < oy1 * Wo; p += 1024) {
      const int oy = p / Wo, ox0 = p - oy * Wo;
      zf4 d[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float* src = sIn + c * PL + ((oy - oy0) * S) * WP + ox0 * S;  // 16-byte aligned
        KEEP_WEIGHT_READS_LOCAL();
        const float* wk = sWt + c * KK;  // LDS broadcast reads
        zf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
          float v[4 * NQ];
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(src + ky * DIL * WP + 4 * q);
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
          }
#pragma unroll
          for (int kx = 0; kx < K; ++kx) {
            const float w = wk[ky * K + kx];
            acc.x += w * v[kx * DIL];
            acc.y += w * v[kx * DIL + S];
            acc.z += w * v[kx * DIL + 2 * S];
            acc.w += w * v[kx * DIL + 3 * S];
          }
        }
        d[c] = acc;
        zst4(dn + (size_t)c * HWo + p, acc);
      }
      if (!PW) continue;
#pragma unroll
      for (int co = 0; co < C; ++co) {
        KEEP_WEIGHT_READS_LOCAL();
        zf4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ci = 0; ci < C; ++ci) z += sPw[co * C + ci] * d[ci];
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
      KEEP_WEIGHT_READS_LOCAL();
        const float* wk = sWt + c * KK;  // LDS broadcast reads
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
      KEEP_WEIGHT_READS_LOCAL();
      float z = 0.f;
#pragma unroll
      for (int ci = 0; ci < C; ++ci) z += sPw[co * C + ci] * d[ci];
      zput(zn + (size_t)co * HWo + p, z);
      st1[co] += z;
      st2[co] += z * z;
    }
  }
  KSTAMP(3);
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
  KSTAMP(4);
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
static __global__ void __launch_bounds__(256) pw_fwd_kernel(PwFwdBatch bt) {
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
template <int S, bool V4 = false>
__device__ __forceinline__ void pool_fwd_body(const PoolFwdArgs& a, const int bx, const int gx) {
  const int C = a.C, H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
  const int c = bx % C, g0 = bx / C, G = gx / C;
  float sa = 0, sa2 = 0, sm = 0, sm2 = 0;
  if constexpr (V4) {
    // 4 consecutive outputs of one row per thread from a register window of the input rows they
    // touch, loaded straight from global memory (16-byte loads; stride 1: 3 x 6 inputs, stride 2:
    // 3 x 9), no LDS and no barrier: 9 load instructions per 4 outputs instead of 36. The taps are
    // visited in the scalar path's order (first maximal element in row-major order, NaN wins).
    // zavg / zmax leave as one 16-byte (bf16: 8-byte) store, the argmax taps as one 4-byte store
    // per 4 outputs (W, Wo % 4 == 0, every operand aligned: host-checked)
    constexpr int WC = S == 1 ? 6 : 9;  // window columns: ix0 - 1 .. ix0 + 4 (S 1) / ib - 1 .. ib + 7 (S 2)
    const int HWo = Ho * Wo;
    for (int n = g0; n < a.N; n += G) {
      const int nc = n * C + c;
      const float* xp = a.x + (size_t)nc * H * W;
      for (int o4 = threadIdx.x * 4; o4 < HWo; o4 += 1024) {
        const int oy = o4 / Wo, ox0 = o4 - oy * Wo, ib = ox0 * S;  // input column of window column 1
        float win[3][WC];
        bool rv[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int iy = oy * S - 1 + r;
          rv[r] = iy >= 0 && iy < H;
          const float* row = xp + (size_t)(rv[r] ? iy : 0) * W;
          const float4 m0 = *reinterpret_cast<const float4*>(row + ib);
          win[r][1] = m0.x;
          win[r][2] = m0.y;
          win[r][3] = m0.z;
          win[r][4] = m0.w;
          if (S == 1) {
            win[r][5] = ib + 4 < W ? row[ib + 4] : 0.f;
          } else {
            const float4 m1 = *reinterpret_cast<const float4*>(row + ib + 4);
            win[r][5] = m1.x;
            win[r][6] = m1.y;
            win[r][7] = m1.z;
            win[r][8] = m1.w;
          }
          win[r][0] = ib > 0 ? row[ib - 1] : 0.f;
        }
        const bool lv = ib > 0, hv = S == 2 || ib + 4 < W;  // window column 0 / WC - 1 inside the row
        zf4 av, mv;
        unsigned args = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float sum = 0.f, mx = -INFINITY;
          int cnt = 0, arg = 0;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky) {
            if (!rv[ky]) continue;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const int wc = t * S + kx;  // input column ib + t*S - 1 + kx
              if ((wc == 0 && !lv) || (wc == WC - 1 && !hv)) continue;
              const float v = win[ky][wc];
              sum += v;
              cnt++;
              if (v > mx || v != v) {  // first maximal element in row-major order (max_pool2d)
                mx = v;
                arg = ky * 3 + kx;
              }
            }
          }
          av[t] = sum / (float)cnt;
          mv[t] = mx;
          args |= (unsigned)arg << (8 * t);
        }
        const size_t oo = (size_t)nc * HWo + o4;
        zst4(a.zavg + oo, av);
        zst4(a.zmax + oo, mv);
        if (a.amax) *reinterpret_cast<unsigned*>(a.amax + oo) = args;
        sa += (av.x + av.y) + (av.z + av.w);
        sa2 += (av.x * av.x + av.y * av.y) + (av.z * av.z + av.w * av.w);
        sm += (mv.x + mv.y) + (mv.z + mv.w);
        sm2 += (mv.x * mv.x + mv.y * mv.y) + (mv.z * mv.z + mv.w * mv.w);
      }
    }
  }
  for (int n = V4 ? a.N : g0; n < a.N; n += G) {
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
template <bool V4>
__global__ void __launch_bounds__(256) pool_fwd_multi_kernel(PoolFwdBatch bt) {
  const PoolFwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
  if ((int)blockIdx.x < a.nblk) {
    if (a.S == 1) pool_fwd_body<1, V4>(a, blockIdx.x, a.nblk);
    else pool_fwd_body<2, V4>(a, blockIdx.x, a.nblk);
  }
  if (bt.tail.ctr) fold_tail(bt.tail);
}


// A node's stage-1 depthwise-pointwise entries and its pools in ONE launch (both read only the
// node's inputs): blockIdx.y < bt.n runs a dw-pw entry, the rest a pool entry, so the pool
// workgroups fill the chip beside the dw-pw bands instead of running as a launch of their own
// after them (fused narrow layers, no self-fold tails).
template <int C, bool PV4>
__global__ void __launch_bounds__(256) dwpw_pool_multi_kernel(DwPwMultiBatch bt, PoolFwdEntries pe) {
  constexpr bool PW = true;
  const int bx = blockIdx.x;
  if ((int)blockIdx.y < bt.n) {
    const DwPwFwdArgs a = bt.e[blockIdx.y];  // copy: see dwpw_plane_multi_kernel
    if (bx < a.nblk) {
      switch (a.variant) {
        DWPW_CASE(3, 1, 1) DWPW_CASE(3, 1, 2) DWPW_CASE(5, 1, 1) DWPW_CASE(5, 1, 2)
        DWPW_CASE(3, 2, 1) DWPW_CASE(3, 2, 2) DWPW_CASE(5, 2, 1) DWPW_CASE(5, 2, 2)
        default: break;
      }
    }
  } else {
    const PoolFwdArgs a = pe.e[blockIdx.y - bt.n];
    if (bx < a.nblk) {
      if (a.S == 1) pool_fwd_body<1, PV4>(a, bx, a.nblk);
      else pool_fwd_body<2, PV4>(a, bx, a.nblk);
    }
  }
}
#undef DWPW_CASE


// per-channel-count launchers of the mixed-variant kernels (explicitly instantiated in darts_ops_fwd_m<C>.hip)
template <int C>
void launch_dwpw_plane_multi_t(bool pw, dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b);
template <int C>
void launch_dwpw_pool_t(dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b, const PoolFwdEntries& pe);
template <>
void launch_dwpw_plane_multi_t<4>(bool pw, dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b);
template <>
void launch_dwpw_plane_multi_t<8>(bool pw, dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b);
template <>
void launch_dwpw_plane_multi_t<16>(bool pw, dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b);
template <>
void launch_dwpw_pool_t<4>(dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b, const PoolFwdEntries& pe);
template <>
void launch_dwpw_pool_t<8>(dim3 grid, size_t lds, hipStream_t st, const DwPwMultiBatch& b, const PoolFwdEntries& pe);

}  // namespace katib_hip
