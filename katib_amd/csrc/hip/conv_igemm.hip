// Implicit-GEMM convolutions for gfx950: bf16 operands, fp32 accumulation on
// v_mfma_f32_16x16x32_bf16, NHWC activations, [K][R][S][C] filters.
//
// The CIFAR ResNet-18 trial (BASELINE config 3) spends >90 % of its time in MIOpen's
// naive fallback kernels for several bf16 NHWC shapes on this stack (profiles/
// resnet18_*), and the ENAS child networks need the same k x k / stride / dilation
// family (reference op_library.py:22-155). Three kernels cover training:
//
//  fwd   y[m][k]  = sum_(r,s,c) x[pix(m,r,s)][c] * w[k][r][s][c]     M = N*OH*OW, N = K
//  dgrad dx[m][c] = sum_(r,s,k) dy[pix'(m,r,s)][k] * wt[c][r][s][k]   M = N*H*W,   N = C
//  wgrad dw[k][(r,s,c)] = sum_p dy[p][k] * x[pix(p,r,s)][c]          split over p, fp32 atomics
//
// fwd/dgrad: both operands are reduction-contiguous (16-byte chunks of 8 channels), so
// every thread gathers fixed rows x fixed 8-channel chunk per stage straight into
// registers (zero for padding / stride holes), writes them to a double-buffered LDS
// image with 16-B padded rows (conflict-free ds_read_b128 fragment reads) and the
// 4 waves (2 x 2) run 2 MFMA k-steps per 64-deep stage. Block -> tile order is XCD
// aware: the tiles that share an im2col row block sit on one XCD (one L2).
// Strided dgrad (MODE 2): with stride s only the taps r = (ih + ph) mod s (+ s, ...) reach an
// input row, so 3/4 of a 3x3 / stride-2 reduction would multiply zeros. The input pixels are
// split into s_h x s_w phase classes (blockIdx.y); each class is its own implicit GEMM over just
// its taps (1x1, 1x2, 2x1 or 2x2 of the 3x3 filter), reading the [C][R][S][K] filter rows at
// those taps only.
// wgrad: the reduction runs over pixels, which are strided in both operands, so the
// LDS images stay in natural [pixel][channel] layout and the MFMA fragments are read
// with the gfx950 transposing ds_read_b64_tr_b16.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdlib>

#include "conv_igemm.h"

namespace katib_hip {
namespace conv {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native vector: HIP's uint4 class (unions) defeats SROA -> scratch
typedef __hip_bfloat16 bf16;

constexpr int kBK = 64;       // reduction depth per LDS stage
constexpr int kPad = 8;       // bf16 row padding (16 B)
constexpr int kThreads = 256;  // 4 waves as 2 x 2

// Division by a runtime divisor d as a multiply-high (Granlund-Montgomery round-up form):
// n / d = (umulhi(n, m) + n) >> s, exact for n < 2^31 (host-side make_fastdiv). The wgrad gather
// decomposes every staged pixel index into (image, row, column): two integer divisions per
// 16-byte load were ~70 VALU instructions each (profiles/conv_wgrad_r06.log).
struct FastDiv {
  unsigned m, s;
};
FastDiv make_fastdiv(unsigned d) {
  unsigned s = 0;
  while ((1ull << s) < d) ++s;
  const unsigned long long m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FastDiv{(unsigned)m, s};
}
__device__ __forceinline__ unsigned fdiv(unsigned n, FastDiv f) { return (__umulhi(n, f.m) + n) >> f.s; }

__device__ inline int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ---------------------------------------------------------------- fwd / dgrad
template <int MODE, int BM, int BN>
__global__ __launch_bounds__(kThreads) void igemm_kernel(ConvGeom g, const bf16* __restrict__ src,
                                                         const bf16* __restrict__ wmat, bf16* __restrict__ y,
                                                         float* __restrict__ y32, int M, int N, int Kd,
                                                         const bf16* __restrict__ add_d,
                                                         const bf16* __restrict__ add_y) {
  constexpr int WM = BM / 2, WN = BN / 2, RM = WM / 16, RN = WN / 16;
  constexpr int LD = kBK + kPad;
  constexpr int AR = BM / 32, BR = BN / 32;  // rows per thread per stage
  __shared__ __align__(16) bf16 smem[2 * (BM + BN) * LD];
  bf16* As = smem;
  bf16* Bs = smem + 2 * BM * LD;

  const int tilesN = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / tilesN) * BM, n0 = (wg % tilesN) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int kc = tid & 7, trow = tid >> 3;
  // MODE 2: this workgroup's phase class (py, px), its pixel grid Hc x Wc and its taps
  int py = 0, px = 0, Hc = 1, Wc = 1, r0 = 0, s0 = 0, Ss = 1;
  if (MODE == 2) {
    py = blockIdx.y / g.sw;
    px = blockIdx.y - py * g.sw;
    Hc = (g.H - py + g.sh - 1) / g.sh;
    Wc = (g.W - px + g.sw - 1) / g.sw;
    M = g.N * Hc * Wc;
    r0 = (py + g.ph) % g.sh;
    s0 = (px + g.pw) % g.sw;
    const int Rr = r0 < g.R ? (g.R - r0 + g.sh - 1) / g.sh : 0;
    Ss = s0 < g.S ? (g.S - s0 + g.sw - 1) / g.sw : 0;
    Kd = Rr * Ss * g.K;  // this class's reduction; the filter rows keep their full R*S*K stride
    if (m0 >= M) return;  // uniform per workgroup: the grid is sized for the largest class
  }
  auto class_pix = [&](int m) {  // MODE 2 class row -> input pixel
    const int hw = Hc * Wc, n = m / hw, rem = m - n * hw, i2 = rem / Wc, j2 = rem - i2 * Wc;
    return (n * g.H + i2 * g.sh + py) * g.W + j2 * g.sw + px;
  };

  // per-thread gathered rows: image base pixel and the (h, w) origin of the window
  int a_base[AR], a_h[AR], a_w[AR];
  bool a_ok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + trow + 32 * i;
    a_ok[i] = m < M;
    const int mm = a_ok[i] ? m : 0;
    if (MODE == 0) {
      const int hw = g.OH * g.OW, n = mm / hw, rem = mm - n * hw, oh = rem / g.OW, ow = rem - oh * g.OW;
      a_base[i] = n * g.H * g.W;
      a_h[i] = oh * g.sh - g.ph;
      a_w[i] = ow * g.sw - g.pw;
    } else if (MODE == 1) {
      const int hw = g.H * g.W, n = mm / hw, rem = mm - n * hw, ih = rem / g.W, iw = rem - ih * g.W;
      a_base[i] = n * g.OH * g.OW;
      a_h[i] = ih + g.ph;
      a_w[i] = iw + g.pw;
    } else {
      const int hw = Hc * Wc, n = mm / hw, rem = mm - n * hw, i2 = rem / Wc, j2 = rem - i2 * Wc;
      a_base[i] = n * g.OH * g.OW;
      a_h[i] = i2 * g.sh + py + g.ph;
      a_w[i] = j2 * g.sw + px + g.pw;
    }
  }
  const int64_t wrow = MODE == 2 ? (int64_t)g.R * g.S * g.K : Kd;  // filter row stride
  const bf16* b_row[BR];
  bool b_ok[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + trow + 32 * i;
    b_ok[i] = n < N;
    b_row[i] = wmat + (int64_t)(b_ok[i] ? n : 0) * wrow;
  }

  u32x4 ra[AR], rb[BR];
  const u32x4 zero = {0u, 0u, 0u, 0u};
  auto gload = [&](int kt) {
    const int kk = kt * kBK + kc * 8;
    const bool kin = kk < Kd;
    const int CH = MODE == 0 ? g.C : g.K;
    const int rs = kk / CH, ch = kk - rs * CH;
    int r, s;
    if (MODE == 2) {
      const int rr = rs / Ss;
      r = r0 + rr * g.sh;
      s = s0 + (rs - rr * Ss) * g.sw;
    } else {
      r = rs / g.S;
      s = rs - r * g.S;
    }
    const int boff = MODE == 2 ? (r * g.S + s) * g.K + ch : kk;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      u32x4 v = zero;
      if (kin && a_ok[i]) {
        if (MODE == 2) {
          // the class guarantees divisibility; only the image border can cut a tap
          const int th = a_h[i] - r, tw = a_w[i] - s;
          if (th >= 0 && tw >= 0) {
            const int oh = th / g.sh, ow = tw / g.sw;
            if (oh < g.OH && ow < g.OW)
              v = *reinterpret_cast<const u32x4*>(src + (int64_t)(a_base[i] + oh * g.OW + ow) * g.K + ch);
          }
        } else if (MODE == 0) {
          const int ih = a_h[i] + r * g.dh, iw = a_w[i] + s * g.dw;
          if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
            v = *reinterpret_cast<const u32x4*>(src + (int64_t)(a_base[i] + ih * g.W + iw) * g.C + ch);
        } else {
          int oh = a_h[i] - r * g.dh, ow = a_w[i] - s * g.dw;
          bool ok = oh >= 0 && ow >= 0;
          if (ok && g.sh > 1) {
            ok = (oh % g.sh) == 0;
            oh /= g.sh;
          }
          if (ok && g.sw > 1) {
            ok = (ow % g.sw) == 0;
            ow /= g.sw;
          }
          if (ok && oh < g.OH && ow < g.OW)
            v = *reinterpret_cast<const u32x4*>(src + (int64_t)(a_base[i] + oh * g.OW + ow) * g.K + ch);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = (kin && b_ok[i]) ? *reinterpret_cast<const u32x4*>(b_row[i] + boff) : zero;
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AR; ++i)
      *reinterpret_cast<u32x4*>(As + (buf * BM + trow + 32 * i) * LD + kc * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<u32x4*>(Bs + (buf * BN + trow + 32 * i) * LD + kc * 8) = rb[i];
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (Kd + kBK - 1) / kBK;
  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int ks = 0; ks < kBK / 32; ++ks) {
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int a = 0; a < RM; ++a)
        af[a] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const u32x4*>(As + (buf * BM + wr * WM + a * 16 + fr) * LD + ks * 32 + fk));
#pragma unroll
      for (int b = 0; b < RN; ++b)
        bfg[b] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const u32x4*>(Bs + (buf * BN + wc * WN + b * 16 + fr) * LD + ks * 32 + fk));
#pragma unroll
      for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfg[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D of 16x16x32 -> col = lane & 15, row = 4 * (lane >> 4) + j
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) {
      const int col = n0 + wc * WN + b * 16 + fr;
      if (col >= N) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + wr * WM + a * 16 + 4 * (lane >> 4) + j;
        if (row >= M) continue;
        const int64_t o = (int64_t)(MODE == 2 ? class_pix(row) : row) * N + col;
        if (y32) {
          y32[o] = acc[a][b][j];
        } else {
          float v = acc[a][b][j];
          if (MODE >= 1 && add_d != nullptr) {  // residual-branch gradient (ReLU-masked by add_y)
            const float ad = __bfloat162float(add_d[o]);
            v += (add_y == nullptr || __bfloat162float(add_y[o]) > 0.f) ? ad : 0.f;
          }
          y[o] = __float2bfloat16(v);
        }
      }
    }
}

// ---------------------------------------------------------------- wgrad
template <int BMW, int BNW>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(ConvGeom g, const bf16* __restrict__ x,
                                                         const bf16* __restrict__ dy, float* __restrict__ dw, int P,
                                                         int Kd, int chunk, FastDiv fd_hw, FastDiv fd_ow) {
  constexpr int BP = 64;  // pixels per LDS stage (2 MFMA k-steps)
  constexpr int WM = BMW / 2, WN = BNW / 2, RM = WM / 16, RN = WN / 16;
  constexpr int LDA = BMW + kPad, LDB = BNW + kPad;
  constexpr int AC = BP * BMW / 8 / kThreads, BC = BP * BNW / 8 / kThreads;  // 16-B chunks per thread
  __shared__ __align__(16) bf16 smem[2 * BP * (LDA + LDB)];
  bf16* As = smem;
  bf16* Bs = smem + 2 * BP * LDA;

  const int K = g.K;
  const int tilesN = (Kd + BNW - 1) / BNW;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / tilesN) * BMW, n0 = (wg % tilesN) * BNW;
  const int p_begin = blockIdx.y * chunk, p_end = min(P, p_begin + chunk);
  if (p_begin >= p_end) return;  // uniform per block
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int hw = g.OH * g.OW;

  // fixed per-thread chunk columns: A (dy) chunk -> (pixel row, 8 output channels)
  int a_prow[AC], a_col[AC];
#pragma unroll
  for (int i = 0; i < AC; ++i) {
    const int id = tid + kThreads * i;
    a_prow[i] = id / (BMW / 8);
    a_col[i] = m0 + (id % (BMW / 8)) * 8;
  }
  // B (im2col x) chunk -> (pixel row, 8 channels at one (r, s))
  int b_prow[BC], b_col[BC], b_r[BC], b_s[BC], b_c[BC];
#pragma unroll
  for (int i = 0; i < BC; ++i) {
    const int id = tid + kThreads * i;
    b_prow[i] = id / (BNW / 8);
    const int col = n0 + (id % (BNW / 8)) * 8;
    b_col[i] = col;
    const int rs = col / g.C;
    b_c[i] = col - rs * g.C;
    const int r = rs / g.S;
    b_r[i] = r * g.dh - g.ph;  // input row / column offsets of the tap: ih = oh * sh + b_r
    b_s[i] = (rs - r * g.S) * g.dw - g.pw;
  }
  u32x4 ra[AC], rb[BC];
  const u32x4 zero = {0u, 0u, 0u, 0u};
  auto gload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < AC; ++i) {
      const int p = p0 + a_prow[i];
      // unconditional load from a clamped offset, zero selected afterwards: straight-line code
      // instead of one exec-masked branch per load
      const bool ok = p < p_end && a_col[i] < K;
      const u32x4 t = *reinterpret_cast<const u32x4*>(dy + (ok ? p * K + a_col[i] : 0));
      ra[i] = ok ? t : zero;
    }
#pragma unroll
    for (int i = 0; i < BC; ++i) {
      const int p = p0 + b_prow[i];
      // 32-bit offsets: the binding bounds N*H*W*C and N*OH*OW*K below 2^31
      const int n = (int)fdiv((unsigned)p, fd_hw), rem = p - n * hw, oh = (int)fdiv((unsigned)rem, fd_ow),
                ow = rem - oh * g.OW;
      const int ih = oh * g.sh + b_r[i], iw = ow * g.sw + b_s[i];
      const bool ok = p < p_end && b_col[i] < Kd && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const u32x4 t = *reinterpret_cast<const u32x4*>(x + (ok ? ((n * g.H + ih) * g.W + iw) * g.C + b_c[i] : 0));
      rb[i] = ok ? t : zero;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AC; ++i)
      *reinterpret_cast<u32x4*>(As + (buf * BP + a_prow[i]) * LDA + (a_col[i] - m0)) = ra[i];
#pragma unroll
    for (int i = 0; i < BC; ++i)
      *reinterpret_cast<u32x4*>(Bs + (buf * BP + b_prow[i]) * LDB + (b_col[i] - n0)) = rb[i];
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads: lane 16g + 4q + pp addresses row (8g + q [+4]) cols (c0 + 4pp)
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  gload(p_begin);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int p0 = p_begin; p0 < p_end; p0 += BP) {
    const bool more = p0 + BP < p_end;
    if (more) gload(p0 + BP);
#pragma unroll
    for (int ks = 0; ks < BP / 32; ++ks) {
      const int prow = buf * BP + ks * 32 + 8 * tg + tq;
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int a = 0; a < RM; ++a) {
        const bf16* p1 = As + prow * LDA + wr * WM + a * 16 + 4 * tp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1 + 4 * LDA));
        af[a] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int b = 0; b < RN; ++b) {
        const bf16* p1 = Bs + prow * LDB + wc * WN + b * 16 + 4 * tp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1));
        const s16x4 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1 + 4 * LDB));
        bfg[b] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int a = 0; a < RM; ++a)
#pragma unroll
        for (int b = 0; b < RN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfg[b], acc[a][b], 0, 0, 0);
    }
    if (more) sstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  const int fr = lane & 15;
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) {
      const int col = n0 + wc * WN + b * 16 + fr;
      if (col >= Kd) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + wr * WM + a * 16 + 4 * (lane >> 4) + j;
        if (row < K) unsafeAtomicAdd(dw + (int64_t)row * Kd + col, acc[a][b][j]);
      }
    }
}


// ---------------------------------------------------------------- 3x3 / stride 1 / pad 1 from an LDS patch
// The im2col gather of igemm_kernel re-reads every input pixel for each of the 9 taps (9x the
// input through L2 per output-channel tile). For the unit-stride 3x3 layers a workgroup instead
// owns TH full output rows of one image: per 64-channel chunk it stages the (TH + 2) x (W + 2)
// input patch once (zero border), then walks the 9 taps, staging only that tap's [BN][64] filter
// slice and reading the MFMA A fragments from the patch at the tap's shifted pixel offsets.
// FLIP = the input gradient (dgrad of a 3x3 / s1 / p1 conv is the same conv of dy with the
// filter rotated by 180 degrees: patch offset (2 - r, 2 - s) with the weights of tap (r, s)).
template <int BN, int TW, int TH, bool FLIP>
__global__ __launch_bounds__(kThreads) void conv3x3_patch_kernel(ConvGeom g, const bf16* __restrict__ src,
                                                                 const bf16* __restrict__ wmat,
                                                                 bf16* __restrict__ y, int Cin, int Cout,
                                                                 const bf16* __restrict__ add_d,
                                                                 const bf16* __restrict__ add_y) {
  // a tile = IPT images x TH output rows x TW (= W) columns = 128 pixels; small planes (8x8, 4x4)
  // put several whole images in one tile, each with its own zero-bordered patch
  constexpr int BM = 128, IPT = BM / (TH * TW), PW = TW + 2, PH = TH + 2, NPIX = IPT * PH * PW;
  static_assert(IPT * TH * TW == BM, "tile must be 128 pixels");
  constexpr int WM = BM / 2, WN = BN / 2, RM = WM / 16, RN = WN / 16;
  constexpr int LD = kBK + kPad;
  extern __shared__ __align__(16) bf16 dsm[];
  bf16* Ps = dsm;                  // [NPIX][LD]   input patch(es), one 64-channel chunk
  bf16* Bs = dsm + NPIX * LD;      // [BN][LD]     one tap's filter slice
  const int H = g.H;               // == OH (stride 1, pad 1); W == TW
  const int rows_tiles = H / TH;   // IPT > 1 only when TH == H (rows_tiles == 1)
  const int tilesN = Cout / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wg / tilesN, n0 = (wg % tilesN) * BN;
  const int img0 = (tm / rows_tiles) * IPT, oh0 = (tm % rows_tiles) * TH;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int64_t wrow = 9 * (int64_t)Cin;

  f32x4 acc[RM][RN];
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment pixel -> patch row base (tap (0, 0)); the tap adds (r, s)
  int prow[RM];
#pragma unroll
  for (int a = 0; a < RM; ++a) {
    const int m = wr * WM + a * 16 + fr, im = m / (TH * TW), rem = m - im * (TH * TW), ohl = rem / TW,
              ow = rem - ohl * TW;
    prow[a] = im * PH * PW + ohl * PW + ow;
  }
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const int nch = Cin / kBK;
  for (int cc = 0; cc < nch; ++cc) {
    // stage the patch(es): NPIX pixels x 8 chunks of 8 channels
    for (int i = tid; i < NPIX * 8; i += kThreads) {
      const int px = i >> 3, ch = (i & 7) * 8, im = px / (PH * PW), q = px - im * (PH * PW), pr = q / PW,
                pc = q - pr * PW;
      const int ih = oh0 - 1 + pr, iw = pc - 1;
      u32x4 v = zero;
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)TW)
        v = *reinterpret_cast<const u32x4*>(src + (((int64_t)(img0 + im) * H + ih) * TW + iw) * Cin + cc * kBK + ch);
      *reinterpret_cast<u32x4*>(Ps + px * LD + ch) = v;
    }
    for (int t = 0; t < 9; ++t) {
      // this tap's filter slice [BN][64]
      for (int i = tid; i < BN * 8; i += kThreads) {
        const int row = i >> 3, ch = (i & 7) * 8;
        *reinterpret_cast<u32x4*>(Bs + row * LD + ch) =
            *reinterpret_cast<const u32x4*>(wmat + (int64_t)(n0 + row) * wrow + (int64_t)t * Cin + cc * kBK + ch);
      }
      __syncthreads();
      const int r = t / 3, sx = t - 3 * r;
      const int off = FLIP ? (2 - r) * PW + (2 - sx) : r * PW + sx;
#pragma unroll
      for (int ks = 0; ks < kBK / 32; ++ks) {
        bf16x8 af[RM], bfg[RN];
#pragma unroll
        for (int a = 0; a < RM; ++a)
          af[a] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(Ps + (prow[a] + off) * LD + ks * 32 + fk));
#pragma unroll
        for (int b = 0; b < RN; ++b)
          bfg[b] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(Bs + (wc * WN + b * 16 + fr) * LD + ks * 32 + fk));
#pragma unroll
        for (int a = 0; a < RM; ++a)
#pragma unroll
          for (int b = 0; b < RN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfg[b], acc[a][b], 0, 0, 0);
      }
      __syncthreads();  // Bs (and, after the last tap, Ps) are rewritten next
    }
  }
#pragma unroll
  for (int a = 0; a < RM; ++a)
#pragma unroll
    for (int b = 0; b < RN; ++b) {
      const int col = n0 + wc * WN + b * 16 + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = wr * WM + a * 16 + 4 * (lane >> 4) + j, im = m / (TH * TW), rem = m - im * (TH * TW),
                  ohl = rem / TW, ow = rem - ohl * TW;
        const int64_t o = (((int64_t)(img0 + im) * H + oh0 + ohl) * TW + ow) * Cout + col;
        float v = acc[a][b][j];
        if (add_d != nullptr) {
          const float ad = __bfloat162float(add_d[o]);
          v += (add_y == nullptr || __bfloat162float(add_y[o]) > 0.f) ? ad : 0.f;
        }
        y[o] = __float2bfloat16(v);
      }
    }
}

template <int BN, int TW, int TH, bool FLIP>
hipError_t launch_patch(const ConvGeom& g, const bf16* src, const bf16* wm, bf16* y, int Cin, int Cout, hipStream_t st,
                        const bf16* add_d, const bf16* add_y) {
  constexpr int IPT = 128 / (TW * TH), NPIX = IPT * (TH + 2) * (TW + 2);
  const size_t lds = sizeof(bf16) * (size_t)(NPIX + BN) * (kBK + kPad);
  const int grid = (g.N / IPT) * (g.H / TH) * (Cout / BN);
  hipLaunchKernelGGL((conv3x3_patch_kernel<BN, TW, TH, FLIP>), dim3(grid), dim3(kThreads), lds, st, g, src, wm, y, Cin,
                     Cout, add_d, add_y);
  return hipGetLastError();
}

// 3x3 / s1 / p1 / d1 on 32x32 (4-row tiles), 16x16 (8-row tiles) or 8x8 (2 images per tile) planes
// with 64-channel chunks on both sides; anything else keeps the im2col kernel. 4x4 planes (8 images
// per tile) measured slower than the im2col kernel at ResNet-18's l4 (fwd 72 -> 102 us: 256 workgroups
// of 9 serial tap stages for 512 channels).
bool patch_ok(const ConvGeom& g, int Cin, int Cout) {
  if (!(g.R == 3 && g.S == 3 && g.sh == 1 && g.sw == 1 && g.ph == 1 && g.pw == 1 && g.dh == 1 &&
                     g.dw == 1 && g.OH == g.H && g.OW == g.W && Cin % 64 == 0 && Cout % 64 == 0))
    return false;
  if (g.W == 32 && g.H % 4 == 0) return true;
  if (g.W == 16 && g.H % 8 == 0) return true;
  return g.W == 8 && g.H == 8 && g.N % 2 == 0;  // l3: fwd 44.7 -> 38.3, dgrad 48.8 -> 37.1 us
}

template <bool FLIP>
hipError_t dispatch_patch(const ConvGeom& g, const bf16* src, const bf16* wm, bf16* y, int Cin, int Cout,
                          hipStream_t st, const bf16* add_d, const bf16* add_y) {
  const bool wide = Cout % 128 == 0 && (int64_t)g.N * g.H * g.W / 128 * (Cout / 128) >= 512;
#define PATCH(TW, TH)                                                                      \
  return wide ? launch_patch<128, TW, TH, FLIP>(g, src, wm, y, Cin, Cout, st, add_d, add_y) \
              : launch_patch<64, TW, TH, FLIP>(g, src, wm, y, Cin, Cout, st, add_d, add_y)
  if (g.W == 32) PATCH(32, 4);
  if (g.W == 16) PATCH(16, 8);
  if (g.W == 8) PATCH(8, 8);
  PATCH(4, 4);
#undef PATCH
}

template <int MODE, int BM, int BN>
hipError_t launch_igemm(const ConvGeom& g, const bf16* src, const bf16* wm, bf16* y, float* y32, int M, int N, int Kd,
                        hipStream_t st, const bf16* add_d, const bf16* add_y) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int classes = MODE == 2 ? g.sh * g.sw : 1;  // M is the largest (first) class there
  hipLaunchKernelGGL((igemm_kernel<MODE, BM, BN>), dim3(grid, classes), dim3(kThreads), 0, st, g, src, wm, y, y32, M,
                     N, Kd, add_d, add_y);
  return hipGetLastError();
}

template <int MODE>
hipError_t dispatch(const ConvGeom& g, const bf16* src, const bf16* wm, bf16* y, float* y32, int M, int N, int Kd,
                    hipStream_t st, const bf16* add_d = nullptr, const bf16* add_y = nullptr) {
  const bool wide = N > 64;
  const int tiles128 = ((M + 127) / 128) * ((N + (wide ? 127 : 63)) / (wide ? 128 : 64));
  const bool tall = tiles128 >= 512;  // else halve BM to fill the 256 CUs
  if (wide) return tall ? launch_igemm<MODE, 128, 128>(g, src, wm, y, y32, M, N, Kd, st, add_d, add_y)
                        : launch_igemm<MODE, 64, 128>(g, src, wm, y, y32, M, N, Kd, st, add_d, add_y);
  return tall ? launch_igemm<MODE, 128, 64>(g, src, wm, y, y32, M, N, Kd, st, add_d, add_y)
              : launch_igemm<MODE, 64, 64>(g, src, wm, y, y32, M, N, Kd, st, add_d, add_y);
}

}  // namespace

hipError_t launch_fwd(const ConvGeom& g, const bf16* x, const bf16* w, bf16* y, float* out_f32, hipStream_t st) {
  if (out_f32 == nullptr && patch_ok(g, g.C, g.K)) return dispatch_patch<false>(g, x, w, y, g.C, g.K, st, nullptr, nullptr);
  return dispatch<0>(g, x, w, y, out_f32, g.N * g.OH * g.OW, g.K, g.R * g.S * g.C, st);
}

hipError_t launch_dgrad(const ConvGeom& g, const bf16* dy, const bf16* wt, bf16* dx, hipStream_t st, const bf16* add_d,
                        const bf16* add_y) {
  constexpr bool phase_split = true;
  if (patch_ok(g, g.K, g.C)) return dispatch_patch<true>(g, dy, wt, dx, g.K, g.C, st, add_d, add_y);
  // 1x1 strided (the shortcut): one class holds every tap, the unit-stride path is as fast (measured)
  if (phase_split && (g.sh > 1 || g.sw > 1) && g.dh == 1 && g.dw == 1 && g.R * g.S > 1) {
    const int M0 = g.N * ((g.H + g.sh - 1) / g.sh) * ((g.W + g.sw - 1) / g.sw);  // class (0, 0): the largest
    const int rs0 = ((g.R + g.sh - 1) / g.sh) * ((g.S + g.sw - 1) / g.sw) * g.K;
    return dispatch<2>(g, dy, wt, dx, nullptr, M0, g.C, rs0, st, add_d, add_y);
  }
  return dispatch<1>(g, dy, wt, dx, nullptr, g.N * g.H * g.W, g.C, g.R * g.S * g.K, st, add_d, add_y);
}

hipError_t launch_wgrad(const ConvGeom& g, const bf16* x, const bf16* dy, float* dw32, hipStream_t st) {
  const int P = g.N * g.OH * g.OW, Kd = g.R * g.S * g.C;
  const bool wideM = g.K > 64, wideN = Kd > 64;
  const int tiles = ((g.K + (wideM ? 127 : 63)) / (wideM ? 128 : 64)) * ((Kd + (wideN ? 127 : 63)) / (wideN ? 128 : 64));
  constexpr int BP = 64;
  // Split-K over pixels: every split adds its 128 x 128 fp32 tile into dw32 with atomics, so the
  // split count trades fill (workgroups) against atomic traffic (tiles x splits x 64 KB).
  // Round-5 sweep on the ResNet-18 shapes (profiles/conv_graph_table_r05.log): 2048 WGs / >= 4
  // stages (the old policy) 1.64 ms for the nine layers' fwd+bwd, 512 / >= 16: 1.42 ms - the
  // 128 x 128 tiles of l2-l4 spent most of their time in atomics (l3 wgrad 110 -> 61 us).
  // Round 6 (profiles/conv_wgrad_r06.log): split-K slabs + a reduce launch instead of the atomics,
  // and operand loads issued two stages ahead, both measured slower; the gather's divisions went
  // to FastDiv (nine layers 500 -> 476 us).
  constexpr int target_wg = 512, min_stages = 16;
  int splits = (target_wg + tiles - 1) / tiles;
  const int max_splits = (P + min_stages * BP - 1) / (min_stages * BP);  // >= min_stages stages per block
  splits = splits < 1 ? 1 : (splits > max_splits ? max_splits : splits);
  if (splits < 1) splits = 1;
  int chunk = (P + splits - 1) / splits;
  chunk = (chunk + BP - 1) / BP * BP;
  splits = (P + chunk - 1) / chunk;
  dim3 grid(tiles, splits);
  const FastDiv fh = make_fastdiv((unsigned)(g.OH * g.OW)), fo = make_fastdiv((unsigned)g.OW);
  if (wideM && wideN)
    hipLaunchKernelGGL((wgrad_kernel<128, 128>), grid, dim3(kThreads), 0, st, g, x, dy, dw32, P, Kd, chunk, fh, fo);
  else if (wideM)
    hipLaunchKernelGGL((wgrad_kernel<128, 64>), grid, dim3(kThreads), 0, st, g, x, dy, dw32, P, Kd, chunk, fh, fo);
  else if (wideN)
    hipLaunchKernelGGL((wgrad_kernel<64, 128>), grid, dim3(kThreads), 0, st, g, x, dy, dw32, P, Kd, chunk, fh, fo);
  else
    hipLaunchKernelGGL((wgrad_kernel<64, 64>), grid, dim3(kThreads), 0, st, g, x, dy, dw32, P, Kd, chunk, fh, fo);
  return hipGetLastError();
}

}  // namespace conv
}  // namespace katib_hip
