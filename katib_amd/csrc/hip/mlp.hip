// Fused MLP training kernels for gfx950 (BASELINE config 2: TPE over lr / batch size / width
// of an MNIST MLP). One train step of 784 -> h -> h/2 -> 10 is nine launches,
// all graph-captured, with no separate bias, activation, gather, cast, loss or optimizer
// kernels:
//
//  lin_fwd    Y = act(X W^T + b): bf16 MFMA (v_mfma_f32_16x16x32_bf16) over K-contiguous
//             operands staged through padded LDS rows; optional row gather of X (the
//             minibatch indices into the device-resident dataset), bias + ReLU epilogue, or
//             a ReLU-derivative mask epilogue (dgrad: dX = (dY W) * [X_act > 0] with the
//             transposed bf16 weight shadow as the K-contiguous operand).
//  lin_wgrad  dW = dY^T X reduced over the whole minibatch inside one workgroup (the
//             minibatch is the reduction, <= a few hundred rows), both operands read with
//             ds_read_b64_tr_b16, and SGD-with-momentum applied in the epilogue: fp32
//             master, momentum buffer, bf16 weight and transposed-weight shadows; the
//             workgroups of the first K tile also reduce and update the bias.
//  xent_small cross-entropy + its gradient for a handful of classes, one lane per row.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "mlp.h"

namespace katib_hip {
namespace mlp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 64, BN = 64, BK = 64, PAD = 8, LD = BK + PAD;

__device__ __forceinline__ float bf2f(u16 b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

// ------------------------------------------------------------------ Y = epi(A B^T)
// A [M][K] (rows optionally gathered through idx), B [N][K], both K-contiguous; K % 8 == 0.
// epi: + bias, ReLU (relu != 0), or * [mask > 0] (mask [M][N] bf16). Output bf16 [M][N].
__global__ __launch_bounds__(256) void gemm_nt_k(const u16* __restrict__ A, const int64_t* __restrict__ idx,
                                                 const u16* __restrict__ B, const float* __restrict__ bias,
                                                 const u16* __restrict__ mask, u16* __restrict__ Y, int M, int N,
                                                 int K, int relu) {
  __shared__ __align__(16) u16 smem[2 * (BM + BN) * LD];
  u16* As = smem;
  u16* Bs = smem + 2 * BM * LD;
  const int tilesN = (N + BN - 1) / BN;
  const int m0 = (blockIdx.x / tilesN) * BM, n0 = (blockIdx.x % tilesN) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const int kc = tid & 7, trow = tid >> 3;  // 32 rows x 8 chunks of 16 B per pass
  const u16* arow[2];
  const u16* brow[2];
  bool aok[2], bok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + trow + 32 * i, n = n0 + trow + 32 * i;
    aok[i] = m < M;
    bok[i] = n < N;
    const int64_t am = aok[i] ? (idx ? idx[m] : m) : 0;
    arow[i] = A + am * K;
    brow[i] = B + (int64_t)(bok[i] ? n : 0) * K;
  }
  u32x4 ra[2], rb[2];
  const u32x4 zero = {0u, 0u, 0u, 0u};
  auto gload = [&](int kt) {
    const int kk = kt * BK + kc * 8;
    const bool kin = kk < K;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ra[i] = (kin && aok[i]) ? *reinterpret_cast<const u32x4*>(arow[i] + kk) : zero;
      rb[i] = (kin && bok[i]) ? *reinterpret_cast<const u32x4*>(brow[i] + kk) : zero;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<u32x4*>(As + (buf * BM + trow + 32 * i) * LD + kc * 8) = ra[i];
      *reinterpret_cast<u32x4*>(Bs + (buf * BN + trow + 32 * i) * LD + kc * 8) = rb[i];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
        af[a] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const u32x4*>(As + (buf * BM + wr * 32 + a * 16 + fr) * LD + ks * 32 + fk));
#pragma unroll
      for (int b = 0; b < 2; ++b)
        bfr[b] = __builtin_bit_cast(
            bf16x8, *reinterpret_cast<const u32x4*>(Bs + (buf * BN + wc * 32 + b * 16 + fr) * LD + ks * 32 + fk));
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = n0 + wc * 32 + b * 16 + fr;
      if (col >= N) continue;
      const float bv = bias ? bias[col] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m0 + wr * 32 + a * 16 + 4 * (lane >> 4) + j;
        if (row >= M) continue;
        float v = acc[a][b][j] + bv;
        if (relu) v = fmaxf(v, 0.f);
        if (mask && !(bf2f(mask[(int64_t)row * N + col]) > 0.f)) v = 0.f;
        Y[(int64_t)row * N + col] = f2bf(v);
      }
    }
}

// ------------------------------------------------------------------ dW = dY^T X, fused SGD
// dY [M][N] bf16, X [M][K] bf16 (rows gathered through idx when given), W [N][K] fp32 master.
// One workgroup per 64 x 64 tile of W, reducing over all M rows.
__global__ __launch_bounds__(256) void wgrad_sgd_k(const u16* __restrict__ dY, const u16* __restrict__ X,
                                                   const int64_t* __restrict__ idx, int M, int N, int K,
                                                   float* __restrict__ W, float* __restrict__ Wm,
                                                   u16* __restrict__ W16, u16* __restrict__ W16t,
                                                   float* __restrict__ bias, float* __restrict__ bm,
                                                   const float* __restrict__ lr_p, float mom) {
  constexpr int BP = 64;
  constexpr int LDA = BN + PAD, LDB = BK + PAD;
  __shared__ __align__(16) u16 smem[2 * BP * (LDA + LDB)];
  __shared__ float bsum[4][64];
  u16* As = smem;                 // [buf][m][n]
  u16* Bs = smem + 2 * BP * LDA;  // [buf][m][k]
  const int tilesK = (K + BK - 1) / BK;
  const int n0 = (blockIdx.x / tilesK) * BN, k0 = (blockIdx.x % tilesK) * BK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 1, wc = wid & 1;
  const bool do_bias = bias != nullptr && k0 == 0;
  // 64 rows x 8 chunks per operand per stage: 2 chunks per thread each
  int prow[2], pch[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + 256 * i;
    prow[i] = id >> 3;
    pch[i] = id & 7;
  }
  u32x4 ra[2], rb[2];
  const u32x4 zero = {0u, 0u, 0u, 0u};
  auto gload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = p0 + prow[i];
      const int n = n0 + pch[i] * 8, k = k0 + pch[i] * 8;
      ra[i] = (m < M && n < N) ? *reinterpret_cast<const u32x4*>(dY + (int64_t)m * N + n) : zero;
      const int64_t xm = m < M ? (idx ? idx[m] : m) : 0;
      rb[i] = (m < M && k < K) ? *reinterpret_cast<const u32x4*>(X + xm * K + k) : zero;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      *reinterpret_cast<u32x4*>(As + (buf * BP + prow[i]) * LDA + pch[i] * 8) = ra[i];
      *reinterpret_cast<u32x4*>(Bs + (buf * BP + prow[i]) * LDB + pch[i] * 8) = rb[i];
    }
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  gload(0);
  sstore(0);
  __syncthreads();
  int buf = 0;
  for (int p0 = 0; p0 < M; p0 += BP) {
    const bool more = p0 + BP < M;
    if (more) gload(p0 + BP);
    if (do_bias && tid < 256) {  // column sums of the staged dY tile: 4 row groups x 64 columns
      const int c = tid & 63, rg = tid >> 6;
      for (int r = rg; r < BP; r += 4) bacc += bf2f(As[(buf * BP + r) * LDA + c]);
    }
#pragma unroll
    for (int ks = 0; ks < BP / 32; ++ks) {
      const int pr = buf * BP + ks * 32 + 8 * tg + tq;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const u16* p1 = As + pr * LDA + wr * 32 + a * 16 + 4 * tp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1 + 4 * LDA));
        af[a] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const u16* p1 = Bs + pr * LDB + wc * 32 + b * 16 + 4 * tp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1 + 4 * LDB));
        bfr[b] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    if (more) sstore(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  const float lr = lr_p[0];
  // SGD with momentum (torch semantics, dampening 0): buf = mom * buf + g; p -= lr * buf
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int k = k0 + wc * 32 + b * 16 + (lane & 15);
      if (k >= K) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wr * 32 + a * 16 + 4 * (lane >> 4) + j;
        if (n >= N) continue;
        const int64_t o = (int64_t)n * K + k;
        const float mb = mom * Wm[o] + acc[a][b][j];
        const float p = W[o] - lr * mb;
        Wm[o] = mb;
        W[o] = p;
        const u16 pb = f2bf(p);
        W16[o] = pb;
        W16t[(int64_t)k * N + n] = pb;
      }
    }
  if (do_bias) {
    bsum[tid >> 6][tid & 63] = bacc;
    __syncthreads();
    if (tid < 64 && n0 + tid < N) {
      const float g = (bsum[0][tid] + bsum[1][tid]) + (bsum[2][tid] + bsum[3][tid]);
      const float mb = mom * bm[n0 + tid] + g;
      bm[n0 + tid] = mb;
      bias[n0 + tid] -= lr * mb;
    }
  }
}

// ------------------------------------------------------------------ softmax cross-entropy, few classes
// logits [M][ld] bf16 (first C columns real); dlogits = (softmax - onehot) / M (pad columns 0);
// stats[0] += sum of losses / M, stats[1] += number of correct argmax predictions.
__global__ __launch_bounds__(256) void xent_small_k(const u16* __restrict__ logits, const int64_t* __restrict__ y,
                                                    const int64_t* __restrict__ idx, u16* __restrict__ dl, int M,
                                                    int C, int ld, float* __restrict__ stats) {
  __shared__ float red[2][4];
  const int r = blockIdx.x * 256 + threadIdx.x;
  float loss = 0.f, correct = 0.f;
  if (r < M) {
    const u16* L = logits + (int64_t)r * ld;
    const int64_t t = y[idx ? idx[r] : r];
    float mx = -INFINITY;
    int arg = 0;
    for (int c = 0; c < C; ++c) {
      const float v = bf2f(L[c]);
      if (v > mx) {
        mx = v;
        arg = c;
      }
    }
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(bf2f(L[c]) - mx);
    const float lse = mx + __logf(s);
    loss = (t >= 0 && t < C) ? (lse - bf2f(L[t])) / M : 0.f;
    correct = (arg == t) ? 1.f : 0.f;
    for (int c = 0; c < ld; ++c)
      dl[(int64_t)r * ld + c] = f2bf(c < C ? (__expf(bf2f(L[c]) - lse) - (c == t ? 1.f : 0.f)) / M : 0.f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_xor(loss, o, 64);
    correct += __shfl_xor(correct, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = loss;
    red[1][threadIdx.x >> 6] = correct;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(stats, (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]));
    atomicAdd(stats + 1, (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
  }
}

}  // namespace

hipError_t lin_fwd(const bf16* x, const int64_t* idx, const bf16* w, const float* bias, const bf16* mask, bf16* y,
                   int M, int N, int K, int relu, hipStream_t st) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(gemm_nt_k, dim3(grid), dim3(256), 0, st, reinterpret_cast<const u16*>(x), idx,
                     reinterpret_cast<const u16*>(w), bias, reinterpret_cast<const u16*>(mask),
                     reinterpret_cast<u16*>(y), M, N, K, relu);
  return hipGetLastError();
}

hipError_t lin_wgrad_sgd(const bf16* dy, const bf16* x, const int64_t* idx, int M, int N, int K, float* w, float* wm,
                         bf16* w16, bf16* w16t, float* bias, float* bm, const float* lr, float momentum,
                         hipStream_t st) {
  const int grid = ((N + BN - 1) / BN) * ((K + BK - 1) / BK);
  hipLaunchKernelGGL(wgrad_sgd_k, dim3(grid), dim3(256), 0, st, reinterpret_cast<const u16*>(dy),
                     reinterpret_cast<const u16*>(x), idx, M, N, K, w, wm, reinterpret_cast<u16*>(w16),
                     reinterpret_cast<u16*>(w16t), bias, bm, lr, momentum);
  return hipGetLastError();
}

hipError_t xent_small(const bf16* logits, const int64_t* y, const int64_t* idx, bf16* dl, int M, int C, int ld,
                      float* stats, hipStream_t st) {
  hipLaunchKernelGGL(xent_small_k, dim3((M + 255) / 256), dim3(256), 0, st, reinterpret_cast<const u16*>(logits), y,
                     idx, reinterpret_cast<u16*>(dl), M, C, ld, stats);
  return hipGetLastError();
}

}  // namespace mlp
}  // namespace katib_hip
