// 256 x 256-tile bf16 GEMM for the GPT-2 projections, forward and backward (gfx950):
//   C = op(A) op(B), op(A)[M][K] from A stored [M][K] (K-major) or [K][M] (MN-major),
//                    op(B)[K][N] from B stored [N][K] (K-major) or [K][N] (MN-major),
//   bf16 C (+ bias[N]) (EPI 0), bf16 U = C + bias and G = gelu_tanh(U) (EPI 1), or fp32 split-K slabs
//   [slice][M][N] (EPI 2). Forward = (K, K), dgrad = (K, MN), wgrad = (MN, MN): no transposed copies.
//
// Structure (cdna_hip_programming.md §5, "the 256^2 8-phase template", built for this layout family):
//   * 512 threads = 8 waves in two groups of 4; group g owns output rows [128 g, 128 g + 128) and each
//     wave of it 64 columns: 128 x 64 per wave = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (the
//     16x16x32 shape: at equal cycles per FLOP it holds a higher clock than 32x32x16 on random data,
//     MI355X_MICROARCH.md DVFS item 7).
//   * K-step 64; two LDS buffers of four 16 KB half-tiles [A0 | A1 | B0 | B1] (128 KB, one workgroup
//     per CU); group g stages A_g and B_g with global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip).
//   * Each K-tile runs as 4 phases of {fragment reads + one half of a half-tile's DMA, barrier, 16 MFMAs
//     (one 64 x 32 quadrant over K = 64) between s_setprio(1/0), barrier}. Group 1 runs one barrier
//     behind group 0, so on every SIMD one wave reads LDS and issues DMA while its partner computes
//     (ping-pong), and the DMA of tile k+1 / k+2 stays in flight across the barriers: each wave waits
//     for its own loads with a counted vmcnt once per K-tile (never __syncthreads, whose fence would
//     drain the DMA).
//   * Phase plan of K-tile t (buffer t & 1): P1 reads all B fragments + A rows 0-63 (16 ds_read_b128),
//     DMA A(t+1) half 1; P2 MFMAs only; P3 reads A rows 64-127 (into the same registers), DMA B(t+2)
//     half 0; P4 DMA B(t+2) half 1 + A(t+2) half 0 and the wait that retires tile t+1 (vmcnt 6: three
//     half-blocks of DMA stay in flight; A(t+1) had three phases to land). 64 fragment VGPRs + 128
//     accumulators. A_g is read by group g alone (free once its P3 reads retired); B_g by both groups,
//     free for group 0's DMA only from P3 (group 1's P1 reads retire in the segment that ends P2).
//     Measured alternative (profiles/gemm256_r06.log): the DMA two tiles ahead with the next tile's B
//     fragments read in P4 - 8192^3 equal, the MN-major GPT-2 shapes 10 % slower.
//   * K-major half-tile image: 128 rows x 128 B, 16-byte chunk c of row r at slot c ^ ((r >> 1) & 7):
//     every 16-lane phase of a ds_read_b128 fragment read then hits 16 distinct slots of the 256-byte
//     bank row (conflict-free; the (r & 7) form of gemm_bf16.hip is 2-way). The swizzle is applied to
//     the DMA's global source address (the LDS destination of an LDS-DMA is lane-linear) and undone on
//     the read. MN-major half-tile: 64 k rows x 256 B with gemm_bf16.hip's slot XOR, fragments by two
//     ds_read_b64_tr_b16 (hardware transpose).
//   * XCD-aware, bijective tile order (each XCD owns a contiguous range of row-major tiles: A panels
//     re-read from its own L2). M, N multiples of 128: the last tile row / column may be half outside;
//     its staging origin is clamped (re-reads valid rows) and its stores are skipped.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gemm_bf16.h"

namespace katib_hip {
namespace gemm {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(3))) s16x4* lds_s16x4;

constexpr int T = 256, BK = 64, HALF = 16384, BUF = 4 * HALF, LDS_BYTES = 2 * BUF;

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

__device__ __forceinline__ float gelu_tanh(float u) {
  const float z2 = (2.f * 0.7978845608028654f * 1.4426950408889634f) * u * (1.f + 0.044715f * u * u);
  return 0.5f * u * (2.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z2) + 1.f));
}

__device__ __forceinline__ int ksw(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int mn_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

// DMA block `blk` (0..15, 1 KB) of a half-tile image whose first mn row (K-major) / column (MN-major) is mn0
template <bool MN>
__device__ __forceinline__ void stage_blk(const uint16_t* __restrict__ src, int ld, int mn0, int k0, char* img, int blk,
                                          int lane) {
  if constexpr (MN) {
    const int row = blk * 4 + (lane >> 4);  // k row, 16 lanes per 256-byte row
    const int chunk = (lane & 15) ^ mn_swz(row);
    __builtin_amdgcn_global_load_lds(src + (size_t)(k0 + row) * ld + mn0 + chunk * 8, (lds_ptr)(img + blk * 1024), 16,
                                     0, 0);
  } else {
    const int row = blk * 8 + (lane >> 3);  // mn row, 8 lanes per 128-byte row
    const int chunk = (lane & 7) ^ ksw(row);
    __builtin_amdgcn_global_load_lds(src + (size_t)(mn0 + row) * ld + k0 + chunk * 8, (lds_ptr)(img + blk * 1024), 16,
                                     0, 0);
  }
}

// MFMA operand fragment: mn index mn + (lane & 15), k = kk * 32 + 8 (lane >> 4) + 0..7
template <bool MN>
__device__ __forceinline__ bf16x8 frag(const char* img, int mn, int kk, int lane) {
  if constexpr (MN) {
    const int li = lane & 15, q = lane >> 4;
    const int col = mn + 4 * (li & 3), chunk = col >> 3, half = (col >> 2) & 1;
    const int r0 = kk * 32 + 8 * q + (li >> 2), r1 = r0 + 4;
    const char* p0 = img + r0 * 256 + ((chunk ^ mn_swz(r0)) << 4) + half * 8;
    const char* p1 = img + r1 * 256 + ((chunk ^ mn_swz(r1)) << 4) + half * 8;
    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4)(p0));
    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4)(p1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
  } else {
    const int row = mn + (lane & 15), chunk = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((chunk ^ ksw(row)) << 4));
  }
}

// a raw workgroup barrier that nothing is scheduled across (no fence: LDS-DMA stays in flight)
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 16 MFMAs: accumulator rows i0..i0+3 x columns j0..j0+1 over the K-tile's two 32-deep slices
// The accumulators pass through empty asm statements before and after the cluster: the MFMA
// intrinsic touches no memory, so without them LLVM sinks part of a cluster past the next barrier
// (into the partner's compute segment) and the ping-pong collapses (seen in the .s: 6 of 16 MFMAs left).
__device__ __forceinline__ void pin(f32x4 (&acc)[8][4], int i0, int j0) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[i0 + i][j0 + j]));
}

__device__ __forceinline__ void quad(f32x4 (&acc)[8][4], const bf16x8 (&a)[2][4], const bf16x8 (&b)[2][4], int i0,
                                     int j0) {
  pin(acc, i0, j0);
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], b[kk][j0 + j], acc[i0 + i][j0 + j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
  pin(acc, i0, j0);
}

// ABL (measurement builds only, launch_g256_ablate): 1 no DMA in the K loop (tiles 0 / 1 re-used),
// 2 no fragment reads in the K loop (registers of the first read re-used), 3 neither, 4 no stagger
template <bool A_MN, bool B_MN, int EPI, int ABL = 0>
__global__ void __launch_bounds__(512) g256_kernel(const uint16_t* __restrict__ A, int lda, const uint16_t* __restrict__ B,
                                                   int ldb, const uint16_t* __restrict__ bias, void* __restrict__ Cv,
                                                   uint16_t* __restrict__ G, int M, int N, int kslice) {
  __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];  // the ONLY LDS object (DMA waits, guide §5 item 4a)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = wave >> 2, wq = wave & 3;
  const int TN = (N + T - 1) / T, nwg = TN * ((M + T - 1) / T), b = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8, loc = b / 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  // grouped order within the XCD's range: GM row panels at a time, column-major inside the group, so
  // the ~32 workgroups an XCD runs at once share 4 A panels and ~8 B panels (rather than 1 A panel and
  // 32 B panels): 2.7x fewer operand bytes per K-step from beyond the XCD's L2
  constexpr int GM = 4;
  const int TM = (M + T - 1) / T, grp = t / (GM * TN), gm = min(TM - grp * GM, GM), tg = t % (GM * TN);
  const int m0 = (grp * GM + tg % gm) * T, n0 = (tg / gm) * T;
  const int kbeg = blockIdx.y * kslice, nk = kslice / BK;
  const int am0 = min(m0 + g * 128, M - 128), bn0 = min(n0 + g * 128, N - 128);  // this group's staging origins
  const int cb = (wq & 1) * 64;                                                  // this wave's columns in its B half

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stageA = [&](int kt, int part) {
    char* img = lds + (kt & 1) * BUF + g * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) stage_blk<A_MN>(A, lda, am0, kbeg + kt * BK, img, wq * 4 + part * 2 + i, lane);
  };
  auto stageB = [&](int kt, int part) {
    char* img = lds + (kt & 1) * BUF + 2 * HALF + g * HALF;
#pragma unroll
    for (int i = 0; i < 2; ++i) stage_blk<B_MN>(B, ldb, bn0, kbeg + kt * BK, img, wq * 4 + part * 2 + i, lane);
  };
  constexpr bool kDma = ABL != 1 && ABL != 3, kReads = ABL != 2 && ABL != 3;
  auto wait_next = [&](int kt) {
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  // prologue: B(0), A(0), B(1), A(1) half 0; wait for tile 0 (the 6 DMA of tile 1 may stay in flight),
  // then group 1 falls one barrier behind
  stageB(0, 0);
  stageB(0, 1);
  stageA(0, 0);
  stageA(0, 1);
  if (nk > 1) {
    stageB(1, 0);
    stageB(1, 1);
    stageA(1, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
  if (ABL != 4 && g == 1) bar();
  bf16x8 bq[2][4], a4[2][4];
  if constexpr (!kReads) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bq[kk][j] = frag<B_MN>(lds + 2 * HALF + (wq >> 1) * HALF, cb + j * 16, kk, lane);
        a4[kk][j] = frag<A_MN>(lds + g * HALF, j * 16, kk, lane);
      }
  }

  for (int kt = 0; kt < nk; ++kt) {
    const char* ia = lds + (kt & 1) * BUF + g * HALF;
    const char* ib = lds + (kt & 1) * BUF + 2 * HALF + (wq >> 1) * HALF;
    // P1: all B fragments + A rows 0-63; DMA A(t+1) half 1; quadrant (rows 0-63, cols 0-31)
    if constexpr (kReads) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j) bq[kk][j] = frag<B_MN>(ib, cb + j * 16, kk, lane);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[kk][i] = frag<A_MN>(ia, i * 16, kk, lane);
    }
    if (kDma && kt + 1 < nk) stageA(kt + 1, 1);
    bar();
    quad(acc, a4, bq, 0, 0);
    bar();
    // P2: quadrant (rows 0-63, cols 32-63)
    bar();
    quad(acc, a4, bq, 0, 2);
    bar();
    // P3: A rows 64-127 (into the registers of rows 0-63); DMA B(t+2) half 0 (B of tile t was read in P1);
    // quadrant (rows 64-127, cols 32-63)
    if constexpr (kReads) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[kk][i] = frag<A_MN>(ia, 64 + i * 16, kk, lane);
    }
    if (kDma && kt + 2 < nk) stageB(kt + 2, 0);
    bar();
    quad(acc, a4, bq, 4, 2);
    bar();
    // P4: DMA B(t+2) half 1 + A(t+2) half 0 (A_g of tile t was read in P1 / P3); the wait that retires
    // tile t+1 (this wave's own DMA: the 6 issued after A(t+1) half 1 may stay in flight), group 1 in its
    // read segment, group 0 after its MFMAs - both before the barrier that precedes tile t+1's reads;
    // quadrant (rows 64-127, cols 0-31)
    if (kDma && kt + 2 < nk) {
      stageB(kt + 2, 1);
      stageA(kt + 2, 0);
    }
    if (ABL == 4 || g == 1) wait_next(kt);
    bar();
    quad(acc, a4, bq, 4, 0);
    if (ABL != 4 && g == 0) wait_next(kt);
    bar();
  }
  if (ABL != 4 && g == 0) bar();  // group 0 catches up: every wave's reads and MFMAs issued, the LDS is free
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue through a wave-private 16 KB LDS tile (row-major), 16-byte row-segment stores
  const int orow = m0 + g * 128, ocol = n0 + (wq >> 1) * 128 + cb;
  if (orow >= M || ocol >= N) return;
  char* tile = lds + wave * 16384;
  if constexpr (EPI == 2) {
    float* C = static_cast<float*>(Cv) + (size_t)blockIdx.y * M * N;
    float* tf = reinterpret_cast<float*>(tile);
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {  // 64 rows x 64 fp32 per pass
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) tf[(i * 16 + (lane >> 4) * 4 + e) * 64 + j * 16 + (lane & 15)] = acc[pass * 4 + i][j][e];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int row = it * 4 + (lane >> 4), ch = lane & 15;
        *reinterpret_cast<float4*>(C + (size_t)(orow + pass * 64 + row) * N + ocol + ch * 4) =
            *reinterpret_cast<const float4*>(tf + row * 64 + ch * 4);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  } else {
    uint16_t* C = static_cast<uint16_t*>(Cv);
    float bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = bias ? bf2f(bias[ocol + j * 16 + (lane & 15)]) : 0.f;
#pragma unroll
    for (int pass = 0; pass < (EPI == 1 ? 2 : 1); ++pass) {
      uint16_t* out = pass ? G : C;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = bf2f(f2bf(acc[i][j][e] + bv[j]));
            if (pass) v = gelu_tanh(v);
            *reinterpret_cast<uint16_t*>(tile + (i * 16 + (lane >> 4) * 4 + e) * 128 + (j * 16 + (lane & 15)) * 2) = f2bf(v);
          }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int row = it * 8 + (lane >> 3), ch = lane & 7;
        *reinterpret_cast<uint4*>(out + (size_t)(orow + row) * N + ocol + ch * 8) =
            *reinterpret_cast<const uint4*>(tile + row * 128 + ch * 16);
      }
      if (EPI == 1 && pass == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  }
}

}  // namespace

// measurement-only ablations of the NT bf16 kernel (benchmarks/bench_gemm256.py --ablate): wrong results
hipError_t launch_g256_ablate(const void* A, const void* B, void* C, int M, int N, int K, int variant, hipStream_t st) {
  if (!supported256(M, N, K, 1)) return hipErrorInvalidValue;
  const dim3 grid(((M + T - 1) / T) * ((N + T - 1) / T), 1);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
#define G256A(V) \
  hipLaunchKernelGGL((g256_kernel<false, false, 0, V>), grid, dim3(512), 0, st, a, K, b, K, nullptr, C, nullptr, M, N, K)
  switch (variant) {
    case 1: G256A(1); break;
    case 2: G256A(2); break;
    case 3: G256A(3); break;
    case 4: G256A(4); break;
    default: G256A(0); break;
  }
#undef G256A
  return hipGetLastError();
}

bool supported256(int M, int N, int K, int splitk) {
  return M > 0 && N > 0 && K > 0 && splitk >= 1 && M % 128 == 0 && N % 128 == 0 && K % (BK * splitk) == 0;
}

hipError_t launch_g256(const void* A, int lda, bool a_mn, const void* B, int ldb, bool b_mn, const void* bias, void* C,
                       void* G, bool out_f32, int splitk, int M, int N, int K, hipStream_t st) {
  if (!supported256(M, N, K, splitk) || (out_f32 && (bias || G)) || (!out_f32 && splitk != 1)) return hipErrorInvalidValue;
  const dim3 grid(((M + T - 1) / T) * ((N + T - 1) / T), splitk);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
  const uint16_t* bb = static_cast<const uint16_t*>(bias);
  uint16_t* g = static_cast<uint16_t*>(G);
  const int ks = K / splitk;
#define G256(AM, BMN, E) \
  hipLaunchKernelGGL((g256_kernel<AM, BMN, E>), grid, dim3(512), 0, st, a, lda, b, ldb, bb, C, g, M, N, ks)
#define G256_E(AM, BMN)           \
  if (out_f32) G256(AM, BMN, 2); \
  else if (g) G256(AM, BMN, 1);  \
  else G256(AM, BMN, 0);
  if (a_mn && b_mn) {
    G256_E(true, true)
  } else if (a_mn) {
    G256_E(true, false)
  } else if (b_mn) {
    G256_E(false, true)
  } else {
    G256_E(false, false)
  }
#undef G256_E
#undef G256
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace katib_hip
