// bf16 GEMM on the gfx950 matrix cores for the GPT-2 projections (forward):
//   C[M][N] = A[M][K] . W[N][K]^T + bias[N]          (EPI 0: qkv, proj, fc2; LM head without bias)
//   U = A . W^T + bias, G = gelu_tanh(U)             (EPI 1: fc, GELU fused, U kept for gelu_bwd)
// A row-major (activations), W row-major [N][K] (nn.Linear weight): both operands are K-contiguous,
// so each MFMA fragment is one 16-byte LDS row read for A and W alike.
//
// 128 x 128 output tile per 256-thread workgroup (4 waves of 64 x 64, 4 x 4 v_mfma_f32_16x16x32_bf16
// accumulators each), K-step 64:
//   * staging: global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip), two LDS buffers: the next
//     K-tile streams in while the current one feeds the MFMAs, one barrier per K-tile;
//   * LDS image lane-linear (the DMA writes base + lane*16); bank conflicts of the fragment reads
//     (16 lanes = 16 rows of one 16-byte column) are broken by XOR-swizzling the 16-byte chunk with
//     the row on the GLOBAL source address and undoing it on the read (slot = chunk ^ (row & 7));
//   * XCD-aware tile order: workgroup b runs on XCD b % 8, so tiles are renumbered such that each
//     XCD owns a contiguous range of (row-block, column-block) tiles and re-reads its A panels from
//     its own L2 (bijective for any tile count);
//   * epilogue through LDS: bias (+ GELU) in fp32 on the accumulators, bf16 tile staged in LDS,
//     written back as 16-byte row segments.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gemm_bf16.h"

namespace katib_hip {
namespace gemm {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;  // one operand's K-tile (16 KB)

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

__device__ __forceinline__ float gelu_tanh(float u) {
  const float z2 = (2.f * 0.7978845608028654f * 1.4426950408889634f) * u * (1.f + 0.044715f * u * u);  // 2z log2(e)
  return 0.5f * u * (2.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z2) + 1.f));
}

// d gelu_tanh / du (the contract of transformer.hip gelu_df: tanh through exp)
// (hardware exp2 + reciprocal: in a GEMM epilogue the full-precision divide was most of the cost)
__device__ __forceinline__ float gelu_tanh_df(float u) {
  const float u2 = u * u;
  const float z2 = (2.f * 0.7978845608028654f * 1.4426950408889634f) * u * (1.f + 0.044715f * u2);  // 2z log2(e)
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z2) + 1.f);
  return 0.5f * (1.f + t) + (0.5f * 0.7978845608028654f) * u * (1.f - t * t) * (1.f + 3.f * 0.044715f * u2);
}

// one operand K-tile (128 rows x 64 bf16) -> LDS: 4 DMA instructions per thread
__device__ __forceinline__ void stage(const uint16_t* __restrict__ src, int ld, int row0, int k0, char* lds, int wave,
                                      int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = i * 4 + wave;           // 8-row block of this wave instruction
    const int row = blk * 8 + (lane >> 3);  // 8 lanes per 128-byte row
    const int slot = lane & 7;
    const int chunk = slot ^ (row & 7);     // swizzle on the source
    const uint16_t* g = src + (size_t)(row0 + row) * ld + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(g, (lds_ptr)(lds + blk * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag(const char* lds, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
}

// Two LDS buffers, one barrier per K-tile with the DMA drained before it (2 workgroups per CU): measured
// fastest of 2 / 3 / 4 stages on MI355X (profiles/gemm_bf16_r03.log: 3 / 4 stages at one workgroup per CU
// 1.3-1.6x slower).
template <int EPI>
__global__ void __launch_bounds__(256) gemm_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                      const uint16_t* __restrict__ bias, uint16_t* __restrict__ C,
                                                      uint16_t* __restrict__ G, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * TILE_BYTES];  // [stage][A|W][128][64] bf16
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
  // XCD-aware tile renumbering (bijective): XCD x = b % 8 gets the x-th contiguous range
  const int NB = N / BN, nwg = NB * (M / BM), b = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8, loc = b / 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int m0 = (t / NB) * BM, n0 = (t % NB) * BN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  auto stage_tile = [&](int kt) {
    char* d = lds + (kt & 1) * 2 * TILE_BYTES;
    stage(A, K, m0, kt * BK, d, wave, lane);
    stage(W, K, n0, kt * BK, d + TILE_BYTES, wave, lane);
  };
  auto compute = [&](int kt) {
    const char* la = lds + (kt & 1) * 2 * TILE_BYTES;
    const char* lw = la + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
      bf16x8 a[4], w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(la, wr * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = frag(lw, wc * 64 + j * 16 + (lane & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], w[j], acc[i][j], 0, 0, 0);
    }
  };
  stage_tile(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage_tile(kt + 1);  // the other buffer: its readers passed the last barrier
    compute(kt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: wave tile 64 x 64 -> LDS (bf16, row-major, 128 B rows) -> 16-byte global stores
  char* tile_u = lds + wave * 8192;           // pre-activation / output
  char* tile_g = lds + 32768 + wave * 8192;   // GELU output (EPI 1)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = j * 16 + (lane & 15);
    const float bv = bias ? bf2f(bias[n0 + wc * 64 + col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = i * 16 + (lane >> 4) * 4 + e;
        const uint16_t u = f2bf(acc[i][j][e] + bv);
        *reinterpret_cast<uint16_t*>(tile_u + row * 128 + col * 2) = u;
        if (EPI == 1) *reinterpret_cast<uint16_t*>(tile_g + row * 128 + col * 2) = f2bf(gelu_tanh(bf2f(u)));
      }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // wave-private tile: order LDS writes before reads
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int row = it * 8 + (lane >> 3), ch = lane & 7;
    const size_t go = (size_t)(m0 + wr * 64 + row) * N + n0 + wc * 64 + ch * 8;
    *reinterpret_cast<uint4*>(C + go) = *reinterpret_cast<const uint4*>(tile_u + row * 128 + ch * 16);
    if (EPI == 1) *reinterpret_cast<uint4*>(G + go) = *reinterpret_cast<const uint4*>(tile_g + row * 128 + ch * 16);
  }
}

// ------------------------------------------------------------------------------------------------
// Layout-native variants for the backward GEMMs (no transposed copies):
//   dgrad  dX[M][N] = dY[M][K] . W[K][N]      A K-contiguous, B MN-contiguous   ("NN")
//   wgrad  dW[M][N] = dY^T X: A = dY [K][M], B = X [K][N]   both MN-contiguous   ("TN")
// An MN-contiguous operand K-tile (64 k rows x 128 mn, 256-byte rows) is staged by the same
// lane-linear LDS-DMA as the K-contiguous one, and its MFMA fragments (8 consecutive k of one mn
// column per lane) are read with the hardware transpose ds_read_b64_tr_b16: per 16-lane group a
// 4-row x 16-column block arrives column-major, two reads per fragment. Bank conflicts: the eight
// rows a 32-lane half reads (q = 0..3 of k groups 8g and 8g + 8) each cover two 16-byte slots of a
// 256-byte row; the slot XOR 2 * ((r & 3) | ((r >> 3) & 1) << 2) gives them eight distinct even
// slot pairs (all 64 banks once), applied on the DMA source address and undone on the read.
// Split-K (gridDim.y slices, fp32 output slabs [slice][M][N]) gives the long-K wgrad shapes
// (K = tokens) enough workgroups; a row-sum kernel folds the slabs.
// ------------------------------------------------------------------------------------------------
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4* lds_s16x4;

__device__ __forceinline__ constexpr int mn_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

// one MN-contiguous operand K-tile (64 k rows x 128 mn bf16) -> LDS: 4 DMA instructions per thread
__device__ __forceinline__ void stage_mn(const uint16_t* __restrict__ src, int ld, int mn0, int k0, char* lds,
                                         int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = i * 4 + wave;           // 4-row (1 KB) block of this wave instruction
    const int row = blk * 4 + (lane >> 4);  // k row: 16 lanes per 256-byte row
    const int chunk = (lane & 15) ^ mn_swz(row);
    const uint16_t* g = src + (size_t)(k0 + row) * ld + mn0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(g, (lds_ptr)(lds + blk * 1024), 16, 0, 0);
  }
}

// MFMA operand fragment of mn columns [mn_base, mn_base + 16), k = kk * 32 + 8 (lane >> 4) + j
__device__ __forceinline__ bf16x8 frag_mn(const char* lds, int mn_base, int kk, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const int col = mn_base + 4 * (li & 3), chunk = col >> 3, half = (col >> 2) & 1;
  const int r0 = kk * 32 + 8 * g + (li >> 2), r1 = r0 + 4;
  const char* p0 = lds + r0 * 256 + ((chunk ^ mn_swz(r0)) << 4) + half * 8;
  const char* p1 = lds + r1 * 256 + ((chunk ^ mn_swz(r1)) << 4) + half * 8;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4)(p0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4)(p1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// C (+)= op(A) op(B) over k slice blockIdx.y; OUT_F32: fp32 slab [slice][M][N], else bf16 (+ bias)
// gu (bf16 output only): C = (op(A) op(B) (+ bias)) * gelu_tanh'(gu), the GELU backward folded into the
// dgrad epilogue (gu = the pre-activation, same [M][N] layout as C). cpart (bf16 output only): fp32
// column sums of the stored C per 64-row block, cpart[M / 64][N] (the bias gradient's first stage)
template <bool A_MN, bool B_MN, bool OUT_F32>
__global__ void __launch_bounds__(256) gemm_lt_kernel(const uint16_t* __restrict__ A, int lda,
                                                      const uint16_t* __restrict__ B, int ldb,
                                                      const uint16_t* __restrict__ bias, void* __restrict__ Cv,
                                                      int M, int N, int kslice, const uint16_t* __restrict__ gu,
                                                      float* __restrict__ cpart) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * TILE_BYTES];  // [stage][A|B][16 KB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
  const int NB = N / BN, nwg = NB * (M / BM), b = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8, loc = b / 8;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
  const int m0 = (t / NB) * BM, n0 = (t % NB) * BN;
  const int kbeg = blockIdx.y * kslice;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kslice / BK;
  auto stage_tile = [&](int kt) {
    char* d = lds + (kt & 1) * 2 * TILE_BYTES;
    const int k0 = kbeg + kt * BK;
    if constexpr (A_MN) stage_mn(A, lda, m0, k0, d, wave, lane);
    else stage(A, lda, m0, k0, d, wave, lane);
    if constexpr (B_MN) stage_mn(B, ldb, n0, k0, d + TILE_BYTES, wave, lane);
    else stage(B, ldb, n0, k0, d + TILE_BYTES, wave, lane);
  };
  auto compute = [&](int kt) {
    const char* la = lds + (kt & 1) * 2 * TILE_BYTES;
    const char* lb = la + TILE_BYTES;
    // both k sub-steps' fragments issued up front: the second half's LDS reads are in flight
    // while the first half's MFMAs run (the wait before them is counted, not a drain)
    bf16x8 a[2][4], w[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[kk][i] = A_MN ? frag_mn(la, wr * 64 + i * 16, kk, lane) : frag(la, wr * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[kk][j] = B_MN ? frag_mn(lb, wc * 64 + j * 16, kk, lane) : frag(lb, wc * 64 + j * 16 + (lane & 15), chunk);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk][i], w[kk][j], acc[i][j], 0, 0, 0);
  };
  stage_tile(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage_tile(kt + 1);  // the other buffer: its readers passed the last barrier
    compute(kt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if constexpr (OUT_F32) {
    // fp32 slab rows of this slice: each wave stages its 64 x 64 tile in LDS (256-byte rows) and
    // writes 16-byte row segments
    float* C = static_cast<float*>(Cv) + (size_t)blockIdx.y * M * N;
    float* tile = reinterpret_cast<float*>(lds + wave * 16384);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[(i * 16 + (lane >> 4) * 4 + e) * 64 + j * 16 + (lane & 15)] = acc[i][j][e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int row = it * 4 + (lane >> 4), ch = lane & 15;
      *reinterpret_cast<float4*>(C + (size_t)(m0 + wr * 64 + row) * N + n0 + wc * 64 + ch * 4) =
          *reinterpret_cast<const float4*>(tile + row * 64 + ch * 4);
    }
  } else {
    uint16_t* C = static_cast<uint16_t*>(Cv);
    char* tile_u = lds + wave * 8192;
    // GELU-backward epilogue: the pre-activation segments this lane stores, loaded before the
    // accumulator shuffle so their latency hides behind it
    uint4 uu[8];
    if (gu) {
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int row = it * 8 + (lane >> 3), ch = lane & 7;
        uu[it] = *reinterpret_cast<const uint4*>(gu + (size_t)(m0 + wr * 64 + row) * N + n0 + wc * 64 + ch * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j * 16 + (lane & 15);
      const float bv = bias ? bf2f(bias[n0 + wc * 64 + col]) : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          *reinterpret_cast<uint16_t*>(tile_u + (i * 16 + (lane >> 4) * 4 + e) * 128 + col * 2) = f2bf(acc[i][j][e] + bv);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = it * 8 + (lane >> 3), ch = lane & 7;
      uint4 v = *reinterpret_cast<const uint4*>(tile_u + row * 128 + ch * 16);
      if (gu) {
        uint32_t* pv = reinterpret_cast<uint32_t*>(&v);
        const uint32_t* pu = reinterpret_cast<const uint32_t*>(&uu[it]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = bf2f((uint16_t)(pv[k] & 0xffff)) * gelu_tanh_df(bf2f((uint16_t)(pu[k] & 0xffff)));
          const float hi = bf2f((uint16_t)(pv[k] >> 16)) * gelu_tanh_df(bf2f((uint16_t)(pu[k] >> 16)));
          pv[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
        }
      }
      if (cpart) {
        const uint32_t* pv = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          cs[2 * k] += bf2f((uint16_t)(pv[k] & 0xffff));
          cs[2 * k + 1] += bf2f((uint16_t)(pv[k] >> 16));
        }
      }
      *reinterpret_cast<uint4*>(C + (size_t)(m0 + wr * 64 + row) * N + n0 + wc * 64 + ch * 8) = v;
    }
    if (cpart) {
      // the 8 lanes sharing a column chunk (lane & 7) hold the wave's 64 rows: fold them, lanes 0-7 store
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = cs[e];
        x += __shfl_xor(x, 8, 64);
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        cs[e] = x;
      }
      if (lane < 8) {
        float* dst = cpart + (size_t)((m0 + wr * 64) >> 6) * N + n0 + wc * 64 + lane * 8;
        *reinterpret_cast<float4*>(dst) = float4{cs[0], cs[1], cs[2], cs[3]};
        *reinterpret_cast<float4*>(dst + 4) = float4{cs[4], cs[5], cs[6], cs[7]};
      }
    }
  }
}

}  // namespace

hipError_t launch_lt(const void* A, int lda, bool a_mn, const void* B, int ldb, bool b_mn, const void* bias, void* C,
                     bool out_f32, int splitk, int M, int N, int K, hipStream_t st, const void* gelu_u,
                     float* colpart) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || splitk < 1 || K % (splitk * BK) ||
      (!out_f32 && splitk != 1) || ((gelu_u || colpart) && out_f32))
    return hipErrorInvalidValue;
  const uint16_t* gu = static_cast<const uint16_t*>(gelu_u);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
  const uint16_t* bb = static_cast<const uint16_t*>(bias);
  const int ks = K / splitk;
  const dim3 grid((M / BM) * (N / BN), splitk);
#define LT_LAUNCH(AM, BMN, F32) \
  hipLaunchKernelGGL((gemm_lt_kernel<AM, BMN, F32>), grid, dim3(256), 0, st, a, lda, b, ldb, bb, C, M, N, ks, gu, \
                     colpart)
  if (out_f32) {
    if (a_mn && b_mn) LT_LAUNCH(true, true, true);
    else if (a_mn) LT_LAUNCH(true, false, true);
    else if (b_mn) LT_LAUNCH(false, true, true);
    else LT_LAUNCH(false, false, true);
  } else {
    if (a_mn && b_mn) LT_LAUNCH(true, true, false);
    else if (a_mn) LT_LAUNCH(true, false, false);
    else if (b_mn) LT_LAUNCH(false, true, false);
    else LT_LAUNCH(false, false, false);
  }
#undef LT_LAUNCH
  return hipGetLastError();
}

bool supported(int M, int N, int K) { return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0; }

hipError_t launch_nt(const void* A, const void* W, const void* bias, void* C, void* G, int M, int N, int K,
                     hipStream_t st) {
  if (!supported(M, N, K)) return hipErrorInvalidValue;
  const dim3 grid((M / BM) * (N / BN));
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* w = static_cast<const uint16_t*>(W);
  const uint16_t* bb = static_cast<const uint16_t*>(bias);
  uint16_t* c = static_cast<uint16_t*>(C);
  uint16_t* g = static_cast<uint16_t*>(G);
  if (g) hipLaunchKernelGGL((gemm_nt_kernel<1>), grid, dim3(256), 0, st, a, w, bb, c, g, M, N, K);
  else hipLaunchKernelGGL((gemm_nt_kernel<0>), grid, dim3(256), 0, st, a, w, bb, c, nullptr, M, N, K);
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace katib_hip
