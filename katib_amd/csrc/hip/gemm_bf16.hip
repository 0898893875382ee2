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
#include <cstdlib>

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
  const float z = 0.7978845608028654f * (u + 0.044715f * u * u * u);
  const float e = __expf(2.f * z);
  return 0.5f * u * (1.f + (1.f - 2.f / (e + 1.f)));
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

// STAGES LDS buffers; STAGES - 1 K-tiles in flight while one is consumed. STAGES == 2: one
// barrier per K-tile with the DMA drained before it (2 workgroups per CU). STAGES >= 3 (1 per CU):
// the DMA of the next STAGES - 2 tiles stays in flight across the raw s_barrier, each wave waiting
// only for its own loads of the tile about to be read with a counted vmcnt (8 DMA instructions
// per thread per tile), never __syncthreads() (its fence would wait vmcnt(0) and drain the pipe).
template <int EPI, int STAGES>
__global__ void __launch_bounds__(256) gemm_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                      const uint16_t* __restrict__ bias, uint16_t* __restrict__ C,
                                                      uint16_t* __restrict__ G, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char lds[STAGES * 2 * TILE_BYTES];  // [stage][A|W][128][64] bf16
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
    char* d = lds + (kt % STAGES) * 2 * TILE_BYTES;
    stage(A, K, m0, kt * BK, d, wave, lane);
    stage(W, K, n0, kt * BK, d + TILE_BYTES, wave, lane);
  };
  auto compute = [&](int kt) {
    const char* la = lds + (kt % STAGES) * 2 * TILE_BYTES;
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
  if constexpr (STAGES == 2) {
    stage_tile(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage_tile(kt + 1);  // the other buffer: its readers passed the last barrier
      compute(kt);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
      if (p < nk) stage_tile(p);
    for (int kt = 0; kt < nk; ++kt) {
      // this wave's loads of tile kt have landed: the younger tiles' 8 DMA each may stay in flight
      const int younger = min(nk - 1 - kt, STAGES - 2);
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // every wave's tile-kt loads landed, and every wave finished reading tile kt - 1's buffer,
      // which the next stage_tile refills
      __builtin_amdgcn_s_barrier();
      if (kt + STAGES - 1 < nk) stage_tile(kt + STAGES - 1);
      compute(kt);
    }
    __builtin_amdgcn_s_barrier();  // all reads done before the epilogue reuses the LDS
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

}  // namespace

bool supported(int M, int N, int K) { return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0; }

hipError_t launch_nt(const void* A, const void* W, const void* bias, void* C, void* G, int M, int N, int K,
                     hipStream_t st) {
  if (!supported(M, N, K)) return hipErrorInvalidValue;
  const dim3 grid((M / BM) * (N / BN));
  // 2 stages at 2 workgroups per CU measured fastest on MI355X (GPT-2 projections: 3 / 4 stages at one
  // workgroup per CU are 1.3-1.6x slower, profiles/gemm_bf16_r03.log)
  static const int stages = getenv("KATIB_HIP_GEMM_STAGES") ? atoi(getenv("KATIB_HIP_GEMM_STAGES")) : 2;
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* w = static_cast<const uint16_t*>(W);
  const uint16_t* bb = static_cast<const uint16_t*>(bias);
  uint16_t* c = static_cast<uint16_t*>(C);
  uint16_t* g = static_cast<uint16_t*>(G);
#define GEMM_LAUNCH(S)                                                                              \
  if (g) hipLaunchKernelGGL((gemm_nt_kernel<1, S>), grid, dim3(256), 0, st, a, w, bb, c, g, M, N, K); \
  else hipLaunchKernelGGL((gemm_nt_kernel<0, S>), grid, dim3(256), 0, st, a, w, bb, c, nullptr, M, N, K);
  if (stages == 2) {
    GEMM_LAUNCH(2)
  } else if (stages == 4) {
    GEMM_LAUNCH(4)
  } else {
    GEMM_LAUNCH(3)
  }
#undef GEMM_LAUNCH
  return hipGetLastError();
}

}  // namespace gemm
}  // namespace katib_hip
