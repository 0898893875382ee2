// Argument blocks for the DARTS edge kernels (darts_ops.hip). Passed by value.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

namespace katib_hip {

// Storage type of the per-op intermediates of a DARTS edge (depthwise outputs d, pre-BN op
// outputs z: ~90 % of a supernet step's activation bytes). fp32 by default; the bf16 build
// variant (-DKATIB_DARTS_ZBF16, _hipkern_zbf16.so) stores them as bf16 and keeps everything
// else fp32: node states, every gradient, BN statistics and reductions, weights, the math.
#ifdef KATIB_DARTS_ZBF16
typedef __hip_bfloat16 zt;
constexpr bool kZbf16 = true;
#else
typedef float zt;
constexpr bool kZbf16 = false;
#endif
typedef float zf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float z2f(float v) { return v; }
__device__ __forceinline__ float z2f(__hip_bfloat16 v) { return __bfloat162float(v); }
__device__ __forceinline__ void zput(float* p, float v) { *p = v; }
__device__ __forceinline__ void zput(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }
// 4 consecutive elements (16-byte fp32 / 8-byte bf16 access; callers keep 16-byte alignment)
__device__ __forceinline__ zf4 zld4(const float* p) { return *reinterpret_cast<const zf4*>(p); }
__device__ __forceinline__ zf4 zld4(const __hip_bfloat16* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return zf4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
             __uint_as_float(u.y & 0xffff0000u)};
}
__device__ __forceinline__ void zst4(float* p, zf4 v) { *reinterpret_cast<zf4*>(p) = v; }
__device__ __forceinline__ void zst4(__hip_bfloat16* p, zf4 v) {
  __hip_bfloat16 b[4] = {__float2bfloat16(v.x), __float2bfloat16(v.y), __float2bfloat16(v.z), __float2bfloat16(v.w)};
  *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(b);
}

// Offset of channel plane (n, c) of an [N][C][HW] tensor, or of a node-major one
// ([nodes][N][C / nodes][HW]: a DARTS cell output kept as its nodes' buffers instead of a concatenation)
__host__ __device__ __forceinline__ size_t plane_off(int n, int c, int N, int C, int nodes, size_t HW) {
  if (nodes <= 1) return ((size_t)n * C + c) * HW;
  const int Cn = C / nodes, k = c / Cn;
  return (((size_t)k * N + n) * Cn + (c - k * Cn)) * HW;
}

constexpr int kMaxOps = 8;
constexpr int kMaxUpd = 4;  // update-only BN layers per combine entry (the separable convs' first stages)
constexpr int kMaxC = 256;
// Cross-workgroup sums (BN statistics, BN-backward reductions, weight gradients) go to kRep
// replicas of the accumulator, workgroup b adding into replica b % kRep: global float atomics
// execute memory-side and same-address adds serialise, so bounding the adders per address
// (grid / kRep) keeps every flush short. Consumers sum the replicas (bn_moments / prologues);
// weight-gradient replicas are folded once per backward pass (fold_rows).
#ifndef KATIB_HIP_REP
#define KATIB_HIP_REP 32
#endif
constexpr int kRep = KATIB_HIP_REP;

struct BNRef {              // where a BN layer's normalisation statistics come from
  const double* sums;       // training: replica r at sums + r*rstride: [2*C] = (sum, sum of squares)
  float* rmean;             // running stats (read in eval, updated by combine in training)
  float* rvar;
  float inv_count;          // 1 / (N*H*W)
  float eps;
  int eval;
  int C;
  int rep;                  // replicas to sum (1 or kRep)
  int rstride;              // doubles between replicas
};

struct GradSrc {            // d(loss)/d(z) evaluated on the fly: BN backward of a weighted op
  const float* g;           // upstream gradient (dout of the edge, or a stored stage gradient)
  const zt* z;              // pre-BN tensor
  const double* S1;         // [C] sum g            (replica r at + r*rstride)
  const double* S2;         // [C] sum g * zhat
  BNRef bn;
  const float* w;           // softmax weights (nullptr -> 1)
  int widx;
  int eval;
  int rep;
  int rstride;
};

struct DwPwFwdArgs {
  const void* x;  // node state (fp32), or the previous stage's z (zt) when it carries an input BN
  BNRef inbn; const float* dw; const float* pw;
  zt* d; zt* z; double* stats;  // stats: kRep replicas of [2C]
  int N, C, H, W, Ho, Wo, pad, chunk, use_mfma;
  int variant;  // dwpw_plane_multi_kernel: ((K == 5) * 4 + (dil == 2) * 2 + (S == 2)) * 4 + prebn * 2 + vec
  int nblk;     // dwpw_plane_multi_kernel: workgroups of this entry (grid.x is the max over entries)
  int vout = 0; // dwpw_plane: 4 output pixels per thread, 16-byte stores (host: vec_mask())
};

struct PwFwdArgs {
  const void* x;  // relu: node state (fp32); identity: a wide dw-pw stage's depthwise output d (zt)
  const float* pw; zt* z; double* stats;  // stats: kRep replicas of [2*CoutTotal]
  int N, Cin, Cout, CoutTotal, co_off, H, W, Ho, Wo, S, off;
  int relu;  // 1: input = relu(x) (StdConv / FactorizedReduce); 0: identity (pointwise half of a dw-pw stage)
  int xnodes;  // relu: x node-major [xnodes][N][Cin / xnodes][H][W] when > 1 (a cell output kept as its nodes)
};

struct PoolFwdArgs {
  const float* x; zt* zavg; zt* zmax; double* stats_avg; double* stats_max; unsigned char* amax;
  int N, C, H, W, Ho, Wo;  // stats: kRep replicas of [2C] each
  int S, nblk;             // pool_fwd_multi_kernel: per-entry stride and workgroups
};

struct CombineFwdArgs {
  const zt* z[kMaxOps]; BNRef bn[kMaxOps]; int widx[kMaxOps]; int nops;
  BNRef upd[kMaxUpd]; int nupd;  // extra BN layers whose running stats are updated here (not summed)
  const float* w; int id_idx; const float* xid; const float* gamma; const float* beta;
  float* out; int N, C, HW; float momentum; int update_running; int accumulate;
};

struct CombineBwdArgs {
  const float* dout; const zt* z[kMaxOps]; BNRef bn[kMaxOps]; int nops;
  const float* xid; double* red; int N, C, HW;  // red: kRep replicas of [(nops+1)*C + 1]
  double* gw; int widx[kMaxOps]; int id_idx;  // optional: d(loss)/d(softmax weight), kRep replicas of [nw]
  int rstride, gwstride;
};

struct PwBwdArgs {
  GradSrc gs; const float* pw; const zt* ain; const float* x; float* dd; float* gx; float* gW;
  int gstride;  // floats between gW replicas (0: single accumulator)
  int N, Cin, Cout, CoutTotal, co_off, H, W, Ho, Wo, S, off, mode, need_dx;
  int overwrite;  // mode 1, stride 1: gx = masked grad instead of += (the kernel covers every pixel)
  int xnodes;     // mode 1: x and gx node-major [xnodes][N][Cin / xnodes][H][W] (> 1)
};

struct DwBwdArgs {
  const void* x;  // node state (fp32), or the stage-1 z (zt) when it carries an input BN
  BNRef inbn; const float* dw; const float* dd; float* gout; float* gW; double* red;
  int gstride;  // floats between gW replicas (0: single accumulator); red: kRep replicas of [2C]
  int N, C, H, W, Ho, Wo, pad, chunk;
  int overwrite;  // non-PREBN: gout = masked grad (first writer of this input gradient) instead of +=
  int variant, nbands, nblk;  // dw_bwd_plane_multi_kernel: dw_bwd_variant, row bands, workgroups of this entry
  int vin = 0;  // dw_bwd_plane, stride 1: 4 input pixels per thread, 16-byte stores (host: vec_mask())
};
constexpr int dw_bwd_variant(int K, int dil, int S, bool prebn) {
  return (((K == 5) * 4 + (dil == 2) * 2 + (S == 2)) << 1) | (prebn ? 1 : 0);
}
constexpr int dw_variant_k(int v) { return (v >> 3) & 1 ? 5 : 3; }
constexpr int dw_variant_dil(int v) { return (v >> 2) & 1 ? 2 : 1; }
constexpr int dw_variant_s(int v) { return (v >> 1) & 1 ? 2 : 1; }
constexpr bool dw_variant_prebn(int v) { return v & 1; }

struct FoldArgs {  // buf[0][i] = sum_r buf[r][i]; rows 1.. zeroed
  float* buf; int n; int rows;
};

constexpr int kMaxSeg = 128;  // two stacked passes' folds in one launch
struct FoldF64Args {  // per segment: p[i] = sum_{r < kRep} p[r*rstride + i]; replicas 1.. zeroed
  double* p[kMaxSeg]; int n[kMaxSeg]; int rstride[kMaxSeg]; int nseg; int total;
};

struct PoolBwdArgs {
  GradSrc ga; GradSrc gm; const float* x; const float* dout_id; const float* w; int id_idx; float* gx;
  const unsigned char* amax;
  const float* extra[4]; int nextra;  // other input-gradient parts of this edge summed in (conv backward)
  int overwrite;  // gx = result instead of +=
  int N, C, H, W, Ho, Wo;
  int S;          // pool_bwd_multi_kernel: per-entry stride
};

// Self-folding launches: a producer of replicated f64 reductions (BN statistics, BN-backward
// sums, d alpha) folds them itself instead of leaving it to a fold_f64 launch. Every workgroup,
// once its replica atomics have completed (s_waitcnt vmcnt(0): device-scope atomics are
// performed memory-side, so no L2 write-back fence is involved), adds 1 to an arrival counter;
// the workgroup that arrives last sums replicas 1.. into replica 0 with returning exchanges
// (replica r <- 0) and one atomic add, then re-arms the counter. Consumers in later launches read
// replica 0 only. Folding a segment twice is harmless (the second pass adds zeros).
constexpr int kTailSeg = 16;
constexpr int kFoldShards = 32;     // arrival counter shards per launch
constexpr int kFoldCtrStride = 32;  // uints between counters (one 128-byte line each)
constexpr int kFoldCtrSlot = (1 + kFoldShards) * kFoldCtrStride;  // uints per launch: top + shards
struct FoldTail {
  unsigned* ctr;   // kFoldCtrSlot uints: top counter, then the shard counters; zero between launches; nullptr: off
  int nseg;
  double* p[kTailSeg];
  int n[kTailSeg];
  int rs[kTailSeg];  // doubles between replicas
};

// Edge batches: one launch runs the same kernel for up to M edges of a DARTS node that share
// shapes (blockIdx.y = edge). Passed by value in the kernarg segment: ROCm 7.2 passes by-value
// arguments beyond 4 KB, eagerly and through captured graphs alike (scripts/kernarg_big_probe.hip:
// 28,000 B checked on MI355X, profiles/kernarg_big_probe_r06.log), so the capacities hold the
// entries of BOTH finite-difference Hessian passes (hip_darts.stacked_passes): the +eps and -eps
// passes go out as one launch per kernel type. combine_fwd stays at 4: its entries are the edges of
// ONE node summed into one output (register arrays sized by the capacity).
template <typename A, int M>
struct Batch {
  A e[M];
  int n;
  FoldTail tail;
  static constexpr int kCap = M;
};
using DwPwFwdBatch = Batch<DwPwFwdArgs, 16>;
using CombineFwdBatch = Batch<CombineFwdArgs, 4>;  // all edges of a node (B5: up to 4) in one launch
using PwFwdBatch = Batch<PwFwdArgs, 32>;
using PoolFwdBatch = Batch<PoolFwdArgs, 16>;
using CombineBwdBatch = Batch<CombineBwdArgs, 8>;
using PwBwdBatch = Batch<PwBwdArgs, 32>;  // a node's pointwise backward entries (2 sep stages + 2 dil per edge, <= 4 edges), x2 stacked
using DwBwdBatch = Batch<DwBwdArgs, 40>;  // a node's stage-1 depthwise backward entries (<= 5 edges x 4: darts-gpu.yaml), x2 stacked
using PoolBwdBatch = Batch<PoolBwdArgs, 16>;
using DwPwMultiBatch = Batch<DwPwFwdArgs, 40>;  // a node's stage-1 (or stage-2) dw-pw entries (<= 5 edges x 4, x2 stacked), mixed K/dil/S

// Whole input gradient of one DARTS edge (except the stride-2 skip's FactorizedReduce, which
// accumulates afterwards): the transposed depthwise convolutions of the separable stage-1 and the
// dilated convolutions (masked by relu'(x)), max / avg pool backward and the identity skip, formed
// in LDS and written once (edge_bwd_kernel).
struct EdgeBwdArgs {
  const float* x; float* gx; int overwrite;
  // conv slots: 0 sep 3x3, 1 sep 5x5 (dilation 1), 2 dil 3x3, 3 dil 5x5 (dilation 2)
  const float* dw[4]; const float* dd[4]; float* gW[4]; int gstride[4]; int conv_mask;
  GradSrc ga; GradSrc gm; const unsigned char* amax;  // ga.z / gm.z null: that pool is absent
  const float* dout_id; const float* w; int id_idx;   // identity skip (stride 1)
  int N, C, H, W, Ho, Wo, S, nb, nblk;
};
using EdgeBwdBatch = Batch<EdgeBwdArgs, 4>;
constexpr size_t kKernargMax = 24576;  // well inside the 28,000 B checked on MI355X
static_assert(sizeof(EdgeBwdBatch) <= kKernargMax, "edge_bwd batch exceeds the kernarg budget");
static_assert(sizeof(DwPwFwdBatch) <= kKernargMax && sizeof(CombineFwdBatch) <= kKernargMax &&
                  sizeof(PwFwdBatch) <= kKernargMax && sizeof(PoolFwdBatch) <= kKernargMax &&
                  sizeof(CombineBwdBatch) <= kKernargMax && sizeof(PwBwdBatch) <= kKernargMax &&
                  sizeof(DwBwdBatch) <= kKernargMax && sizeof(PoolBwdBatch) <= kKernargMax &&
                  sizeof(DwPwMultiBatch) <= kKernargMax,
              "kernel argument batches exceed the kernarg budget");

void launch_dwpw_fwd(const DwPwFwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st);
void launch_dw_bwd(const DwBwdBatch& b, int K, int dil, int S, bool prebn, hipStream_t st);
// mixed-variant depthwise backward (distinct outputs per entry, variant = dw_bwd_variant); false: not launched
bool launch_dw_bwd_multi(DwBwdBatch b, hipStream_t st);
void launch_pw_fwd(const PwFwdBatch& b, hipStream_t st);
void launch_pool_fwd(const PoolFwdBatch& b, int S, hipStream_t st);
void launch_pool_bwd(const PoolBwdBatch& b, int S, hipStream_t st);
// mixed-variant launches: one launch for entries with different kernel size / dilation / stride
bool launch_dwpw_multi(DwPwMultiBatch b, hipStream_t st);
void launch_pool_fwd_multi(PoolFwdBatch b, hipStream_t st);
// a node's pool entries beside its stage-1 dw-pw entries in one launch (no fold tail)
struct PoolFwdEntries {
  PoolFwdArgs e[PoolFwdBatch::kCap];
  int n;
};
static_assert(sizeof(DwPwMultiBatch) + sizeof(PoolFwdEntries) <= kKernargMax, "kernarg budget");
// false: nothing launched (not the fused narrow-layer plane path, or a self-fold tail is on)
bool launch_dwpw_pool_multi(DwPwMultiBatch b, const PoolFwdBatch& pb, hipStream_t st);
void launch_pool_bwd_multi(const PoolBwdBatch& b, hipStream_t st);
void launch_combine_fwd(const CombineFwdBatch& b, hipStream_t st);
// false (nothing launched): shapes / alignment outside the fused kernel's plane layout
bool launch_edge_bwd(EdgeBwdBatch b, hipStream_t st);
void launch_combine_bwd_reduce(const CombineBwdBatch& b, hipStream_t st);
void launch_pw_bwd(const PwBwdBatch& b, hipStream_t st);
int max_blocks();
void launch_fold_rows(const FoldArgs& a, hipStream_t st);
void launch_fold_f64(const FoldF64Args& a, hipStream_t st);
void set_max_blocks(int n);
// diagnostic build (-DKATIB_HIP_STAMPS): stamp every workgroup's phases of the `call`-th launch of
// `kind` (StampKind, darts_ops_dev.h) into buf[wg * 8 + phase]; kind 0 disarms
void stamps_arm(int kind, int call, unsigned long long* buf);
bool stamps_compiled();

}  // namespace katib_hip
